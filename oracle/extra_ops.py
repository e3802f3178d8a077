"""numpy restatements of the operators an ONNX export feeds RTen's optimizer
(the LayerNorm / GELU primitives and the shape subgraph): ReduceMean, Pow,
Sqrt, Shape, ConstantOfShape, Concat, Slice, Expand and int32 Add / Sub /
Mul / Div.

TEST INFRASTRUCTURE ONLY (parity checker).  Float arithmetic is done on
float32 arrays element by element in the reference's order (numpy's float32
add / mul / div / sqrt are IEEE single operations, as Rust's are).
"""
from __future__ import annotations

import numpy as np

from rten_oracle import OpError

F32 = np.float32


def _contig(a, dtype=None):
    """C-contiguous copy that keeps 0-d arrays 0-d (np.ascontiguousarray does not)."""
    return np.array(a, dtype=dtype, order="C", copy=True)


def _resolve_axis(ndim, axis):
    """resolve_axis (src/ops/mod.rs:1087-1089)."""
    if axis < -ndim or axis >= ndim:
        raise OpError(5, "Axis is invalid")
    return axis + ndim if axis < 0 else axis


def slice_sum_rows(rows):
    """slice_sum (src/slice_reductions.rs:38-55) of every row of a 2-D f32 array."""
    rows = np.asarray(rows, F32)
    n = rows.shape[1]
    total = np.zeros(rows.shape[0], F32)
    for c0 in range(0, n, 8):
        ch = rows[:, c0:c0 + 8]
        if ch.shape[1] == 8:
            z0, z1, z2, z3 = (ch[:, 0] + ch[:, 4], ch[:, 1] + ch[:, 5], ch[:, 2] + ch[:, 6],
                              ch[:, 3] + ch[:, 7])
            s = ((z0 + z1) + z2) + z3
        else:
            s = np.zeros(rows.shape[0], F32)
            for j in range(ch.shape[1]):
                s = s + ch[:, j]
        total = total + s
    return total


def iter_sum_rows(rows):
    """iter_sum (src/slice_reductions.rs:58-85) of every row of a 2-D f32 array."""
    rows = np.asarray(rows, F32)
    n = rows.shape[1]
    total = np.zeros(rows.shape[0], F32)
    i, left = 0, n
    while left > 4:
        left -= 4
        a, b, c, d = rows[:, i], rows[:, i + 1], rows[:, i + 2], rows[:, i + 3]
        total = total + ((a + b) + (c + d))
        i += 4
    for j in range(i, n):
        total = total + rows[:, j]
    return total


def reduce_mean(x, axes=None, keep_dims=False):
    """reduce_mean -> reduce (src/ops/reduce.rs:225-353) on a contiguous f32 input."""
    x = _contig(x, F32)
    nd = x.ndim
    if axes is None or len(axes) == 0:
        resolved = list(range(nd))
    else:
        resolved = sorted(_resolve_axis(nd, int(a)) for a in axes)
    if nd == 0:
        return F32(iter_sum_rows(x.reshape(1, 1))[0] / F32(1))
    if x.size == 0:
        raise OpError(5, "Cannot reduce empty tensor")
    # reduced_inner_dims: the SORTED axes compared with ndim-1, ndim-2, ...
    # (reduce.rs:250-256) -- in practice only a single last axis qualifies.
    inner = all(ax == nd - 1 - i for i, ax in enumerate(resolved))
    red_shape = [1 if d in resolved else s for d, s in enumerate(x.shape)]
    if inner:
        # contiguous chunks of the trailing reduced dims: reduce_slice = slice_sum / len
        L = x.size if len(resolved) == nd else int(np.prod(x.shape[nd - len(resolved):]))
        rows = x.reshape(-1, L)
        out = slice_sum_rows(rows) / F32(L)
    elif len(resolved) == 1:
        ax = resolved[0]
        lanes = np.moveaxis(x, ax, -1).reshape(-1, x.shape[ax])
        # lanes(axis) iterate the other dims in row-major order, as moveaxis does
        out = iter_sum_rows(lanes) / F32(x.shape[ax])
        out = out.reshape([s for d, s in enumerate(x.shape) if d != ax])
        out = np.expand_dims(out, ax)
    else:
        keep = [d for d in range(nd) if d not in resolved]
        t = np.transpose(x, keep + resolved)
        L = int(np.prod([x.shape[d] for d in resolved]))
        out = iter_sum_rows(t.reshape(-1, L)) / F32(L)
    out = np.asarray(out, F32).reshape(red_shape)
    if not keep_dims:
        out = out.reshape([s for d, s in enumerate(x.shape) if d not in resolved])
    return _contig(out, F32)


def _powf(x, y):
    """powf with the fast paths of src/ops/binary_elementwise.rs:742-751."""
    x = np.asarray(x, F32)
    y = np.asarray(y, F32)
    with np.errstate(all="ignore"):
        general = np.power(x, y).astype(F32)
        sq = x * x
        cube = (x * x) * x
    return np.where(y == F32(2), sq, np.where(y == F32(3), cube, general)).astype(F32)


def pow_(a, b):
    """Pow (src/ops/binary_elementwise.rs:754-760)."""
    a = np.asarray(a, F32)
    b = np.asarray(b, F32)
    if b.size == 1:
        return _contig(_powf(a, b.reshape(())), F32)
    try:
        shape = np.broadcast_shapes(a.shape, b.shape)
    except ValueError:
        raise OpError(3, "Cannot broadcast inputs")
    return _contig(_powf(np.broadcast_to(a, shape), np.broadcast_to(b, shape)), F32)


def sqrt(x):
    """Sqrt (src/ops/unary_elementwise.rs:653): correctly rounded."""
    with np.errstate(all="ignore"):
        return _contig(np.sqrt(np.asarray(x, F32)), F32)


def shape(x):
    """Shape (src/ops/layout.rs:347-363): int32 [ndim]."""
    return np.array(np.asarray(x).shape, np.int32).reshape(np.asarray(x).ndim)


def constant_of_shape(shape_t, value):
    """ConstantOfShape (src/ops/generate.rs:28-42); value an int or a float."""
    s = np.asarray(shape_t)
    if s.dtype != np.int32:
        raise OpError(1, "Input 0 has incorrect type")
    if s.ndim != 1:
        raise OpError(5, "Input 0 has wrong number of dims")
    dt = np.int32 if isinstance(value, (int, np.integer)) else F32
    return np.full([int(v) for v in s], value, dt)


def concat(inputs, axis):
    """Concat (src/ops/concat.rs:15-121)."""
    first = np.asarray(inputs[0])
    ax = _resolve_axis(first.ndim, int(axis))
    for o in inputs[1:]:
        o = np.asarray(o)
        if o.dtype != first.dtype:
            raise OpError(1, "Input 1 has incorrect type")
        if o.ndim != first.ndim:
            raise OpError(3, "Tensors must have the same number of dimensions")
        for d in range(first.ndim):
            if d != ax and o.shape[d] != first.shape[d]:
                raise OpError(3, "Dimensions must be the same except for concat axis")
    return _contig(np.concatenate([np.asarray(i) for i in inputs], axis=ax))


def _clamp(v, lo, hi):
    return max(lo, min(hi, v))


def slice_(x, starts, ends, axes=None, steps=None):
    """Slice (src/ops/slice.rs:18-65) with SliceRange clamping / resolution
    (rten-tensor/src/slice_range.rs:242-331)."""
    x = np.asarray(x)
    starts = [int(v) for v in np.asarray(starts).reshape(-1)]
    ends = [int(v) for v in np.asarray(ends).reshape(-1)]
    stp = [int(v) for v in np.asarray(steps).reshape(-1)] if steps is not None else None
    if stp is not None and any(s == 0 for s in stp):
        raise OpError(5, "steps must be non-zero")
    ranges = [(0, d, 1) for d in x.shape]
    for i, (s, e) in enumerate(zip(starts, ends)):
        ax = _resolve_axis(x.ndim, int(np.asarray(axes).reshape(-1)[i])) if axes is not None else i
        st = stp[i] if stp is not None else 1
        ranges[ax] = (s, e, st)
    index = []
    for (s, e, st), n in zip(ranges, x.shape):
        lo, hi = (-n, n) if st > 0 else (-n - 1, n - 1)
        s, e = _clamp(s, lo, hi), _clamp(e, lo, hi)
        if st > 0:
            rs = s if s >= 0 else n + s
            re = e if e >= 0 else n + e
            re = max(re, rs)
            index.append(np.arange(rs, re, st))
        else:
            # resolve() counts backwards from the last index
            rs = n - 1 - s if s >= 0 else -s - 1
            re = n - 1 - e if e >= 0 else -e - 1
            re = max(re, rs)
            # index_range: start n-1-rs, end n-1-re (exclusive), step st
            index.append(np.arange(n - 1 - rs, n - 1 - re, st))
    out = x[np.ix_(*index)] if x.ndim else x
    return _contig(out)


def expand(x, shape_t):
    """Expand (src/ops/layout.rs:17-101)."""
    x = np.asarray(x)
    target = [int(v) for v in np.asarray(shape_t).reshape(-1)]
    try:
        out_shape = np.broadcast_shapes(x.shape, tuple(target))
    except ValueError:
        raise OpError(3, "Cannot broadcast input with target shape")
    return _contig(np.broadcast_to(x, out_shape))


def int_binary(op, a, b):
    """Add / Sub / Mul / Div on int32 tensors (binary_elementwise.rs, wrapping
    i32 arithmetic; Div truncates toward zero)."""
    a = np.asarray(a, np.int32)
    b = np.asarray(b, np.int32)
    try:
        np.broadcast_shapes(a.shape, b.shape)
    except ValueError:
        raise OpError(3, "Cannot broadcast inputs")
    a64, b64 = a.astype(np.int64), b.astype(np.int64)
    if op == "Add":
        r = a64 + b64
    elif op == "Sub":
        r = a64 - b64
    elif op == "Mul":
        r = a64 * b64
    else:
        if (b64 == 0).any():
            raise OpError(5, "Division by zero")
        q = np.abs(a64) // np.abs(b64)
        r = np.where((a64 < 0) ^ (b64 < 0), -q, q)
    return _contig(((r + 2 ** 31) % 2 ** 32 - 2 ** 31).astype(np.int32))
