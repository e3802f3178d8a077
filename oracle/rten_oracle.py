"""ctypes binding for the CPU oracle (librten_oracle.so).

TEST INFRASTRUCTURE ONLY: a CPU restatement of RTen's f32 operator path
(see rten_oracle.h for the reference file:line of every function).  Only
tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may
import this module; the product path never does.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "librten_oracle.so")

_i64p = C.POINTER(C.c_int64)
_f32p = C.POINTER(C.c_float)

ORC_RELU, ORC_CLIP, ORC_GELU, ORC_ERF, ORC_SIGMOID, ORC_TANH, ORC_EXP, ORC_SILU = range(8)
UNARY = {"Relu": 0, "Clip": 1, "Gelu": 2, "Erf": 3, "Sigmoid": 4, "Tanh": 5, "Exp": 6, "Silu": 7}
BINARY = {"Add": 0, "Sub": 1, "Mul": 2, "Div": 3}


class OpError(RuntimeError):
    """Mirrors RTen's OpError: ``kind`` is the variant name, str() its message."""

    KINDS = {1: "IncorrectInputType", 2: "IncorrectOutputType", 3: "IncompatibleInputShapes",
             4: "MissingInputs", 5: "InvalidValue", 6: "UnsupportedValue"}

    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code
        self.kind = self.KINDS.get(code, "Unknown")


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise RuntimeError(f"oracle library missing: build with `make -C {_HERE}`")
        _lib = C.CDLL(_LIB_PATH)
        _lib.orc_last_error.restype = C.c_char_p
    return _lib


def _check(code):
    if code != 0:
        raise OpError(code, lib().orc_last_error().decode())


def _f(a):
    return a.ctypes.data_as(_f32p)


def _c(a):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a


def _shape(shape):
    arr = (C.c_int64 * max(1, len(shape)))(*shape)
    return arr


def num_threads() -> int:
    return lib().orc_num_threads()


def set_num_threads(n: int):
    lib().orc_set_num_threads(int(n))


def reset_num_threads() -> int:
    """Re-resolve the thread count from RTEN_NUM_THREADS like
    rten::threading::thread_pool (src/threading.rs:41-62)."""
    return lib().orc_reset_threads()


def cpu_counts():
    """(logical, physical) as num_cpus::get / get_physical (num_cpus 1.16)."""
    lg, ph = C.c_int(), C.c_int()
    lib().orc_cpu_counts(C.byref(lg), C.byref(ph))
    return lg.value, ph.value


def xorshift(seed: int, n: int, state=None) -> np.ndarray:
    """XorShiftRng::new(seed).next_f32() x n (rten-tensor/src/rng.rs)."""
    st = C.c_uint64(seed)
    out = np.empty(n, dtype=np.float32)
    lib().orc_xorshift_fill(C.byref(st), _f(out), C.c_int64(n))
    return out


def gemm(a, b, alpha=1.0, beta=0.0, out=None, bias=None):
    """GemmExecutor::gemm_bias over (possibly strided) 2-D numpy views."""
    a = np.asarray(a, dtype=np.float32)
    b = np.asarray(b, dtype=np.float32)
    m, k = a.shape
    k2, n = b.shape
    assert k == k2
    if out is None:
        out = np.zeros((m, n), dtype=np.float32)
    assert out.dtype == np.float32 and (out.size == 0 or out.strides[1] == 4)
    out_rs = out.strides[0] // 4 if out.size else max(n, 1)
    bias_p = None
    if bias is not None:
        bias = _c(bias)
        bias_p = _f(bias)
    _check(lib().orc_gemm(_f(out), C.c_int64(out_rs), _f(a),
                          C.c_int64(a.strides[0] // 4), C.c_int64(a.strides[1] // 4), _f(b),
                          C.c_int64(b.strides[0] // 4), C.c_int64(b.strides[1] // 4),
                          C.c_int64(m), C.c_int64(n), C.c_int64(k), C.c_float(alpha),
                          C.c_float(beta), bias_p))
    return out


def gemm_gflops_1t(m: int, n: int, k: int, seconds: float = 0.5) -> float:
    """Single-thread GFLOP/s of gemm() at one of the reference's bench_gemm
    shapes (src/gemm.rs:1782-1903 times m = n = k square products): best of
    the runs made within `seconds`.  The thread count is restored after."""
    return gemm_gflops(m, n, k, seconds, threads=1)


def cpu_topology() -> dict:
    """What the CPUs this process may run on are (sched_getaffinity, sysfs):
    logical CPUs, the distinct physical cores and packages under them, and
    whether SMT is on -- so a thread count can be read as cores or
    hyperthreads."""
    import os

    cpus = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    cores, pkgs = set(), set()
    for c in cpus:
        base = f"/sys/devices/system/cpu/cpu{c}/topology/"
        try:
            core = open(base + "core_id").read().strip()
            pkg = open(base + "physical_package_id").read().strip()
        except OSError:
            core, pkg = str(c), "0"
        cores.add((pkg, core))
        pkgs.add(pkg)
    smt = None
    try:
        smt = open("/sys/devices/system/cpu/smt/active").read().strip() == "1"
    except OSError:
        pass
    return {"affinity_cpus": len(cpus), "physical_cores_in_affinity": len(cores), "packages": len(pkgs),
            "smt_active": smt}


def gemm_gflops(m: int, n: int, k: int, seconds: float = 0.5, threads: int = 1) -> float:
    """GFLOP/s of gemm() on `threads` threads (the pool the reference's
    GEMM parallelises its column blocks over, src/gemm.rs:733-930); best of
    the runs made within `seconds`.  The thread count is restored after."""
    import time

    prev = num_threads()
    set_num_threads(int(threads))
    try:
        a = ((xorshift(11, m * k) - 0.5).reshape(m, k))
        b = ((xorshift(12, k * n) - 0.5).reshape(k, n))
        out = np.zeros((m, n), np.float32)
        gemm(a, b, out=out)
        best = float("inf")
        t_end = time.perf_counter() + seconds
        while True:
            t0 = time.perf_counter()
            gemm(a, b, out=out)
            best = min(best, time.perf_counter() - t0)
            if time.perf_counter() > t_end:
                break
        return 2.0 * m * n * k / best / 1e9
    finally:
        set_num_threads(prev)


def reference_gemm(a, b, alpha=1.0, beta=0.0, out=None, bias=None):
    a, b = _c(a), _c(b)
    m, k = a.shape
    n = b.shape[1]
    out = np.zeros((m, n), np.float32) if out is None else _c(out)
    bias_p = None
    if bias is not None:
        bias = _c(bias)
        bias_p = _f(bias)
    lib().orc_reference_gemm(_f(out), _f(a), _f(b), C.c_int64(m), C.c_int64(n), C.c_int64(k),
                             C.c_float(alpha), C.c_float(beta), bias_p)
    return out


def output_size_and_padding(in_hw, k_hw, strides, padding="fixed", pads=(0, 0, 0, 0),
                            dilations=(1, 1)):
    out_hw = (C.c_int64 * 2)()
    pads_out = (C.c_int64 * 4)()
    mode = 1 if padding == "same" else 0
    _check(lib().orc_output_size_and_padding(
        C.c_int64(in_hw[0]), C.c_int64(in_hw[1]), C.c_int64(k_hw[0]), C.c_int64(k_hw[1]),
        C.c_int64(strides[0]), C.c_int64(strides[1]), C.c_int(mode), _shape(list(pads)),
        C.c_int64(dilations[0]), C.c_int64(dilations[1]), out_hw, pads_out))
    return (out_hw[0], out_hw[1]), tuple(pads_out)


def conv(x, w, bias=None, pads=(0, 0, 0, 0), strides=(1, 1), dilations=(1, 1), groups=1,
         padding="fixed"):
    """Conv op (src/ops/conv.rs:86-280).  pads = [top, left, bottom, right]
    (2-D) or [left, right] (1-D)."""
    x, w = _c(x), _c(w)
    nd = x.ndim
    if nd == 4:
        (oh, ow), _ = output_size_and_padding(x.shape[2:], w.shape[2:], strides, padding, pads,
                                              dilations)
        out = np.empty((x.shape[0], w.shape[0], oh, ow), np.float32)
    elif nd == 3:
        p4 = (0, pads[0], 0, pads[1]) if len(pads) == 2 else tuple(pads)
        (oh, ow), _ = output_size_and_padding((1, x.shape[2]), (1, w.shape[2]),
                                              (1, strides[0]), padding, p4, (1, dilations[0]))
        out = np.empty((x.shape[0], w.shape[0], ow), np.float32)
    else:
        raise OpError(5, "Input must have 4 dims (NCHW)")
    out_shape = (C.c_int64 * 4)()
    b = _c(bias) if bias is not None else None
    _check(lib().orc_conv(_f(x), _shape(x.shape), C.c_int(nd), _f(w), _shape(w.shape),
                          _f(b) if b is not None else None, C.c_int(1 if padding == "same" else 0),
                          _shape(list(pads)), _shape(list(strides)), _shape(list(dilations)),
                          C.c_int64(groups), _f(out), out_shape))
    return out


def conv_transpose_output_size(in_hw, k_hw, strides, padding="fixed", pads=(0, 0, 0, 0)):
    """conv_transpose_output_size_and_padding (src/ops/conv.rs:382-440); the
    pads come back in the reference's order (Same: top, bottom, left, right)."""
    out_hw = (C.c_int64 * 2)()
    pads_out = (C.c_int64 * 4)()
    _check(lib().orc_conv_transpose_output_size(
        C.c_int64(in_hw[0]), C.c_int64(in_hw[1]), C.c_int64(k_hw[0]), C.c_int64(k_hw[1]),
        C.c_int(1 if padding == "same" else 0), _shape(list(pads)), C.c_int64(strides[0]),
        C.c_int64(strides[1]), out_hw, pads_out))
    return (out_hw[0], out_hw[1]), tuple(pads_out)


def conv_transpose(x, w, bias=None, pads=(0, 0, 0, 0), strides=(1, 1), padding="fixed"):
    """ConvTranspose (src/ops/conv.rs:443-535).  w is [C, O, kh, kw] (or
    [C, O, kw] for 1-D, pads [left, right], strides [s])."""
    x, w = _c(x), _c(w)
    nd = x.ndim
    if nd == 4:
        (oh, ow), _ = conv_transpose_output_size(x.shape[2:], w.shape[2:], strides, padding, pads)
        out = np.empty((x.shape[0], w.shape[1], oh, ow), np.float32)
    elif nd == 3:
        p4 = (0, pads[0], 0, pads[1]) if len(pads) == 2 else tuple(pads)
        (oh, ow), _ = conv_transpose_output_size((1, x.shape[2]), (1, w.shape[2]),
                                                 (1, strides[0]), padding, p4)
        out = np.empty((x.shape[0], w.shape[1], ow), np.float32)
    else:
        raise OpError(5, "Input must have 4 dims (NCHW)")
    out_shape = (C.c_int64 * 4)()
    b = _c(bias) if bias is not None else None
    _check(lib().orc_conv_transpose(_f(x), _shape(x.shape), C.c_int(nd), _f(w), _shape(w.shape),
                                    _f(b) if b is not None else None,
                                    C.c_int(1 if padding == "same" else 0), _shape(list(pads)),
                                    _shape(list(strides)), _f(out), out_shape))
    return out


def max_pool(x, kernel, strides=(1, 1), pads=(0, 0, 0, 0), padding="fixed"):
    x = _c(x)
    (oh, ow), _ = output_size_and_padding(x.shape[2:], kernel, strides, padding, pads)
    out = np.empty((x.shape[0], x.shape[1], oh, ow), np.float32)
    os_ = (C.c_int64 * 4)()
    _check(lib().orc_max_pool(_f(x), _shape(x.shape), _shape(list(kernel)),
                              _shape(list(strides)), C.c_int(1 if padding == "same" else 0),
                              _shape(list(pads)), _f(out), os_))
    return out


def average_pool(x, kernel, strides=(1, 1), pads=(0, 0, 0, 0), count_include_pad=False,
                 padding="fixed"):
    x = _c(x)
    (oh, ow), _ = output_size_and_padding(x.shape[2:], kernel, strides, padding, pads)
    out = np.empty((x.shape[0], x.shape[1], oh, ow), np.float32)
    os_ = (C.c_int64 * 4)()
    _check(lib().orc_average_pool(_f(x), _shape(x.shape), _shape(list(kernel)),
                                  _shape(list(strides)), C.c_int(1 if padding == "same" else 0),
                                  _shape(list(pads)), C.c_int(int(count_include_pad)), _f(out),
                                  os_))
    return out


def global_average_pool(x):
    x = _c(x)
    out = np.empty((x.shape[0], x.shape[1], 1, 1), np.float32)
    _check(lib().orc_global_average_pool(_f(x), _shape(x.shape), _f(out)))
    return out


def batch_norm(x, scale, bias, mean, var, epsilon=1e-5):
    x = _c(x)
    out = np.empty_like(x)
    _check(lib().orc_batch_norm(_f(x), _shape(x.shape), C.c_int(x.ndim), _f(_c(scale)),
                                _f(_c(bias)), _f(_c(mean)), _f(_c(var)), C.c_float(epsilon),
                                _f(out)))
    return out


def binary(op, a, b):
    a, b = _c(a), _c(b)
    nd = max(a.ndim, b.ndim)
    try:
        shape = np.broadcast_shapes(a.shape, b.shape)
    except ValueError:
        raise OpError(3, "Cannot broadcast inputs")
    out = np.empty(shape, np.float32)
    os_ = (C.c_int64 * max(1, nd))()
    ond = C.c_int()
    _check(lib().orc_binary(C.c_int(BINARY[op]), _f(a), _shape(a.shape), C.c_int(a.ndim), _f(b),
                            _shape(b.shape), C.c_int(b.ndim), _f(out), os_, C.byref(ond)))
    return out


def add(a, b):
    return binary("Add", a, b)


def unary(op, x, p0=0.0, p1=0.0):
    x = _c(x)
    out = np.empty_like(x)
    _check(lib().orc_unary(C.c_int(UNARY[op]), _f(x), C.c_int64(x.size), _f(out), C.c_float(p0),
                           C.c_float(p1)))
    return out


def relu(x):
    return unary("Relu", x)


def clip(x, lo=None, hi=None):
    f32 = np.finfo(np.float32)
    return unary("Clip", x, f32.min if lo is None else lo, f32.max if hi is None else hi)


def softmax(x, axis=-1):
    x = _c(x)
    out = np.empty_like(x)
    _check(lib().orc_softmax(_f(x), _shape(x.shape), C.c_int(x.ndim), C.c_int64(axis), _f(out)))
    return out


def log_softmax(x, axis=-1):
    x = _c(x)
    out = np.empty_like(x)
    _check(lib().orc_log_softmax(_f(x), _shape(x.shape), C.c_int(x.ndim), C.c_int64(axis), _f(out)))
    return out


def instance_norm(x, scale, bias, epsilon=1e-5):
    x, scale, bias = _c(x), _c(scale), _c(bias)
    out = np.empty_like(x)
    _check(lib().orc_instance_norm(_f(x), _shape(x.shape), C.c_int(x.ndim), _f(scale), C.c_int64(scale.size),
                                   _f(bias), C.c_int64(bias.size), C.c_float(epsilon), _f(out)))
    return out


def layer_norm(x, scale, bias=None, axis=-1, epsilon=1e-5):
    x = _c(x)
    out = np.empty_like(x)
    b = _c(bias) if bias is not None else None
    _check(lib().orc_layer_norm(_f(x), _shape(x.shape), C.c_int(x.ndim), _f(_c(scale)),
                                _f(b) if b is not None else None, C.c_int64(axis),
                                C.c_float(epsilon), _f(out)))
    return out


def gemm_op(a, b, c=None, alpha=1.0, beta=1.0, trans_a=False, trans_b=False):
    a, b = _c(a), _c(b)
    m = a.shape[1] if trans_a else a.shape[0]
    n = b.shape[0] if trans_b else b.shape[1]
    out = np.empty((m, n), np.float32)
    cp, cs, cn = None, None, 0
    if c is not None:
        c = _c(c)
        cp, cs, cn = _f(c), _shape(c.shape), c.ndim
    _check(lib().orc_gemm_op(_f(a), _shape(a.shape), _f(b), _shape(b.shape), cp, cs, C.c_int(cn),
                             C.c_float(alpha), C.c_float(beta), C.c_int(int(trans_a)),
                             C.c_int(int(trans_b)), _f(out)))
    return out


def matmul(a, b):
    a, b = _c(a), _c(b)
    prefix = np.broadcast_shapes(a.shape[:-2], b.shape[:-2])
    out = np.empty(tuple(prefix) + (a.shape[-2], b.shape[-1]), np.float32)
    os_ = (C.c_int64 * 16)()
    ond = C.c_int()
    _check(lib().orc_matmul(_f(a), _shape(a.shape), C.c_int(a.ndim), _f(b), _shape(b.shape),
                            C.c_int(b.ndim), _f(out), os_, C.byref(ond)))
    return out


# ---------------------------------------------------------------------------
# Index / select / convert: numpy restatements (exact data movement)
# ---------------------------------------------------------------------------

def gather(x, indices, axis):
    """gather (src/ops/gather.rs:21-76): numpy.take along the resolved axis;
    negative entries count from the end (SliceItem::Index)."""
    x = np.asarray(x)
    idx = np.asarray(indices, np.int64)
    if not -x.ndim <= axis < x.ndim:
        raise OpError(5, "Axis is invalid")
    axis = axis % x.ndim
    n = x.shape[axis]
    res = np.where(idx < 0, idx + n, idx)
    if ((res < 0) | (res >= n)).any():
        raise OpError(5, "Entry in `indices` is out of range")
    return np.take(x, res, axis=axis)


def where(cond, x, y):
    """where_op (src/ops/binary_elementwise.rs:850-929)."""
    cond, x, y = np.asarray(cond), np.asarray(x), np.asarray(y)
    try:
        shape = np.broadcast_shapes(cond.shape, np.broadcast_shapes(x.shape, y.shape))
    except ValueError:
        raise OpError(3, "Cannot broadcast inputs") from None
    return np.where(np.broadcast_to(cond, shape) != 0, np.broadcast_to(x, shape),
                    np.broadcast_to(y, shape)).astype(x.dtype)


def cast_f32_to_i32(x):
    """Cast to Int32 (src/ops/convert.rs:10): Rust `as i32` -- truncation toward
    zero, saturating at the i32 range, NaN -> 0."""
    x = np.asarray(x, np.float32).astype(np.float64)
    out = np.where(np.isnan(x), 0.0, np.clip(np.trunc(x), -2.0 ** 31, 2.0 ** 31 - 1))
    return out.astype(np.int32)


def cast_i32_to_f32(x):
    """Cast to Float (src/ops/convert.rs:14): `as f32`, round to nearest even."""
    return np.asarray(x, np.int32).astype(np.float32)
