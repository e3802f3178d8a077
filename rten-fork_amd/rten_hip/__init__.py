"""Host-side mirror of RTen's operator interface on the MI355X backend.

Every function here calls the C ABI of ``librten_hip.so`` (include/rten_hip.h)
with device tensors; the compute always runs in the hand-written HIP kernels.
There is deliberately no CPU fallback: if the library or a GPU is missing the
call raises.

Names, argument meaning and errors follow the reference operators
(src/ops/*.rs): e.g. ``conv(x, w, bias, padding, groups, strides, dilations)``
is ``rten::ops::conv`` and failures raise :class:`OpError` carrying the same
``OpError`` variant and message.

torch is used only as device-memory plumbing (allocation, streams); no torch
compute op is ever called on the product path.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from typing import Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(_HERE)
# RTENHIP_LIB: an alternative build (timing experiments); default the in-tree library.
LIB_PATH = os.environ.get("RTENHIP_LIB") or os.path.join(_PKG, "librten_hip.so")

MAX_DIMS = 8


class OpError(RuntimeError):
    """RTen's OpError (src/ops/mod.rs:666-686) raised from a status code."""

    KINDS = {1: "IncorrectInputType", 2: "IncorrectOutputType", 3: "IncompatibleInputShapes",
             4: "MissingInputs", 5: "InvalidValue", 6: "UnsupportedValue", 7: "HipError"}

    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code
        self.kind = self.KINDS.get(code, "Unknown")


class Tensor(C.Structure):
    _fields_ = [("data", C.c_void_p), ("ndim", C.c_int32),
                ("shape", C.c_int64 * MAX_DIMS), ("strides", C.c_int64 * MAX_DIMS)]


_lib = None
_lib_lock = threading.Lock()


def lib():
    """Load librten_hip.so (raises if it was not built)."""
    global _lib
    with _lib_lock:
        if _lib is None:
            # torch first: it brings its own HIP runtime, and librten_hip.so must
            # bind to that one.  Loading this library first would map the
            # system libamdhip64 and leave torch and the library on different
            # runtimes (hipSetDevice then fails in the library).
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(f"{LIB_PATH} missing: build it with `make -C {_PKG}` "
                                   "(or __graft_entry__.build())")
            L = C.CDLL(LIB_PATH)
            L.rtenhip_create.restype = C.c_void_p
            L.rtenhip_create.argtypes = [C.c_int]
            L.rtenhip_destroy.argtypes = [C.c_void_p]
            L.rtenhip_set_stream.argtypes = [C.c_void_p, C.c_void_p]
            L.rtenhip_get_stream.restype = C.c_void_p
            L.rtenhip_get_stream.argtypes = [C.c_void_p]
            L.rtenhip_last_error_message.restype = C.c_char_p
            L.rtenhip_build_info.restype = C.c_char_p
            L.rtenhip_synchronize.argtypes = [C.c_void_p]
            if hasattr(L, "rtenhip_graph_create"):
                L.rtenhip_graph_create.restype = C.c_void_p
                L.rtenhip_graph_create.argtypes = [C.c_void_p]
                L.rtenhip_graph_destroy.argtypes = [C.c_void_p]
                L.rtenhip_graph_timing_report.restype = C.c_char_p
                L.rtenhip_graph_timing_report.argtypes = [C.c_void_p]
                L.rtenhip_graph_synchronize.argtypes = [C.c_void_p]
                L.rtenhip_graph_set_deferred_checks.argtypes = [C.c_void_p, C.c_int]
            L.rtenhip_last_error_code.restype = C.c_int32
            L.rtenhip_model_load.restype = C.c_void_p
            L.rtenhip_model_load.argtypes = [C.c_void_p, C.POINTER(C.c_uint8), C.c_size_t]
            L.rtenhip_model_load_with_options.restype = C.c_void_p
            L.rtenhip_model_load_with_options.argtypes = [C.c_void_p, C.POINTER(C.c_uint8),
                                                          C.c_size_t, C.c_int]
            L.rtenhip_model_describe.restype = C.c_char_p
            L.rtenhip_model_describe.argtypes = [C.POINTER(C.c_uint8), C.c_size_t]
            L.rtenhip_model_input_ids.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.c_int32]
            L.rtenhip_model_output_ids.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.c_int32]
            L.rtenhip_graph_describe.restype = C.c_char_p
            L.rtenhip_graph_describe.argtypes = [C.c_void_p]
            L.rtenhip_num_threads.restype = C.c_int32
            L.rtenhip_num_threads.argtypes = [C.c_void_p]
            L.rtenhip_cpu_counts.argtypes = [C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
            _lib = L
    return _lib


EXPORTED_SYMBOLS = [
    "rtenhip_create", "rtenhip_destroy", "rtenhip_set_stream", "rtenhip_get_stream",
    "rtenhip_last_error_message", "rtenhip_synchronize", "rtenhip_malloc", "rtenhip_free",
    "rtenhip_memcpy_h2d", "rtenhip_memcpy_d2h", "rtenhip_build_info",
    "rtenhip_output_size_and_padding", "rtenhip_gemm_f32", "rtenhip_conv_output_shape",
    "rtenhip_conv_f32", "rtenhip_conv_transpose_output_shape", "rtenhip_conv_transpose_f32",
    "rtenhip_gemm_op_f32", "rtenhip_matmul_f32", "rtenhip_max_pool_f32",
    "rtenhip_average_pool_f32", "rtenhip_global_average_pool_f32", "rtenhip_batch_norm_f32",
    "rtenhip_layer_norm_f32", "rtenhip_softmax_f32", "rtenhip_unary_f32", "rtenhip_binary_f32",
    "rtenhip_graph_create", "rtenhip_graph_destroy", "rtenhip_graph_add_value",
    "rtenhip_graph_add_constant", "rtenhip_graph_add_op", "rtenhip_graph_optimize",
    "rtenhip_graph_run", "rtenhip_graph_value_shape", "rtenhip_graph_set_timing",
    "rtenhip_graph_timing_report", "rtenhip_model_load", "rtenhip_model_load_with_options",
    "rtenhip_model_describe", "rtenhip_last_error_code", "rtenhip_model_input_ids",
    "rtenhip_model_output_ids", "rtenhip_graph_node_id", "rtenhip_graph_set_io",
    "rtenhip_graph_plan", "rtenhip_gather_output_shape", "rtenhip_gather_f32",
    "rtenhip_where_output_shape", "rtenhip_where_f32", "rtenhip_cast_f32_to_i32",
    "rtenhip_cast_i32_to_f32", "rtenhip_graph_add_constant_i32", "rtenhip_graph_run_typed",
    "rtenhip_graph_plan_typed", "rtenhip_num_threads", "rtenhip_cpu_counts", "rtenhip_reduce_mean_f32",
    "rtenhip_graph_describe", "rtenhip_log_softmax_f32", "rtenhip_instance_norm_f32",
    "rtenhip_graph_synchronize", "rtenhip_graph_set_deferred_checks",
    "rtenhip_set_exec_stream", "rtenhip_host_alloc", "rtenhip_host_free", "rtenhip_graph_run_host", "rtenhip_graph_wait",
    "rtenhip_sharded_create", "rtenhip_sharded_destroy", "rtenhip_sharded_gather_mode",
    "rtenhip_sharded_graph", "rtenhip_sharded_run_host", "rtenhip_sharded_gathered",
]

# rtenhip_dtype (sg::DataType order, include/rten_hip.h)
DTYPE_INT32 = 0
DTYPE_FLOAT32 = 1


def check(code: int):
    if code != 0:
        raise OpError(code, lib().rtenhip_last_error_message().decode())


def _torch():
    import torch

    return torch


def describe(t) -> Tensor:
    """rtenhip_tensor view of a float32 device torch tensor (no copy)."""
    torch = _torch()
    if t.dtype != torch.float32:
        raise OpError(1, "IncorrectInputType: expected float32")
    if not t.is_cuda:
        raise OpError(1, "tensor must be on the GPU (HIP device)")
    if t.dim() > MAX_DIMS:
        raise OpError(6, "too many dims")
    d = Tensor()
    d.data = t.data_ptr() if t.numel() else None
    d.ndim = t.dim()
    for i, (s, st) in enumerate(zip(t.shape, t.stride())):
        d.shape[i] = s
        d.strides[i] = st
    return d


def _i64(vals):
    vals = list(vals)
    return (C.c_int64 * max(1, len(vals)))(*vals)


class Context:
    """rtenhip_ctx bound to torch's current stream on ``device``."""

    def __init__(self, device: int = 0):
        torch = _torch()
        if not torch.cuda.is_available():
            raise RuntimeError("rten_hip needs a HIP GPU; none is visible")
        self.device = device
        self.ptr = lib().rtenhip_create(device)
        if not self.ptr:
            raise RuntimeError(lib().rtenhip_last_error_message().decode())
        self.sync_stream()

    @property
    def num_threads(self) -> int:
        """RTen's thread-pool size this context reproduces (src/threading.rs:41-62)."""
        return int(lib().rtenhip_num_threads(C.c_void_p(self.ptr)))

    def sync_stream(self, stream=None):
        torch = _torch()
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        check(lib().rtenhip_set_stream(C.c_void_p(self.ptr), C.c_void_p(s.cuda_stream)))

    def use_stream(self, stream):
        """Run this context's graphs on ``stream`` (a torch.cuda.Stream) and
        make it the caller's stream too (rtenhip_set_exec_stream): graph runs
        issued under ``with torch.cuda.stream(stream)`` then need no
        cross-stream events between runs."""
        self.exec_stream = stream  # keep the torch stream alive as long as the context uses it
        check(lib().rtenhip_set_exec_stream(C.c_void_p(self.ptr), C.c_void_p(stream.cuda_stream)))
        self.sync_stream(stream)

    def close(self):
        if self.ptr:
            lib().rtenhip_destroy(C.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def cpu_counts():
    """(logical, physical) CPU counts as num_cpus 1.16 reports them (host only)."""
    lg, ph = C.c_int32(), C.c_int32()
    lib().rtenhip_cpu_counts(C.byref(lg), C.byref(ph))
    return lg.value, ph.value


_default_ctx: Optional[Context] = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    _default_ctx.sync_stream()
    return _default_ctx


def describe_i32(t) -> Tensor:
    """rtenhip_tensor_i32 view of an int32 device torch tensor (same layout as
    rtenhip_tensor; Input::IntTensor, src/ops/mod.rs:177-180)."""
    torch = _torch()
    if t.dtype != torch.int32:
        raise OpError(1, "IncorrectInputType: expected int32")
    if not t.is_cuda:
        raise OpError(1, "tensor must be on the GPU (HIP device)")
    if t.dim() > MAX_DIMS:
        raise OpError(6, "too many dims")
    d = Tensor()
    d.data = t.data_ptr() if t.numel() else None
    d.ndim = t.dim()
    for i, (s, st) in enumerate(zip(t.shape, t.stride())):
        d.shape[i] = s
        d.strides[i] = st
    return d


def gather(x, indices, axis=0, ctx=None):
    """Gather (src/ops/gather.rs:21-76): x float32, indices int32."""
    ctx = ctx or default_context()
    xd, idd = describe(x), describe_i32(indices)
    os_ = (C.c_int64 * MAX_DIMS)()
    ond = C.c_int32()
    check(lib().rtenhip_gather_output_shape(C.byref(xd), C.byref(idd), C.c_int64(axis), os_,
                                            C.byref(ond)))
    y = _empty(tuple(os_[i] for i in range(ond.value)), x)
    yd = describe(y)
    check(lib().rtenhip_gather_f32(C.c_void_p(ctx.ptr), C.byref(xd), C.byref(idd),
                                   C.c_int64(axis), C.byref(yd)))
    return y


def where(cond, x, y, ctx=None):
    """Where (src/ops/binary_elementwise.rs:850-929): cond int32, x/y float32."""
    ctx = ctx or default_context()
    cd, xd, yd = describe_i32(cond), describe(x), describe(y)
    os_ = (C.c_int64 * MAX_DIMS)()
    ond = C.c_int32()
    check(lib().rtenhip_where_output_shape(C.byref(cd), C.byref(xd), C.byref(yd), os_,
                                           C.byref(ond)))
    out = _empty(tuple(os_[i] for i in range(ond.value)), x)
    od = describe(out)
    check(lib().rtenhip_where_f32(C.c_void_p(ctx.ptr), C.byref(cd), C.byref(xd), C.byref(yd),
                                  C.byref(od)))
    return out


def cast(x, to, ctx=None):
    """Cast (src/ops/convert.rs:6-17): to = "int32" (from float32) or "float"
    (from int32)."""
    torch = _torch()
    ctx = ctx or default_context()
    if to == "int32":
        y = torch.empty(tuple(x.shape), dtype=torch.int32, device=x.device)
        xd, yd = describe(x), describe_i32(y)
        check(lib().rtenhip_cast_f32_to_i32(C.c_void_p(ctx.ptr), C.byref(xd), C.byref(yd)))
    elif to == "float":
        y = torch.empty(tuple(x.shape), dtype=torch.float32, device=x.device)
        xd, yd = describe_i32(x), describe(y)
        check(lib().rtenhip_cast_i32_to_f32(C.c_void_p(ctx.ptr), C.byref(xd), C.byref(yd)))
    else:
        raise OpError(6, f"unsupported cast target {to!r}")
    return y


def _empty(shape, like):
    torch = _torch()
    return torch.empty(tuple(shape), dtype=torch.float32, device=like.device)


# ---------------------------------------------------------------------------
# GEMM engine
# ---------------------------------------------------------------------------

def gemm(a, b, alpha: float = 1.0, beta: float = 0.0, out=None, bias=None, ctx=None):
    """GemmExecutor::gemm_bias (src/gemm.rs:465-542) on device matrices."""
    ctx = ctx or default_context()
    m, k = a.shape
    k2, n = b.shape
    if k != k2:
        raise OpError(3, "Columns of matrix `a` must match rows of matrix `b`")
    if out is None:
        out = _empty((m, n), a)
        if beta != 0:
            raise ValueError("beta != 0 needs `out`")
    check(lib().rtenhip_gemm_f32(
        C.c_void_p(ctx.ptr), C.c_int64(m), C.c_int64(n), C.c_int64(k),
        C.c_void_p(a.data_ptr()), C.c_int64(a.stride(0)), C.c_int64(a.stride(1)),
        C.c_void_p(b.data_ptr()), C.c_int64(b.stride(0)), C.c_int64(b.stride(1)),
        C.c_void_p(out.data_ptr()), C.c_int64(out.stride(0)), C.c_float(alpha), C.c_float(beta),
        C.c_void_p(bias.data_ptr() if bias is not None else None)))
    return out


# ---------------------------------------------------------------------------
# Operators (Operator::run bodies)
# ---------------------------------------------------------------------------

ACT = {None: 0, "relu": 1, "clip": 2}


def _padding(padding, ndim):
    """Padding::Same or Fixed pads -> (mode, pads)."""
    if padding is None:
        return 0, [0, 0, 0, 0] if ndim == 4 else [0, 0]
    if isinstance(padding, str):
        if padding.lower() == "same":
            return 1, [0, 0, 0, 0]
        raise OpError(5, f"Unknown padding {padding}")
    return 0, list(padding)


def conv_output_shape(x, w, padding=None, groups=1, strides=None, dilations=None):
    nd = x.dim()
    mode, pads = _padding(padding, nd)
    strides = list(strides or ([1, 1] if nd == 4 else [1]))
    dilations = list(dilations or ([1, 1] if nd == 4 else [1]))
    os_ = (C.c_int64 * 4)()
    ond = C.c_int32()
    xd, wd = describe(x), describe(w)
    check(lib().rtenhip_conv_output_shape(C.byref(xd), C.byref(wd), C.c_int(mode), _i64(pads),
                                          _i64(strides), _i64(dilations), C.c_int64(groups), os_,
                                          C.byref(ond)))
    return tuple(os_[i] for i in range(ond.value))


def conv(x, w, bias=None, padding=None, groups: int = 1, strides=None, dilations=None,
         residual=None, act: Optional[str] = None, act_range=(0.0, 6.0), out=None, ctx=None):
    """Conv (src/ops/conv.rs:86-311).  ``residual`` / ``act`` are the fused
    epilogue the graph optimizer uses for Conv->Add->Relu/Clip chains."""
    ctx = ctx or default_context()
    nd = x.dim()
    mode, pads = _padding(padding, nd)
    strides = list(strides or ([1, 1] if nd == 4 else [1]))
    dilations = list(dilations or ([1, 1] if nd == 4 else [1]))
    shape = conv_output_shape(x, w, padding, groups, strides, dilations)
    y = out if out is not None else _empty(shape, x)
    xd, wd, yd = describe(x), describe(w), describe(y)
    check(lib().rtenhip_conv_f32(
        C.c_void_p(ctx.ptr), C.byref(xd), C.byref(wd),
        C.c_void_p(bias.data_ptr() if bias is not None else None), C.c_int(mode), _i64(pads),
        _i64(strides), _i64(dilations), C.c_int64(groups),
        C.c_void_p(residual.data_ptr() if residual is not None else None), C.c_int(ACT[act]),
        C.c_float(act_range[0]), C.c_float(act_range[1]), C.byref(yd)))
    return y


def conv_transpose(x, w, bias=None, padding=None, strides=None, ctx=None):
    """ConvTranspose (src/ops/conv.rs:443-577): w is [C, O, kh, kw] ([C, O, kw]
    for NCW input); padding None / [top, left, bottom, right] ([left, right]) /
    "same"."""
    ctx = ctx or default_context()
    nd = x.dim()
    mode, pads = _padding(padding, nd)
    strides = list(strides or ([1, 1] if nd == 4 else [1]))
    xd, wd = describe(x), describe(w)
    os_ = (C.c_int64 * 4)()
    ond = C.c_int32()
    check(lib().rtenhip_conv_transpose_output_shape(C.byref(xd), C.byref(wd), C.c_int(mode),
                                                    _i64(pads), _i64(strides), os_, C.byref(ond)))
    y = _empty(tuple(os_[i] for i in range(ond.value)), x)
    yd = describe(y)
    check(lib().rtenhip_conv_transpose_f32(
        C.c_void_p(ctx.ptr), C.byref(xd), C.byref(wd),
        C.c_void_p(bias.data_ptr() if bias is not None else None), C.c_int(mode), _i64(pads),
        _i64(strides), C.byref(yd)))
    return y


def gemm_op(a, b, c=None, alpha=1.0, beta=1.0, transpose_a=False, transpose_b=False, ctx=None):
    """ONNX Gemm (src/ops/matmul.rs:27-81)."""
    ctx = ctx or default_context()
    if a.dim() != 2 or b.dim() != 2:
        raise OpError(5, "Expected 2-D inputs")
    m = a.shape[1] if transpose_a else a.shape[0]
    n = b.shape[0] if transpose_b else b.shape[1]
    y = _empty((m, n), a)
    ad, bd, yd = describe(a), describe(b), describe(y)
    cd = C.byref(describe(c)) if c is not None else None
    check(lib().rtenhip_gemm_op_f32(C.c_void_p(ctx.ptr), C.byref(ad), C.byref(bd), cd,
                                    C.c_float(alpha), C.c_float(beta), C.c_int(int(transpose_a)),
                                    C.c_int(int(transpose_b)), C.byref(yd)))
    return y


def matmul(a, b, ctx=None):
    """MatMul (src/ops/matmul.rs:123-254).  Strided inputs (e.g. a
    FusedTranspose view) are read in place."""
    ctx = ctx or default_context()
    torch = _torch()
    if a.dim() < 2 or b.dim() < 2:
        raise OpError(5, "Inputs must have >= 2 dimensions")
    try:
        prefix = torch.broadcast_shapes(a.shape[:-2], b.shape[:-2])
    except RuntimeError:
        raise OpError(3, "Cannot broadcast shapes")
    y = _empty(tuple(prefix) + (a.shape[-2], b.shape[-1]), a)
    ad, bd, yd = describe(a), describe(b), describe(y)
    check(lib().rtenhip_matmul_f32(C.c_void_p(ctx.ptr), C.byref(ad), C.byref(bd), C.byref(yd)))
    return y


def _pool_out(x, kernel, strides, padding):
    mode, pads = _padding(padding, 4)
    strides = list(strides or [1, 1])
    ohw = (C.c_int64 * 2)()
    po = (C.c_int64 * 4)()
    check(lib().rtenhip_output_size_and_padding(
        C.c_int64(x.shape[2]), C.c_int64(x.shape[3]), C.c_int64(kernel[0]), C.c_int64(kernel[1]),
        C.c_int64(strides[0]), C.c_int64(strides[1]), C.c_int(mode), _i64(pads), C.c_int64(1),
        C.c_int64(1), ohw, po))
    return mode, pads, strides, (x.shape[0], x.shape[1], ohw[0], ohw[1])


def max_pool(x, kernel_size, strides=None, padding=None, ctx=None):
    """MaxPool (src/ops/pooling.rs:358-405)."""
    ctx = ctx or default_context()
    if x.dim() != 4:
        raise OpError(5, "Expected input to have 4 dims")
    mode, pads, strides, shape = _pool_out(x, kernel_size, strides, padding)
    y = _empty(shape, x)
    xd, yd = describe(x), describe(y)
    check(lib().rtenhip_max_pool_f32(C.c_void_p(ctx.ptr), C.byref(xd), _i64(kernel_size),
                                     _i64(strides), C.c_int(mode), _i64(pads), C.byref(yd)))
    return y


def average_pool(x, kernel_size, strides=None, padding=None, count_include_pad=False, ctx=None):
    """AveragePool (src/ops/pooling.rs:240-292)."""
    ctx = ctx or default_context()
    if x.dim() != 4:
        raise OpError(5, "Expected input to have 4 dims")
    mode, pads, strides, shape = _pool_out(x, kernel_size, strides, padding)
    y = _empty(shape, x)
    xd, yd = describe(x), describe(y)
    check(lib().rtenhip_average_pool_f32(C.c_void_p(ctx.ptr), C.byref(xd), _i64(kernel_size),
                                         _i64(strides), C.c_int(mode), _i64(pads),
                                         C.c_int(int(count_include_pad)), C.byref(yd)))
    return y


def global_average_pool(x, ctx=None):
    """GlobalAveragePool (src/ops/pooling.rs:294-356)."""
    ctx = ctx or default_context()
    if x.dim() != 4:
        raise OpError(5, "Expected input to have 4 dims")
    y = _empty((x.shape[0], x.shape[1], 1, 1), x)
    xd, yd = describe(x), describe(y)
    check(lib().rtenhip_global_average_pool_f32(C.c_void_p(ctx.ptr), C.byref(xd), C.byref(yd)))
    return y


def batch_norm(x, scale, bias, mean, var, epsilon=1e-5, out=None, ctx=None):
    """BatchNormalization (src/ops/norm.rs:18-128); ``out=x`` runs in place."""
    ctx = ctx or default_context()
    y = out if out is not None else _empty(x.shape, x)
    xd, yd = describe(x), describe(y)
    check(lib().rtenhip_batch_norm_f32(C.c_void_p(ctx.ptr), C.byref(xd),
                                       C.c_void_p(scale.data_ptr()), C.c_void_p(bias.data_ptr()),
                                       C.c_void_p(mean.data_ptr()), C.c_void_p(var.data_ptr()),
                                       C.c_float(epsilon), C.byref(yd)))
    return y


def layer_normalization(x, scale, bias=None, axis=-1, epsilon=None, ctx=None):
    """LayerNormalization (src/ops/norm.rs:245-317); epsilon defaults to 1e-5."""
    ctx = ctx or default_context()
    y = _empty(x.shape, x)
    xd, sd, yd = describe(x), describe(scale), describe(y)
    bd = C.byref(describe(bias)) if bias is not None else None
    check(lib().rtenhip_layer_norm_f32(C.c_void_p(ctx.ptr), C.byref(xd), C.byref(sd), bd,
                                       C.c_int64(axis), C.c_float(1e-5 if epsilon is None else epsilon),
                                       C.byref(yd)))
    return y


def softmax(x, axis=-1, out=None, ctx=None):
    """Softmax (src/ops/norm.rs:439-470)."""
    ctx = ctx or default_context()
    y = out if out is not None else _empty(x.shape, x)
    xd, yd = describe(x), describe(y)
    check(lib().rtenhip_softmax_f32(C.c_void_p(ctx.ptr), C.byref(xd), C.c_int64(axis),
                                    C.byref(yd)))
    return y


def log_softmax(x, axis=-1, out=None, ctx=None):
    """LogSoftmax (src/ops/norm.rs:381-430)."""
    ctx = ctx or default_context()
    y = out if out is not None else _empty(x.shape, x)
    xd, yd = describe(x), describe(y)
    check(lib().rtenhip_log_softmax_f32(C.c_void_p(ctx.ptr), C.byref(xd), C.c_int64(axis), C.byref(yd)))
    return y


def instance_normalization(x, scale, bias, epsilon=None, out=None, ctx=None):
    """InstanceNormalization (src/ops/norm.rs:131-241); epsilon defaults to 1e-5.
    scale / bias: contiguous device float tensors of C elements."""
    ctx = ctx or default_context()
    y = out if out is not None else _empty(x.shape, x)
    xd, yd = describe(x), describe(y)
    if x.dim() >= 2 and scale.numel() == x.shape[1] and bias.numel() != scale.numel():
        raise OpError(5, "bias length should match channel count")
    check(lib().rtenhip_instance_norm_f32(C.c_void_p(ctx.ptr), C.byref(xd), C.c_void_p(scale.data_ptr()),
                                          C.c_void_p(bias.data_ptr()), C.c_int64(scale.numel()),
                                          C.c_float(1e-5 if epsilon is None else epsilon), C.byref(yd)))
    return y


UNARY = {"Relu": 0, "Clip": 1, "Gelu": 2, "Erf": 3, "Sigmoid": 4, "Tanh": 5, "Exp": 6, "Silu": 7, "Sqrt": 8}


def unary(op: str, x, p0: float = 0.0, p1: float = 0.0, out=None, ctx=None):
    ctx = ctx or default_context()
    y = out if out is not None else _empty(x.shape, x)
    xd, yd = describe(x), describe(y)
    check(lib().rtenhip_unary_f32(C.c_void_p(ctx.ptr), C.c_int(UNARY[op]), C.byref(xd),
                                  C.c_float(p0), C.c_float(p1), C.byref(yd)))
    return y


def relu(x, **kw):
    return unary("Relu", x, **kw)


def clip(x, min=None, max=None, **kw):
    import numpy as np

    f = np.finfo(np.float32)
    return unary("Clip", x, float(f.min if min is None else min), float(f.max if max is None else max), **kw)


def gelu(x, **kw):
    return unary("Gelu", x, **kw)


def erf(x, **kw):
    return unary("Erf", x, **kw)


def sigmoid(x, **kw):
    return unary("Sigmoid", x, **kw)


def tanh(x, **kw):
    return unary("Tanh", x, **kw)


def exp(x, **kw):
    return unary("Exp", x, **kw)


def silu(x, **kw):
    return unary("Silu", x, **kw)


BINARY = {"Add": 0, "Sub": 1, "Mul": 2, "Div": 3, "Pow": 4}


def binary(op: str, a, b, out=None, ctx=None):
    """Broadcasting binary op (src/ops/binary_elementwise.rs:158-256)."""
    ctx = ctx or default_context()
    torch = _torch()
    try:
        shape = torch.broadcast_shapes(a.shape, b.shape)
    except RuntimeError:
        raise OpError(3, "Cannot broadcast inputs")
    y = out if out is not None else _empty(shape, a)
    ad, bd, yd = describe(a), describe(b), describe(y)
    check(lib().rtenhip_binary_f32(C.c_void_p(ctx.ptr), C.c_int(BINARY[op]), C.byref(ad),
                                   C.byref(bd), C.byref(yd)))
    return y


def reduce_mean(x, axes=None, keep_dims=False, ctx=None):
    """ReduceMean (src/ops/reduce.rs:334-400): axes None / [] = all axes."""
    ctx = ctx or default_context()
    nd = x.dim()
    ax = list(axes or [])
    res = sorted((a + nd if a < 0 else a) for a in ax) if ax else list(range(nd))
    shape = [1 if d in res else s for d, s in enumerate(x.shape) if keep_dims or d not in res]
    y = _empty(tuple(shape), x)
    xd, yd = describe(x), describe(y)
    arr = (C.c_int32 * max(1, len(ax)))(*ax)
    check(lib().rtenhip_reduce_mean_f32(C.c_void_p(ctx.ptr), C.byref(xd), arr, C.c_int32(len(ax)),
                                        C.c_int(int(keep_dims)), C.byref(yd)))
    return y


def pow(a, b, **kw):  # noqa: A001  (the operator's name)
    return binary("Pow", a, b, **kw)


def sqrt(x, **kw):
    return unary("Sqrt", x, **kw)


def add(a, b, **kw):
    return binary("Add", a, b, **kw)


def sub(a, b, **kw):
    return binary("Sub", a, b, **kw)


def mul(a, b, **kw):
    return binary("Mul", a, b, **kw)


def div(a, b, **kw):
    return binary("Div", a, b, **kw)
