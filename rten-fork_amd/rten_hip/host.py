"""Host-resident and batch-sharded runs through the C ABI (graph_io.cpp).

These are thin ctypes views of the entry points a Rust ``Model::run`` caller
binds (include/rten_hip.h):

- ``pinned(shape, dtype)``: a numpy array over ``rtenhip_host_alloc`` memory
  (page-locked, what the upload DMA reads directly);
- ``Graph.run_host`` / ``Graph.wait`` (rten_hip/graph.py): ``Model::run`` over
  host arrays, pipelined inside librten_hip.so (two device slots, a
  high-priority copy stream, per-slot events);
- ``ShardedModel``: one ``.rten`` replica per device, the batch split into
  contiguous slices, outputs all-gathered with RCCL when the devices are
  distinct, else copied back shard by shard.

No torch tensor crosses these calls: host numpy arrays in, host arrays out.
"""
from __future__ import annotations

import ctypes as C
from typing import Sequence

import numpy as np

from . import MAX_DIMS, OpError, Tensor, check, lib

_bound = False


def _bind():
    global _bound
    if _bound:
        return lib()
    L = lib()
    L.rtenhip_host_alloc.restype = C.c_void_p
    L.rtenhip_host_alloc.argtypes = [C.c_void_p, C.c_size_t]
    L.rtenhip_host_free.argtypes = [C.c_void_p, C.c_void_p]
    L.rtenhip_graph_run_host.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(Tensor), C.POINTER(C.c_int32),
                                         C.c_int32, C.POINTER(C.c_int32), C.POINTER(Tensor), C.c_int32,
                                         C.POINTER(C.c_uint64)]
    L.rtenhip_graph_wait.argtypes = [C.c_void_p, C.c_uint64]
    L.rtenhip_sharded_create.restype = C.c_void_p
    L.rtenhip_sharded_create.argtypes = [C.POINTER(C.c_uint8), C.c_size_t, C.POINTER(C.c_int32), C.c_int32, C.c_int]
    L.rtenhip_sharded_destroy.argtypes = [C.c_void_p]
    L.rtenhip_sharded_gather_mode.restype = C.c_int32
    L.rtenhip_sharded_gather_mode.argtypes = [C.c_void_p]
    L.rtenhip_sharded_graph.restype = C.c_void_p
    L.rtenhip_sharded_graph.argtypes = [C.c_void_p, C.c_int32]
    L.rtenhip_sharded_run_host.argtypes = [C.c_void_p, C.POINTER(Tensor), C.POINTER(Tensor)]
    L.rtenhip_sharded_gathered.restype = C.c_void_p
    L.rtenhip_sharded_gathered.argtypes = [C.c_void_p, C.c_int32]
    _bound = True
    return L


class _Pinned:
    """Owner of one rtenhip_host_alloc block (freed with the last array view)."""

    def __init__(self, nbytes: int):
        self.ptr = _bind().rtenhip_host_alloc(None, C.c_size_t(max(nbytes, 4)))
        if not self.ptr:
            raise OpError(7, lib().rtenhip_last_error_message().decode())

    def __del__(self):
        try:
            if self.ptr:
                lib().rtenhip_host_free(None, C.c_void_p(self.ptr))
                self.ptr = None
        except Exception:
            pass


def pinned(shape, dtype=np.float32) -> np.ndarray:
    """An uninitialised numpy array in page-locked host memory."""
    dtype = np.dtype(dtype)
    shape = tuple(int(s) for s in shape)
    n = int(np.prod(shape)) if shape else 1
    owner = _Pinned(n * dtype.itemsize)
    buf = (C.c_char * max(n * dtype.itemsize, 1)).from_address(owner.ptr)
    buf._owner = owner  # the array's base keeps the allocation alive
    return np.frombuffer(buf, dtype=dtype, count=n).reshape(shape)


def host_desc(a: np.ndarray) -> Tensor:
    """rtenhip_tensor over a contiguous host numpy array (float32 or int32)."""
    if a.dtype not in (np.float32, np.int32):
        raise OpError(1, "IncorrectInputType: expected float32 or int32")
    if not a.flags["C_CONTIGUOUS"]:
        raise OpError(6, "host arrays must be C-contiguous")
    if a.ndim > MAX_DIMS:
        raise OpError(6, "too many dims")
    d = Tensor()
    d.data = a.ctypes.data if a.size else None
    d.ndim = a.ndim
    st = 1
    for i in range(a.ndim - 1, -1, -1):
        d.shape[i] = a.shape[i]
        d.strides[i] = st
        st *= a.shape[i]
    return d


class ShardedModel:
    """rtenhip_sharded_*: a .rten model replicated on ``devices`` (repeats
    allowed: two shards on one GPU take the host-copy gather), run over host
    batches with the batch split into contiguous slices."""

    def __init__(self, model_bytes: bytes, devices: Sequence[int], optimize: bool = True):
        L = _bind()
        self._bytes = (C.c_uint8 * len(model_bytes)).from_buffer_copy(model_bytes)
        devs = (C.c_int32 * len(devices))(*devices)
        self.ptr = L.rtenhip_sharded_create(self._bytes, C.c_size_t(len(model_bytes)), devs,
                                            C.c_int32(len(devices)), C.c_int(int(optimize)))
        if not self.ptr:
            raise OpError(lib().rtenhip_last_error_code(), lib().rtenhip_last_error_message().decode())
        self.devices = list(devices)

    @property
    def gather_mode(self) -> str:
        return "rccl" if _bind().rtenhip_sharded_gather_mode(C.c_void_p(self.ptr)) else "host"

    def timing_report(self, shard: int) -> str:
        g = _bind().rtenhip_sharded_graph(C.c_void_p(self.ptr), C.c_int32(shard))
        return lib().rtenhip_graph_timing_report(C.c_void_p(g)).decode()

    def run(self, x: np.ndarray, out: np.ndarray) -> np.ndarray:
        """Model::run over the host batch x -> out (both host arrays)."""
        xd, yd = host_desc(x), host_desc(out)
        check(_bind().rtenhip_sharded_run_host(C.c_void_p(self.ptr), C.byref(xd), C.byref(yd)))
        return out

    def close(self):
        if getattr(self, "ptr", None):
            _bind().rtenhip_sharded_destroy(C.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


__all__ = ["pinned", "host_desc", "ShardedModel"]
