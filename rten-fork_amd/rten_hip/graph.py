"""Graph / Model surface (src/graph.rs, src/model.rs) over the C ABI.

``Graph`` mirrors RTen's ``Graph`` builder + ``run`` (graph.rs:509-1073): value,
constant and operator nodes; ``run(inputs, outputs)`` plans, executes on the
GPU and returns device tensors.  ``ModelSpec`` is a plain description of a
model (the content a ``.rten`` file carries) that can be instantiated as a
``Graph`` on the device — or, in tests, evaluated by the CPU oracle.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import (DTYPE_FLOAT32, DTYPE_INT32, MAX_DIMS, OpError, Tensor, _torch, check, default_context,
               describe, describe_i32, lib)


def _attr_str(attrs: dict) -> str:
    parts = []
    for k, v in attrs.items():
        if isinstance(v, str):
            parts.append(f"{k}={v}")
        elif isinstance(v, (list, tuple)):
            parts.append(f"{k}=" + ",".join(repr(float(x)) if isinstance(x, float) else str(int(x)) for x in v))
        elif isinstance(v, bool):
            parts.append(f"{k}={int(v)}")
        elif isinstance(v, float):
            parts.append(f"{k}={v!r}")
        else:
            parts.append(f"{k}={int(v)}")
    return ";".join(parts)


class Graph:
    """Device graph (rtenhip_graph)."""

    def __init__(self, ctx=None):
        self.ctx = ctx or default_context()
        self.ptr = lib().rtenhip_graph_create(C.c_void_p(self.ctx.ptr))
        self.names: Dict[str, int] = {}
        self.input_ids: List[int] = []
        self.output_ids: List[int] = []

    def close(self):
        if getattr(self, "ptr", None):
            lib().rtenhip_graph_destroy(C.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _ret(self, nid: int, name: str) -> int:
        if nid < 0:
            raise OpError(5, lib().rtenhip_last_error_message().decode())
        if name:
            self.names[name] = nid
        return nid

    def add_value(self, name: str) -> int:
        return self._ret(lib().rtenhip_graph_add_value(C.c_void_p(self.ptr), name.encode()), name)

    def add_constant(self, name: str, data: np.ndarray) -> int:
        """Constant tensor: int32 data stays int32 (IntData), anything else is f32."""
        if np.asarray(data).dtype == np.int32:
            data = np.array(data, dtype=np.int32, order="C")  # keeps 0-d scalars 0-d
            shape = (C.c_int64 * max(1, data.ndim))(*data.shape)
            nid = lib().rtenhip_graph_add_constant_i32(C.c_void_p(self.ptr), name.encode(),
                                                      data.ctypes.data_as(C.POINTER(C.c_int32)),
                                                      shape, C.c_int32(data.ndim))
            return self._ret(nid, name)
        data = np.array(data, dtype=np.float32, order="C")
        shape = (C.c_int64 * max(1, data.ndim))(*data.shape)
        nid = lib().rtenhip_graph_add_constant(C.c_void_p(self.ptr), name.encode(),
                                              data.ctypes.data_as(C.POINTER(C.c_float)), shape,
                                              C.c_int32(data.ndim))
        return self._ret(nid, name)

    def add_op(self, name: str, op_type: str, inputs: Sequence[Optional[int]],
               outputs: Sequence[int], attrs: Optional[dict] = None) -> int:
        ins = [(-1 if i is None else int(i)) for i in inputs]
        attrs = dict(attrs or {})
        if op_type == "ConstantOfShape" and "dtype" not in attrs:
            # Scalar::Int / Scalar::Float from the Python type of the value
            attrs["dtype"] = "float" if isinstance(attrs.get("value", 0), float) else "int32"
        ia = (C.c_int32 * max(1, len(ins)))(*ins)
        oa = (C.c_int32 * max(1, len(outputs)))(*outputs)
        nid = lib().rtenhip_graph_add_op(C.c_void_p(self.ptr), name.encode(), op_type.encode(),
                                         _attr_str(attrs).encode(), ia, C.c_int32(len(ins)),
                                         oa, C.c_int32(len(outputs)))
        return self._ret(nid, name)

    def optimize(self):
        check(lib().rtenhip_graph_optimize(C.c_void_p(self.ptr)))

    def describe(self):
        """The graph after optimization, one dict per node (rtenhip_graph_describe):
        kind "op" (with ``op`` = Operator::name(), e.g. "FusedTranspose(MatMul)",
        ``inputs`` / ``outputs`` node ids), "const" or "value"."""
        text = lib().rtenhip_graph_describe(C.c_void_p(self.ptr)).decode()
        nodes = []
        for line in text.splitlines():
            f = line.split("\t")
            d = {"id": int(f[0]), "kind": f[1], "name": f[2]}
            if f[1] == "op":
                d["op"] = f[3]
                d["inputs"] = [int(x) for x in f[4].split(",") if x]
                d["outputs"] = [int(x) for x in f[5].split(",") if x]
            elif f[1] == "const":
                d["shape"] = tuple(int(x) for x in f[3].split("x") if x)
            nodes.append(d)
        return nodes

    def producer(self, value_id: int):
        """The live operator producing ``value_id`` (None for a constant or an input)."""
        for d in self.describe():
            if d["kind"] == "op" and value_id in d["outputs"]:
                return d
        return None

    def node_id(self, name: str) -> int:
        return self.names[name]

    def set_timing(self, enabled: bool):
        check(lib().rtenhip_graph_set_timing(C.c_void_p(self.ptr), C.c_int(int(enabled))))

    def timing_report(self) -> str:
        return lib().rtenhip_graph_timing_report(C.c_void_p(self.ptr)).decode()

    @staticmethod
    def _typed(inputs: Dict[int, object]):
        """Descriptors and element types (Input::FloatTensor / IntTensor) of
        float32 / int32 device tensors."""
        torch = _torch()
        descs, dts = [], []
        for t in inputs.values():
            if t.dtype == torch.int32:
                descs.append(describe_i32(t))
                dts.append(DTYPE_INT32)
            else:
                descs.append(describe(t))
                dts.append(DTYPE_FLOAT32)
        return descs, dts

    def output_info(self, inputs: Dict[int, object], outputs: Sequence[int]):
        """Planned output (shape, dtype) pairs, dtype a torch dtype."""
        torch = _torch()
        in_ids = list(inputs.keys())
        dl, tl = self._typed(inputs)
        descs = (Tensor * max(1, len(in_ids)))(*dl)
        idt = (C.c_int32 * max(1, len(in_ids)))(*tl)
        ia = (C.c_int32 * max(1, len(in_ids)))(*in_ids)
        oa = (C.c_int32 * max(1, len(outputs)))(*outputs)
        shapes = (C.c_int64 * (MAX_DIMS * max(1, len(outputs))))()
        ndims = (C.c_int32 * max(1, len(outputs)))()
        odt = (C.c_int32 * max(1, len(outputs)))()
        check(lib().rtenhip_graph_plan_typed(C.c_void_p(self.ptr), ia, descs, idt, C.c_int32(len(in_ids)),
                                             oa, C.c_int32(len(outputs)), shapes, ndims, odt))
        return [(tuple(shapes[i * MAX_DIMS + d] for d in range(ndims[i])),
                 torch.int32 if odt[i] == DTYPE_INT32 else torch.float32) for i in range(len(outputs))]

    def output_shapes(self, inputs: Dict[int, object], outputs: Sequence[int]):
        return [s for s, _ in self.output_info(inputs, outputs)]

    def synchronize(self):
        """Wait for the queued runs; raises the Gather index error
        ("Entry in `indices` is out of range") of the earliest deferred run
        that recorded one (see set_deferred_checks)."""
        check(lib().rtenhip_graph_synchronize(C.c_void_p(self.ptr)))

    def set_deferred_checks(self, enabled: bool):
        """False (default): a run whose Gather indices are out of range raises
        from that run, like Model::run (gather.rs:52-60); the run waits for its
        own check.  True: runs queue without a host round trip and the error is
        raised by synchronize() only -- never by a later run."""
        check(lib().rtenhip_graph_set_deferred_checks(C.c_void_p(self.ptr), C.c_int(int(enabled))))

    def run(self, inputs: Dict[int, object], outputs: Sequence[int], out=None):
        """Graph::run: inputs {value id: float32 or int32 device tensor};
        returns device tensors (int32 where the graph's value is int32).
        A plan with a Gather on non-constant indices checks them on the device
        and raises their error from this run (set_deferred_checks changes
        that)."""
        torch = _torch()
        self.ctx.sync_stream()
        in_ids = list(inputs.keys())
        if out is None:
            dev = next(iter(inputs.values())).device if inputs else torch.device("cuda")
            out = [torch.empty(s, dtype=dt, device=dev) for s, dt in self.output_info(inputs, outputs)]
        dl, tl = self._typed(inputs)
        descs = (Tensor * max(1, len(in_ids)))(*dl)
        idt = (C.c_int32 * max(1, len(in_ids)))(*tl)
        odescs = (Tensor * max(1, len(out)))(*[describe_i32(t) if t.dtype == torch.int32 else describe(t)
                                                for t in out])
        ia = (C.c_int32 * max(1, len(in_ids)))(*in_ids)
        oa = (C.c_int32 * max(1, len(outputs)))(*outputs)
        check(lib().rtenhip_graph_run_typed(C.c_void_p(self.ptr), ia, descs, idt, C.c_int32(len(in_ids)),
                                            oa, odescs, C.c_int32(len(outputs))))
        return out

    def run_host(self, inputs: Dict[int, np.ndarray], outputs: Sequence[int], out: Sequence[np.ndarray]) -> int:
        """Model::run over HOST arrays (rtenhip_graph_run_host): inputs {value
        id: float32 / int32 numpy array}, outputs written into ``out`` (host
        arrays of the planned shapes; pinned ones from host.pinned overlap the
        forward).  Returns without waiting; the run id goes to wait().  No
        torch tensor is involved: the staging pipeline is librten_hip.so's."""
        from .host import _bind, host_desc

        L = _bind()
        in_ids = list(inputs.keys())
        arrs = list(inputs.values())
        descs = (Tensor * max(1, len(arrs)))(*[host_desc(a) for a in arrs])
        idt = (C.c_int32 * max(1, len(arrs)))(*[DTYPE_INT32 if a.dtype == np.int32 else DTYPE_FLOAT32
                                                  for a in arrs])
        odescs = (Tensor * max(1, len(out)))(*[host_desc(a) for a in out])
        ia = (C.c_int32 * max(1, len(in_ids)))(*in_ids)
        oa = (C.c_int32 * max(1, len(outputs)))(*outputs)
        rid = C.c_uint64(0)
        check(L.rtenhip_graph_run_host(C.c_void_p(self.ptr), ia, descs, idt, C.c_int32(len(in_ids)), oa, odescs,
                                       C.c_int32(len(outputs)), C.byref(rid)))
        return int(rid.value)

    def wait(self, run_id: int = 0):
        """rtenhip_graph_wait: block until host run ``run_id`` (0: every queued
        run) has its outputs on the host; raises its Gather index error."""
        from .host import _bind

        check(_bind().rtenhip_graph_wait(C.c_void_p(self.ptr), C.c_uint64(run_id)))


@dataclass
class Node:
    kind: str                      # "value" | "const" | "op"
    name: str
    data: Optional[np.ndarray] = None
    op_type: str = ""
    attrs: dict = field(default_factory=dict)
    inputs: List[Optional[str]] = field(default_factory=list)
    outputs: List[str] = field(default_factory=list)


class ModelSpec:
    """A model as data: the node list a .rten file holds (schema.fbs Graph)."""

    def __init__(self, name: str):
        self.name = name
        self.nodes: List[Node] = []
        self.inputs: List[str] = []
        self.outputs: List[str] = []
        self._n = 0

    def value(self, name: str) -> str:
        self.nodes.append(Node("value", name))
        return name

    def const(self, name: str, data: np.ndarray) -> str:
        """Constant node: int32 arrays stay int32 (IntData), others are f32."""
        data = np.asarray(data)
        dt = np.int32 if data.dtype == np.int32 else np.float32
        # np.array (not ascontiguousarray) keeps 0-d scalars 0-d
        self.nodes.append(Node("const", name, data=np.array(data, dt, order="C", copy=True)))
        return name

    def op(self, op_type: str, inputs: Sequence[Optional[str]], attrs: Optional[dict] = None,
           name: Optional[str] = None, n_outputs: int = 1) -> str:
        self._n += 1
        name = name or f"{op_type.lower()}_{self._n}"
        outs = [self.value(f"{name}_out" if n_outputs == 1 else f"{name}_out{i}")
                for i in range(n_outputs)]
        self.nodes.append(Node("op", name, op_type=op_type, attrs=dict(attrs or {}),
                               inputs=list(inputs), outputs=outs))
        return outs[0]

    def n_params(self) -> int:
        return sum(n.data.size for n in self.nodes if n.kind == "const")

    def to_graph(self, ctx=None, optimize: bool = True) -> Graph:
        """Instantiate on the device (constants uploaded once)."""
        g = Graph(ctx)
        ids: Dict[str, int] = {}
        for n in self.nodes:
            if n.kind == "value":
                ids[n.name] = g.add_value(n.name)
            elif n.kind == "const":
                ids[n.name] = g.add_constant(n.name, n.data)
        for n in self.nodes:
            if n.kind == "op":
                g.add_op(n.name, n.op_type, [None if i is None else ids[i] for i in n.inputs],
                         [ids[o] for o in n.outputs], n.attrs)
        g.input_ids = [ids[i] for i in self.inputs]
        g.output_ids = [ids[o] for o in self.outputs]
        # The optimizer must know the model outputs (never fuse them away).
        ia = (C.c_int32 * max(1, len(g.input_ids)))(*g.input_ids)
        oa = (C.c_int32 * max(1, len(g.output_ids)))(*g.output_ids)
        check(lib().rtenhip_graph_set_io(C.c_void_p(g.ptr), ia, C.c_int32(len(g.input_ids)), oa,
                                         C.c_int32(len(g.output_ids))))
        if optimize:
            g.optimize()
        return g
