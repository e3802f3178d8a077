""".rten V2 model files: writer (the layout rten-convert produces,
rten-convert/rten_convert/converter.py:1395-1545 and tensor_data.py) and the
device loader binding (``load_model`` -> rtenhip_model_load, src/model.rs:265-522).

The file is a 32-byte header (src/header.rs:57-146: b"RTEN", version 2, model
offset/length, tensor-data offset), a FlatBuffers ``Model`` (src/schema.fbs,
schema_version 1) and a 64-byte-aligned tensor-data segment holding large
constants (``ConstantNode.data_offset``); small constants are stored inline.
There is no flatbuffers package in this image, so ``_Builder`` is a minimal
FlatBuffers encoder: tables with vtables, scalar/offset vectors, strings and
unions, children laid out after their parents (uoffsets point forward).
"""
from __future__ import annotations

import ctypes as C
import os
import struct
from typing import Dict, List, Optional, Tuple

import numpy as np

# sg::OperatorType (schema.fbs:12-121), enum order.
OP_TYPES = [
    "Add", "ArgMin", "ArgMax", "AveragePool", "BatchNormalization", "Cast", "Clip", "Concat",
    "ConstantOfShape", "Conv", "ConvTranspose", "Cos", "CumSum", "Div", "Equal", "Erf", "Expand",
    "Flatten", "Gather", "Gemm", "GlobalAveragePool", "Greater", "GRU", "Identity", "LeakyRelu",
    "Less", "LessOrEqual", "Log", "LogSoftmax", "LSTM", "MatMul", "MaxPool", "Mod", "Mul", "Pad",
    "Pow", "Range", "ReduceMean", "ReduceL2", "Relu", "Reshape", "Resize", "Shape", "Sigmoid",
    "Sin", "Slice", "Split", "Sqrt", "Squeeze", "Softmax", "Sub", "Tanh", "Transpose", "Unsqueeze",
    "Where", "ReduceProd", "ReduceSum", "ReduceMin", "ReduceMax", "NonZero", "ScatterElements",
    "Tile", "Not", "Abs", "Max", "Mean", "Min", "Sum", "OneHot", "Round", "Floor", "Ceil",
    "Reciprocal", "TopK", "Neg", "Exp", "GreaterOrEqual", "Size", "Tan", "Acos", "Asin", "Atan",
    "InstanceNormalization", "HardSigmoid", "HardSwish", "And", "Or", "Xor", "Trilu", "ScatterND",
    "NonMaxSuppression", "Sign", "GatherElements", "LayerNormalization", "ReduceSumSquare",
    "RandomUniform", "Elu", "RandomUniformLike", "RandomNormal", "RandomNormalLike", "Softplus",
    "GatherND", "Gelu", "Einsum", "If"]

# sg::OperatorAttrs union ids (schema.fbs OperatorAttrs, NONE = 0).
ATTRS_AVERAGE_POOL, ATTRS_BATCH_NORM, ATTRS_CONV, ATTRS_CONV_TRANSPOSE, ATTRS_FLATTEN = 2, 3, 7, 8, 9
ATTRS_GEMM, ATTRS_MAX_POOL, ATTRS_RESHAPE, ATTRS_SOFTMAX = 11, 15, 17, 20
ATTRS_TRANSPOSE, ATTRS_LAYER_NORM, ATTRS_GELU = 21, 30, 37
ATTRS_CAST, ATTRS_GATHER = 4, 10
ATTRS_CONCAT, ATTRS_CONSTANT_OF_SHAPE, ATTRS_REDUCE_MEAN = 5, 6, 16
SCALAR_INT, SCALAR_FLOAT = 1, 2  # union Scalar (schema.fbs:236-239)
NODE_OPERATOR, NODE_CONSTANT, NODE_VALUE = 1, 2, 3
CONST_FLOAT_DATA, CONST_INT_DATA = 1, 2
DTYPE_INT32, DTYPE_FLOAT32 = 0, 1
AUTOPAD_SAME, AUTOPAD_NOTSET = 0, 1

# Field slots (vtable index) of every table the writer emits, by field name
# (schema.fbs; pinned against the reference's generated code by
# tests/test_schema_pin.py and tests/golden/schema_slots.json).
SLOTS = {
    "Model": {"schema_version": 0, "graph": 1, "metadata": 2},
    "Graph": {"nodes": 0, "inputs": 1, "outputs": 2, "captures": 3},
    "Node": {"name": 0, "data_type": 1, "data": 2},
    "OperatorNode": {"type_": 0, "attrs_type": 1, "attrs": 2, "inputs": 3, "outputs": 4},
    "ValueNode": {"shape": 0},
    "ConstantNode": {"shape": 0, "data_type": 1, "data": 2, "dtype": 3, "data_offset": 4},
    "FloatData": {"data": 0},
    "IntData": {"data": 0},
    "ConvAttrs": {"auto_pad": 0, "pads": 1, "groups": 2, "strides": 3, "dilations": 4},
    "ConvTransposeAttrs": {"strides": 0, "auto_pad": 1, "pads": 2},
    "MaxPoolAttrs": {"kernel_size": 0, "auto_pad": 1, "pads": 2, "strides": 3},
    "AveragePoolAttrs": {"kernel_size": 0, "auto_pad": 1, "pads": 2, "strides": 3, "count_include_pad": 4},
    "BatchNormalizationAttrs": {"epsilon": 0},
    "GemmAttrs": {"alpha": 0, "beta": 1, "transpose_a": 2, "transpose_b": 3},
    "FlattenAttrs": {"axis": 0},
    "SoftmaxAttrs": {"axis": 0},
    "LayerNormalizationAttrs": {"axis": 0, "epsilon": 1},
    "TransposeAttrs": {"perm": 0},
    "ReshapeAttrs": {"allow_zero": 0},
    "GatherAttrs": {"axis": 0},
    "CastAttrs": {"to": 0},
    "ConcatAttrs": {"axis": 0},
    "ReduceMeanAttrs": {"axes": 0, "keep_dims": 1},
    "ConstantOfShapeAttrs": {"value_type": 0, "value": 1},
    "IntScalar": {"value": 0},
    "FloatScalar": {"value": 0},
    "GeluAttrs": {},
}


def _T(table: str, *fields) -> "Table":
    """Table of schema type ``table`` from (field name, kind, value) triples."""
    slots = SLOTS[table]
    return Table([(slots[name], kind, value) for name, kind, value in fields])


HEADER_LEN = 32
TENSOR_ALIGN = 64
INLINE_MAX_ELEMS = 16

_SCALAR = {"u8": "<B", "bool": "<B", "u16": "<H", "i32": "<i", "u32": "<I", "f32": "<f",
           "u64": "<Q"}


class Table:
    """A FlatBuffers table: fields = [(slot, kind, value)]; kind is a scalar
    kind from _SCALAR or "ref" (value: Table / Vector / String)."""

    def __init__(self, fields):
        self.fields = [f for f in fields if f[2] is not None]


class Vector:
    def __init__(self, kind: str, items):
        self.kind = kind            # "u32" | "i32" | "f32" | "ref"
        self.items = items


class String:
    def __init__(self, s: str):
        self.data = s.encode()


class _Builder:
    """Forward FlatBuffers encoder: the root offset at 0, then each object
    appended after the one that references it."""

    def __init__(self):
        self.buf = bytearray(4)
        self.queue: List[Tuple[int, object]] = []

    def _align(self, a: int, extra: int = 0):
        while (len(self.buf) + extra) % a:
            self.buf.append(0)

    def _put(self, fmt: str, v):
        self.buf += struct.pack(fmt, v)

    def _place(self, obj) -> int:
        if isinstance(obj, String):
            self._align(4)
            pos = len(self.buf)
            self._put("<I", len(obj.data))
            self.buf += obj.data + b"\0"
            return pos
        if isinstance(obj, Vector):
            esize = 8 if obj.kind == "u64" else 4
            self._align(max(4, esize), 4)
            pos = len(self.buf)
            self._put("<I", len(obj.items))
            if obj.kind == "ref":
                for it in obj.items:
                    self.queue.append((len(self.buf), it))
                    self._put("<I", 0)
            elif obj.kind == "f32":
                self.buf += np.asarray(obj.items, "<f4").tobytes()
            else:
                self.buf += struct.pack("<%d%s" % (len(obj.items), _SCALAR[obj.kind][1]),
                                        *obj.items)
            return pos
        assert isinstance(obj, Table)
        size = {k: struct.calcsize(f) for k, f in _SCALAR.items()}
        size["ref"] = 4
        fields = sorted(obj.fields, key=lambda f: -size[f[1]])
        # inline layout: soffset at 0, fields by descending size, each aligned
        offs, cur = {}, 4
        for slot, kind, _ in fields:
            sz = size[kind]
            cur = (cur + sz - 1) // sz * sz
            offs[slot] = cur
            cur += sz
        tsize = (cur + 3) // 4 * 4
        nslots = max([f[0] for f in fields], default=-1) + 1
        # vtable right before the table
        self._align(2)
        vt = len(self.buf)
        self._put("<H", 4 + 2 * nslots)
        self._put("<H", tsize)
        for s in range(nslots):
            self._put("<H", offs.get(s, 0))
        self._align(8)
        pos = len(self.buf)
        self.buf += bytes(tsize)
        struct.pack_into("<i", self.buf, pos, pos - vt)
        for slot, kind, v in fields:
            if kind == "ref":
                self.queue.append((pos + offs[slot], v))
            else:
                struct.pack_into(_SCALAR[kind], self.buf, pos + offs[slot], v)
        return pos

    def finish(self, root: Table) -> bytes:
        self.queue.append((0, root))
        while self.queue:
            at, obj = self.queue.pop(0)
            pos = self._place(obj)
            struct.pack_into("<I", self.buf, at, pos - at)
        self._align(8)
        return bytes(self.buf)


def _u32v(v):
    return Vector("u32", [int(x) for x in v])


def _op_attrs(op_type: str, a: dict):
    """(union type, attrs table) as rten-convert writes them."""
    def padding():
        if str(a.get("auto_pad", "notset")).lower() in ("same", "same_upper"):
            return [("auto_pad", "u8", AUTOPAD_SAME)]
        return [("auto_pad", "u8", AUTOPAD_NOTSET), ("pads", "ref", _u32v(a.get("pads", [0, 0, 0, 0])))]

    if op_type == "Conv":
        return ATTRS_CONV, _T("ConvAttrs", *padding(),
                              ("groups", "u32", int(a.get("groups", 1))),
                              ("strides", "ref", _u32v(a.get("strides", [1, 1]))),
                              ("dilations", "ref", _u32v(a.get("dilations", [1, 1]))))
    if op_type == "ConvTranspose":
        return ATTRS_CONV_TRANSPOSE, _T("ConvTransposeAttrs", ("strides", "ref", _u32v(a.get("strides", [1, 1]))),
                                        *padding())
    if op_type in ("MaxPool", "AveragePool"):
        f = [("kernel_size", "ref", _u32v(a["kernel_size"]))] + padding() + [
            ("strides", "ref", _u32v(a.get("strides", [1, 1])))]
        if op_type == "AveragePool":
            f.append(("count_include_pad", "bool", int(bool(a.get("count_include_pad", 0)))))
            return ATTRS_AVERAGE_POOL, _T("AveragePoolAttrs", *f)
        return ATTRS_MAX_POOL, _T("MaxPoolAttrs", *f)
    if op_type in ("BatchNormalization", "InstanceNormalization"):
        return ATTRS_BATCH_NORM, _T("BatchNormalizationAttrs", ("epsilon", "f32", float(a.get("epsilon", 1e-5))))
    if op_type == "Gemm":
        return ATTRS_GEMM, _T("GemmAttrs", ("alpha", "f32", float(a.get("alpha", 1.0))),
                              ("beta", "f32", float(a.get("beta", 1.0))),
                              ("transpose_a", "bool", int(bool(a.get("transA", 0)))),
                              ("transpose_b", "bool", int(bool(a.get("transB", 0)))))
    if op_type == "Flatten":
        return ATTRS_FLATTEN, _T("FlattenAttrs", ("axis", "i32", int(a.get("axis", 1))))
    if op_type in ("Softmax", "LogSoftmax"):
        return ATTRS_SOFTMAX, _T("SoftmaxAttrs", ("axis", "i32", int(a.get("axis", -1))))
    if op_type == "LayerNormalization":
        return ATTRS_LAYER_NORM, _T("LayerNormalizationAttrs", ("axis", "i32", int(a.get("axis", -1))),
                                    ("epsilon", "f32", float(a.get("epsilon", 1e-5))))
    if op_type == "Transpose":
        perm = a.get("perm")
        return ATTRS_TRANSPOSE, _T("TransposeAttrs", ("perm", "ref", _u32v(perm) if perm is not None else None))
    if op_type == "Reshape":
        return ATTRS_RESHAPE, _T("ReshapeAttrs", ("allow_zero", "bool", int(bool(a.get("allowzero", 0)))))
    if op_type == "Gelu":
        return ATTRS_GELU, _T("GeluAttrs")
    if op_type == "Gather":
        return ATTRS_GATHER, _T("GatherAttrs", ("axis", "i32", int(a.get("axis", 0))))
    if op_type == "Cast":
        # CastAttrs::to, sg::DataType: Int32 = 0 (the schema default), Float = 1
        return ATTRS_CAST, _T("CastAttrs", ("to", "u8", int(a.get("to", 0))))
    if op_type == "Concat":
        return ATTRS_CONCAT, _T("ConcatAttrs", ("axis", "i32", int(a.get("axis", 0))))
    if op_type == "ReduceMean":
        f = [("keep_dims", "bool", int(bool(a.get("keep_dims", 0))))]
        if a.get("axes") is not None:
            f.append(("axes", "ref", Vector("i32", [int(x) for x in a["axes"]])))
        return ATTRS_REDUCE_MEAN, _T("ReduceMeanAttrs", *f)
    if op_type == "ConstantOfShape":
        v = a.get("value", 0)
        is_float = a.get("dtype") == "float" or isinstance(v, float)
        scalar = _T("FloatScalar", ("value", "f32", float(v))) if is_float else _T("IntScalar", ("value", "i32", int(v)))
        return ATTRS_CONSTANT_OF_SHAPE, _T("ConstantOfShapeAttrs",
                                           ("value_type", "u8", SCALAR_FLOAT if is_float else SCALAR_INT),
                                           ("value", "ref", scalar))
    return 0, None


def to_rten_bytes(spec, inline_max: int = INLINE_MAX_ELEMS) -> bytes:
    """Serialize a ModelSpec as a .rten V2 file.  int32 constants, and
    constants read as a shape (Reshape input 1), are stored as int32 like an
    ONNX export."""
    index: Dict[str, int] = {n.name: i for i, n in enumerate(spec.nodes)}
    int_consts = set()
    for n in spec.nodes:
        if n.kind == "op" and n.op_type == "Reshape" and len(n.inputs) > 1 and n.inputs[1]:
            int_consts.add(n.inputs[1])
    tensors: List[np.ndarray] = []
    tensor_off = 0
    nodes = []
    for n in spec.nodes:
        if n.kind == "value":
            data = _T("ValueNode", ("shape", "ref", None))
            kind = NODE_VALUE
        elif n.kind == "const":
            arr = np.asarray(n.data)
            is_int = n.name in int_consts or arr.dtype == np.int32
            arr = arr.astype("<i4" if is_int else "<f4")
            shape = _u32v(arr.shape)
            if arr.size <= inline_max:
                payload = _T("IntData" if is_int else "FloatData",
                             ("data", "ref", Vector("i32" if is_int else "f32", arr.reshape(-1).tolist())))
                data = _T("ConstantNode", ("shape", "ref", shape),
                          ("data_type", "u8", CONST_INT_DATA if is_int else CONST_FLOAT_DATA), ("data", "ref", payload))
            else:
                pad = (-tensor_off) % TENSOR_ALIGN
                tensor_off += pad
                tensors.append((tensor_off, arr))
                data = _T("ConstantNode", ("shape", "ref", shape),
                          ("dtype", "u16", DTYPE_INT32 if is_int else DTYPE_FLOAT32), ("data_offset", "u64", tensor_off))
                tensor_off += arr.size * 4
            kind = NODE_CONSTANT
        else:
            at, attrs = _op_attrs(n.op_type, n.attrs)
            fields = [("type_", "u8", OP_TYPES.index(n.op_type)),
                      ("inputs", "ref", Vector("i32", [-1 if i is None else index[i] for i in n.inputs])),
                      ("outputs", "ref", Vector("i32", [index[o] for o in n.outputs]))]
            if attrs is not None:
                fields += [("attrs_type", "u8", at), ("attrs", "ref", attrs)]
            data = _T("OperatorNode", *fields)
            kind = NODE_OPERATOR
        nodes.append(_T("Node", ("name", "ref", String(n.name)), ("data_type", "u8", kind), ("data", "ref", data)))
    graph = _T("Graph", ("nodes", "ref", Vector("ref", nodes)),
               ("inputs", "ref", _u32v([index[i] for i in spec.inputs])),
               ("outputs", "ref", _u32v([index[o] for o in spec.outputs])))
    model = _T("Model", ("schema_version", "i32", 1), ("graph", "ref", graph))
    fb = _Builder().finish(model)
    tensor_data_offset = (HEADER_LEN + len(fb) + TENSOR_ALIGN - 1) // TENSOR_ALIGN * TENSOR_ALIGN
    out = bytearray(b"RTEN" + struct.pack("<IQQQ", 2, HEADER_LEN, len(fb), tensor_data_offset))
    out += fb
    out += bytes(tensor_data_offset - len(out))
    for off, arr in tensors:
        out += bytes(tensor_data_offset + off - len(out))
        out += arr.tobytes()
    return bytes(out)


def write_rten(spec, path: str, **kw) -> None:
    with open(path, "wb") as f:
        f.write(to_rten_bytes(spec, **kw))


def _bytes(src) -> bytes:
    if isinstance(src, (bytes, bytearray)):
        return bytes(src)
    with open(os.fspath(src), "rb") as f:
        return f.read()


def describe_model(src) -> str:
    """Host-only parse of a .rten file (rtenhip_model_describe)."""
    from . import OpError, lib

    data = _bytes(src)
    buf = C.create_string_buffer(data, len(data))
    r = lib().rtenhip_model_describe(C.cast(buf, C.POINTER(C.c_uint8)), C.c_size_t(len(data)))
    if not r:
        raise OpError(lib().rtenhip_last_error_code(), lib().rtenhip_last_error_message().decode())
    return r.decode()


def load_model(src, ctx=None, optimize: bool = True):
    """Model::load (src/model.rs:190-199): parse a .rten file, upload its
    constants and return a device Graph with input_ids / output_ids set."""
    from . import OpError, default_context, lib
    from .graph import Graph

    data = _bytes(src)
    buf = C.create_string_buffer(data, len(data))
    g = Graph.__new__(Graph)
    g.ctx = ctx or default_context()
    g.names = {}
    ptr = lib().rtenhip_model_load_with_options(C.c_void_p(g.ctx.ptr), C.cast(buf, C.POINTER(C.c_uint8)),
                                                C.c_size_t(len(data)), C.c_int(int(optimize)))
    if not ptr:
        g.ptr = None
        raise OpError(lib().rtenhip_last_error_code(), lib().rtenhip_last_error_message().decode())
    g.ptr = ptr
    ids = (C.c_int32 * 64)()
    n = lib().rtenhip_model_input_ids(C.c_void_p(ptr), ids, 64)
    g.input_ids = [ids[i] for i in range(min(n, 64))]
    n = lib().rtenhip_model_output_ids(C.c_void_p(ptr), ids, 64)
    g.output_ids = [ids[i] for i in range(min(n, 64))]
    return g
