"""The .rten format pinned to the reference's own generated FlatBuffers code
(tests/golden/schema_slots.json, made from src/schema_generated.rs by
tests/golden/make_schema_slots.py), so the writer (rten_hip/rten_file.py) and
the loader (csrc/model.cpp) are checked against the format rather than only
against each other:

- enum values: OperatorType, the OperatorAttrs union, NodeKind, ConstantData,
  ConstantDataType, AutoPad, DataType, Scalar;
- every table field slot the writer emits;
- the loader's decoding of each supported attribute table, with explicit
  values and with every field absent (the schema defaults, read through the
  reference's ReadOp rules, op_registry.rs:239-820).
"""
import json
import os

import numpy as np
import pytest

from rten_hip import rten_file
from rten_hip.graph import ModelSpec

FIX = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "schema_slots.json")))
ENUMS, TABLES = FIX["enums"], FIX["tables"]


def test_operator_type_ids():
    ids = ENUMS["OperatorType"]
    assert rten_file.OP_TYPES == [n for n, _ in sorted(ids.items(), key=lambda kv: kv[1])]


def test_union_and_enum_ids():
    u = ENUMS["OperatorAttrs"]
    R = rten_file
    for const, table in [("ATTRS_AVERAGE_POOL", "AveragePoolAttrs"), ("ATTRS_BATCH_NORM", "BatchNormalizationAttrs"),
                         ("ATTRS_CONV", "ConvAttrs"), ("ATTRS_CONV_TRANSPOSE", "ConvTransposeAttrs"),
                         ("ATTRS_FLATTEN", "FlattenAttrs"), ("ATTRS_GEMM", "GemmAttrs"),
                         ("ATTRS_MAX_POOL", "MaxPoolAttrs"), ("ATTRS_RESHAPE", "ReshapeAttrs"),
                         ("ATTRS_SOFTMAX", "SoftmaxAttrs"), ("ATTRS_TRANSPOSE", "TransposeAttrs"),
                         ("ATTRS_LAYER_NORM", "LayerNormalizationAttrs"), ("ATTRS_GELU", "GeluAttrs"),
                         ("ATTRS_CAST", "CastAttrs"), ("ATTRS_GATHER", "GatherAttrs"),
                         ("ATTRS_CONCAT", "ConcatAttrs"), ("ATTRS_CONSTANT_OF_SHAPE", "ConstantOfShapeAttrs"),
                         ("ATTRS_REDUCE_MEAN", "ReduceMeanAttrs")]:
        assert getattr(R, const) == u[table], const
    assert (R.NODE_OPERATOR, R.NODE_CONSTANT, R.NODE_VALUE) == (
        ENUMS["NodeKind"]["OperatorNode"], ENUMS["NodeKind"]["ConstantNode"], ENUMS["NodeKind"]["ValueNode"])
    assert (R.CONST_FLOAT_DATA, R.CONST_INT_DATA) == (ENUMS["ConstantData"]["FloatData"],
                                                       ENUMS["ConstantData"]["IntData"])
    assert (R.DTYPE_INT32, R.DTYPE_FLOAT32) == (ENUMS["ConstantDataType"]["Int32"],
                                                ENUMS["ConstantDataType"]["Float32"])
    assert (R.AUTOPAD_SAME, R.AUTOPAD_NOTSET) == (ENUMS["AutoPad"]["Same"], ENUMS["AutoPad"]["NotSet"])
    assert (R.SCALAR_INT, R.SCALAR_FLOAT) == (ENUMS["Scalar"]["IntScalar"], ENUMS["Scalar"]["FloatScalar"])
    assert ENUMS["DataType"] == {"Int32": 0, "Float": 1}  # Cast's `to`, as the loader decodes it


@pytest.mark.parametrize("table", sorted(rten_file.SLOTS))
def test_writer_slots(table):
    fields = TABLES.get(table, {})  # field-less tables (GeluAttrs) have no VT_ slots
    for name, slot in rten_file.SLOTS[table].items():
        assert fields[name]["slot"] == slot, (table, name)


def _one_op(op_type, attrs, inputs=1):
    m = ModelSpec("pin")
    x = m.value("x")
    m.inputs = ["x"]
    m.outputs = [m.op(op_type, [x] * inputs, attrs, name="op")]
    return m


def _decoded(spec, monkeypatch=None):
    text = rten_file.describe_model(rten_file.to_rten_bytes(spec))
    line = next(l for l in text.splitlines() if " op op " in l)
    out = {}
    for tok in line.split(" ")[6:]:
        k, v = tok.split("=", 1)
        out[k] = v
    return out


@pytest.mark.parametrize("op_type,attrs,expect", [
    ("Conv", {"pads": [1, 2, 3, 4], "strides": [2, 3], "dilations": [4, 5], "groups": 7},
     {"pads": "1,2,3,4", "strides": "2,3", "dilations": "4,5", "groups": "7"}),
    ("Conv", {"auto_pad": "same"}, {"auto_pad": "same"}),
    ("ConvTranspose", {"strides": [3, 2], "pads": [1, 0, 1, 0]}, {"strides": "3,2", "pads": "1,0,1,0"}),
    ("MaxPool", {"kernel_size": [3, 2], "strides": [2, 1], "pads": [1, 1, 0, 0]},
     {"kernel_size": "3,2", "strides": "2,1", "pads": "1,1,0,0"}),
    ("AveragePool", {"kernel_size": [2, 2], "count_include_pad": 1}, {"count_include_pad": "1"}),
    ("BatchNormalization", {"epsilon": 0.125}, {"epsilon": "0.125"}),
    ("Gemm", {"alpha": 0.5, "beta": 0.25, "transA": 1, "transB": 1},
     {"alpha": "0.5", "beta": "0.25", "transA": "1", "transB": "1"}),
    ("Flatten", {"axis": 3}, {"axis": "3"}),
    ("Softmax", {"axis": -2}, {"axis": "-2"}),
    ("LayerNormalization", {"axis": -2, "epsilon": 0.5}, {"axis": "-2", "epsilon": "0.5"}),
    ("Transpose", {"perm": [2, 0, 1]}, {"perm": "2,0,1"}),
    ("Reshape", {"allowzero": 1}, {"allowzero": "1"}),
    ("Gather", {"axis": -1}, {"axis": "-1"}),
    ("Cast", {"to": 1}, {"to": "1"}),
    ("Concat", {"axis": -3}, {"axis": "-3"}),
    ("ReduceMean", {"axes": [0, -1], "keep_dims": 1}, {"axes": "0,-1", "keep_dims": "1"}),
    ("ConstantOfShape", {"value": 3}, {"value": "3", "dtype": "int32"}),
    ("ConstantOfShape", {"value": -1.5}, {"value": "-1.5", "dtype": "float"}),
])
def test_loader_decodes_attrs(op_type, attrs, expect):
    got = _decoded(_one_op(op_type, attrs, 2 if op_type in ("Gemm", "Reshape", "Gather", "Concat") else 1))
    for k, v in expect.items():
        assert got.get(k) == v, (op_type, k, got)


def _schema_default(table, field):
    d = TABLES[table][field]["default"]
    return {"false": "0", "true": "1", "0.0": "0"}.get(d, d)


@pytest.mark.parametrize("op_type,table,expect", [
    # every field absent -> the schema default, through the reference's ReadOp
    ("Conv", "ConvAttrs", {"auto_pad": "same",                   # AutoPad::Same -> Padding::Same
                           "groups": _schema_default("ConvAttrs", "groups"),
                           "strides": "1,1", "dilations": "1,1"}),  # vec_from_attr(.., &[1, 1])
    ("Gemm", "GemmAttrs", {"alpha": _schema_default("GemmAttrs", "alpha"),
                           "beta": _schema_default("GemmAttrs", "beta"),
                           "transA": _schema_default("GemmAttrs", "transpose_a"),
                           "transB": _schema_default("GemmAttrs", "transpose_b")}),
    ("BatchNormalization", "BatchNormalizationAttrs",
     {"epsilon": _schema_default("BatchNormalizationAttrs", "epsilon")}),
    ("Flatten", "FlattenAttrs", {"axis": _schema_default("FlattenAttrs", "axis")}),
    ("Softmax", "SoftmaxAttrs", {"axis": _schema_default("SoftmaxAttrs", "axis")}),
    ("LayerNormalization", "LayerNormalizationAttrs",
     {"axis": _schema_default("LayerNormalizationAttrs", "axis"),
      "epsilon": _schema_default("LayerNormalizationAttrs", "epsilon")}),
    ("Gather", "GatherAttrs", {"axis": _schema_default("GatherAttrs", "axis")}),
    ("Concat", "ConcatAttrs", {"axis": _schema_default("ConcatAttrs", "axis")}),
    ("Reshape", "ReshapeAttrs", {"allowzero": _schema_default("ReshapeAttrs", "allow_zero")}),
    ("Cast", "CastAttrs", {"to": "0"}),                          # DataType::Int32
    ("ReduceMean", "ReduceMeanAttrs", {"keep_dims": _schema_default("ReduceMeanAttrs", "keep_dims")}),
    ("ConstantOfShape", "ConstantOfShapeAttrs", {"value": "0", "dtype": "int32"}),  # Scalar::NONE -> Int(0)
])
def test_loader_schema_defaults(monkeypatch, op_type, table, expect):
    orig = rten_file._op_attrs

    def empty(t, a):
        at, tab = orig(t, a)
        return (at, rten_file.Table([])) if t == op_type else (at, tab)

    monkeypatch.setattr(rten_file, "_op_attrs", empty)
    got = _decoded(_one_op(op_type, {}, 2 if op_type in ("Gemm", "Reshape", "Gather", "Concat") else 1))
    for k, v in expect.items():
        assert got.get(k) == v, (op_type, k, got)
    if op_type == "ReduceMean":
        assert "axes" not in got
