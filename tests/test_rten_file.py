""".rten V2 files: the writer (rten-convert's layout) and the C++ loader
(Model::load, src/model.rs:265-522; Header::from_buf, src/header.rs:84-131).

CPU tests parse files on the host only (rtenhip_model_describe: no device);
GPU tests load a file into a device graph and check its outputs bit-exactly
against the oracle running the ModelSpec the file was written from.

Parity note: the reference ships no .rten files and cannot be built here (no
Rust toolchain), so no reference-written file is available: the format is
pinned by src/schema.fbs and src/header.rs (field slots, union ids and
defaults transcribed from them), and the error texts by model.rs:677-689,
header.rs:150-158 and op_registry.rs:211-220.
"""
import struct

import numpy as np
import pytest

from rten_hip import OpError, models, rten_file
from rten_hip.graph import ModelSpec


def _model_bytes(spec, **kw):
    return rten_file.to_rten_bytes(spec, **kw)


def _tiny_spec():
    m = ModelSpec("tiny")
    x = m.value("x")
    m.inputs = ["x"]
    w = m.const("w", np.arange(2 * 3 * 3 * 3, dtype=np.float32).reshape(2, 3, 3, 3) / 10)
    b = m.const("b", np.array([0.5, -0.5], np.float32))
    y = m.op("Conv", [x, w, b], {"pads": [1, 1, 1, 1], "strides": [1, 1], "groups": 1}, name="conv")
    y = m.op("Relu", [y], name="relu")
    shape = m.const("shape", np.array([0, -1], np.float32))
    y = m.op("Reshape", [y, shape], name="reshape")
    m.outputs = [y]
    return m


def _parse(desc):
    lines = desc.strip().splitlines()
    nodes = {}
    for ln in lines[2:]:
        idx, kind, rest = ln.split(" ", 2)
        nodes[int(idx)] = (kind, rest)
    return lines[0], lines[1], nodes


def test_header_layout():
    b = _model_bytes(_tiny_spec())
    magic, version, moff, mlen, toff = struct.unpack_from("<4sIQQQ", b, 0)
    assert magic == b"RTEN" and version == 2
    assert moff == 32 and moff + mlen <= len(b)
    assert toff % 64 == 0 and toff >= moff + mlen


def test_describe_round_trip_tiny():
    desc = rten_file.describe_model(_model_bytes(_tiny_spec()))
    ins, outs, nodes = _parse(desc)
    assert ins == "inputs 0"
    kinds = [nodes[i][0] for i in sorted(nodes)]
    assert kinds == ["value", "const", "const", "value", "op", "value", "op", "const", "value", "op"]
    conv = nodes[4][1]
    assert conv.startswith("conv Conv in=0,1,2 out=3")
    assert "pads=1,1,1,1" in conv and "strides=1,1" in conv and "groups=1" in conv
    assert "dilations=1,1" in conv
    assert "allowzero=0" in nodes[9][1]
    # int32 shape constant (Reshape input) and an inline float constant
    assert nodes[7][1].startswith("shape 2 i32 sum=-1")
    assert nodes[2][1].startswith("b 2 sum=0")


@pytest.mark.parametrize("name", ["resnet50", "mobilenet_v2", "bert_encoder", "bert_onnx"])
def test_describe_round_trip_models(name):
    if name == "bert_encoder":
        spec = models.bert_encoder(layers=2, seq=32)
    elif name == "bert_onnx":  # ONNX primitives and the shape subgraph, before RTen's optimizer
        spec = models.bert_encoder(layers=2, seq=32, embeddings=True, vocab=64, unfused=True)
    else:
        spec = getattr(models, name)()
    desc = rten_file.describe_model(_model_bytes(spec))
    _, _, nodes = _parse(desc)
    assert len(nodes) == len(spec.nodes)
    for i, n in enumerate(spec.nodes):
        kind, rest = nodes[i]
        if n.kind == "op":
            assert kind == "op"
            assert rest.split(" ")[1] == n.op_type, (i, rest)
        elif n.kind == "const":
            assert kind == "const"
            s = float(rest.rsplit("sum=", 1)[1])
            exp = float(np.asarray(n.data, np.float64).sum())
            assert abs(s - exp) <= 1e-6 * max(1.0, np.abs(np.asarray(n.data, np.float64)).sum())
            shape = rest.split(" ")[1]
            assert shape == "x".join(str(d) for d in np.asarray(n.data).shape)
        else:
            assert kind == "value"


def test_export_op_attrs_round_trip():
    """Attributes of the ops an ONNX export adds (op_registry.rs: ReduceMean's
    reduce_axes, Concat's axis, ConstantOfShape's Scalar union) survive the
    writer and the loader."""
    m = ModelSpec("export_ops")
    x = m.value("x")
    m.inputs = ["x"]
    r = m.op("ReduceMean", [x], {"axes": [-1, 1], "keep_dims": 1}, name="rm")
    r0 = m.op("ReduceMean", [x], {"keep_dims": 0}, name="rm_all")
    c = m.op("Concat", [r, r], {"axis": -2}, name="cat")
    shp = m.const("shp", np.array([2, 3], np.int32))
    k1 = m.op("ConstantOfShape", [shp], {"value": 7}, name="cos_i")
    k2 = m.op("ConstantOfShape", [shp], {"value": 0.25}, name="cos_f")
    m.outputs = [c, k1, k2, r0]
    _, _, nodes = _parse(rten_file.describe_model(_model_bytes(m)))
    ops = {rest.split(" ")[0]: rest for kind, rest in nodes.values() if kind == "op"}
    assert "axes=-1,1" in ops["rm"] and "keep_dims=1" in ops["rm"]
    assert "axes=" not in ops["rm_all"] and "keep_dims=0" in ops["rm_all"]
    assert "axis=-2" in ops["cat"]
    assert "value=7" in ops["cos_i"] and "dtype=int32" in ops["cos_i"]
    assert "value=0.25" in ops["cos_f"] and "dtype=float" in ops["cos_f"]


def test_norm_op_attrs_round_trip():
    """LogSoftmax reads SoftmaxAttrs and InstanceNormalization reads
    BatchNormalizationAttrs (op_registry.rs:556-564, 587)."""
    m = ModelSpec("norm_ops")
    x = m.value("x")
    m.inputs = ["x"]
    sc = m.const("sc", np.ones(4, np.float32))
    bi = m.const("bi", np.zeros(4, np.float32))
    h = m.op("InstanceNormalization", [x, sc, bi], {"epsilon": 0.5}, name="inorm")
    m.outputs = [m.op("LogSoftmax", [h], {"axis": 1}, name="lsm")]
    _, _, nodes = _parse(rten_file.describe_model(_model_bytes(m)))
    ops = {rest.split(" ")[0]: rest for kind, rest in nodes.values() if kind == "op"}
    assert "InstanceNormalization" in ops["inorm"] and "epsilon=0.5" in ops["inorm"]
    assert "LogSoftmax" in ops["lsm"] and "axis=1" in ops["lsm"]


def test_inline_and_external_constants_agree():
    spec = _tiny_spec()
    a = rten_file.describe_model(_model_bytes(spec, inline_max=0))
    b = rten_file.describe_model(_model_bytes(spec, inline_max=10 ** 9))
    assert a == b


def test_v2_header_errors():
    good = bytearray(_model_bytes(_tiny_spec()))
    bad = bytearray(good)
    struct.pack_into("<I", bad, 4, 3)
    with pytest.raises(OpError, match="invalid header: unsupported file version"):
        rten_file.describe_model(bytes(bad))
    with pytest.raises(OpError, match="invalid header: header is too short"):
        rten_file.describe_model(bytes(good[:20]))
    bad = bytearray(good)
    struct.pack_into("<Q", bad, 8, len(good) + 1)
    with pytest.raises(OpError, match="invalid header: segment offset is invalid"):
        rten_file.describe_model(bytes(bad))
    bad = bytearray(good)
    struct.pack_into("<Q", bad, 16, len(good))
    with pytest.raises(OpError, match="invalid header: segment length is invalid"):
        rten_file.describe_model(bytes(bad))


def test_v1_file_without_header():
    """No "RTEN" magic: the whole buffer is the FlatBuffers model (V1)."""
    b = _model_bytes(_tiny_spec(), inline_max=10 ** 9)
    moff, mlen = struct.unpack_from("<QQ", b, 8)
    v1 = b[moff:moff + mlen]
    assert rten_file.describe_model(v1) == rten_file.describe_model(b)
    # ... but an external constant needs the tensor data section
    b = _model_bytes(_tiny_spec(), inline_max=0)
    moff, mlen = struct.unpack_from("<QQ", b, 8)
    v1 = b[moff:moff + mlen]
    with pytest.raises(OpError, match="graph error: tensor data section missing"):
        rten_file.describe_model(v1)


def test_truncated_model_is_a_parse_error():
    b = _model_bytes(_tiny_spec())
    with pytest.raises(OpError, match="parse error"):
        rten_file.describe_model(b[32:72])


def test_unsupported_operator_error():
    m = ModelSpec("topk")
    x = m.value("x")
    m.inputs = ["x"]
    m.outputs = [m.op("TopK", [x, x], name="topk")]
    with pytest.raises(OpError, match="operator error: operator TopK is not supported or not enabled"):
        rten_file.describe_model(_model_bytes(m))


@pytest.mark.parametrize("mask_op", ["mul", "where"])
def test_bert_embeddings_file_round_trip(mask_op):
    """The embedding / mask subgraph (Gather, Unsqueeze, Cast, Where) and its
    int32 constants survive the .rten round trip: CastAttrs / GatherAttrs are
    decoded (op_registry.rs:421-428, 486), Int32 constants stay int32
    (model.rs:504-520), inline and in the tensor segment alike."""
    spec = models.bert_encoder(layers=1, seq=16, embeddings=True, vocab=50, mask_op=mask_op)
    for inline_max in (0, 10 ** 9):
        desc = rten_file.describe_model(_model_bytes(spec, inline_max=inline_max))
        lines = desc.splitlines()
        assert any(" const emb.position_ids 1x16 i32 sum=120" in l for l in lines)
        assert any(" const mask.axes2 1 i32 sum=2" in l for l in lines)
        assert any("Gather" in l and "axis=0" in l for l in lines)
        if mask_op == "mul":
            assert any(" Cast " in l and "to=1" in l for l in lines)
        else:
            assert any(" Where " in l for l in lines)


def test_wrong_attrs_union_error(monkeypatch):
    m = ModelSpec("conv")
    x = m.value("x")
    m.inputs = ["x"]
    w = m.const("w", np.zeros((1, 1, 1, 1), np.float32))
    m.outputs = [m.op("Conv", [x, w], name="conv")]
    assert "Conv" in rten_file.describe_model(_model_bytes(m))
    # A Conv whose attrs union holds GemmAttrs (op.attrs_as_conv_attrs() is None).
    monkeypatch.setattr(rten_file, "_op_attrs", lambda t, a: (rten_file.ATTRS_GEMM, rten_file.Table([])))
    with pytest.raises(OpError, match="operator error: invalid attributes for operator"):
        rten_file.describe_model(_model_bytes(m))


def test_schema_version_checked():
    b = bytearray(_model_bytes(_tiny_spec()))
    moff = 32
    root = struct.unpack_from("<I", b, moff)[0] + moff
    vt = root - struct.unpack_from("<i", b, root)[0]
    field = struct.unpack_from("<H", b, vt + 4)[0]
    struct.pack_into("<i", b, root + field, 2)
    with pytest.raises(OpError, match="unsupported schema version"):
        rten_file.describe_model(bytes(b))


# --------------------------------------------------------------------------
# Load into a device graph and run (GPU)
# --------------------------------------------------------------------------

def _bits_equal(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.fixture(scope="module")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import rten_hip

    rten_hip.default_context()
    return torch


@pytest.mark.gpu
@pytest.mark.parametrize("optimize", [True, False])
def test_load_resnet50_file_bitexact(gpu, tmp_path, optimize):
    import graph_runner

    spec = models.resnet50()
    path = tmp_path / "resnet50.rten"
    rten_file.write_rten(spec, str(path))
    g = rten_file.load_model(str(path), optimize=optimize)
    x = np.random.default_rng(5).random((2, 3, 224, 224), dtype=np.float32)
    exp = graph_runner.run(spec, {"input": x})[spec.outputs[0]]
    xd = gpu.from_numpy(x).cuda()
    out = None
    for _ in range(2):
        out = g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
        gpu.cuda.synchronize()
        assert _bits_equal(out[0].cpu().numpy(), exp)


@pytest.mark.gpu
def test_load_bert_file_bitexact(gpu):
    import graph_runner

    spec = models.bert_encoder(layers=2, seq=64)
    g = rten_file.load_model(rten_file.to_rten_bytes(spec))
    rng = np.random.default_rng(6)
    x = rng.random((4, 64, 768), dtype=np.float32) - np.float32(0.5)
    mask = np.zeros((4, 1, 1, 64), np.float32)
    mask[-1, :, :, 48:] = -10000.0
    exp = graph_runner.run(spec, {"hidden_states": x, "attention_mask": mask})[spec.outputs[0]]
    out = g.run({g.input_ids[0]: gpu.from_numpy(x).cuda(), g.input_ids[1]: gpu.from_numpy(mask).cuda()},
                g.output_ids)
    gpu.cuda.synchronize()
    assert _bits_equal(out[0].cpu().numpy(), exp)


@pytest.mark.gpu
def test_load_errors_on_device(gpu):
    m = ModelSpec("topk")
    x = m.value("x")
    m.inputs = ["x"]
    m.outputs = [m.op("TopK", [x, x], name="topk")]
    with pytest.raises(OpError, match="operator error: operator TopK"):
        rten_file.load_model(rten_file.to_rten_bytes(m))


@pytest.mark.gpu
def test_load_bert_embeddings_file_bitexact(gpu):
    """A .rten BERT with the embedding Gathers and the int32 mask path runs on
    the device from int32 inputs, bit-exact against the oracle."""
    import graph_runner

    spec = models.bert_encoder(layers=2, seq=32, embeddings=True, vocab=300)
    g = rten_file.load_model(rten_file.to_rten_bytes(spec, inline_max=0))
    rng = np.random.default_rng(8)
    ids = rng.integers(0, 300, (3, 32)).astype(np.int32)
    tt = rng.integers(0, 2, (3, 32)).astype(np.int32)
    am = np.ones((3, 32), np.int32)
    am[1, 20:] = 0
    exp = graph_runner.run(spec, {"input_ids": ids, "token_type_ids": tt, "attention_mask": am})[spec.outputs[0]]
    feed = {g.input_ids[0]: gpu.from_numpy(ids).cuda(), g.input_ids[1]: gpu.from_numpy(tt).cuda(),
            g.input_ids[2]: gpu.from_numpy(am).cuda()}
    out = None
    for _ in range(3):  # eager, capture, replay
        out = g.run(feed, g.output_ids, out=out)
        gpu.cuda.synchronize()
        assert _bits_equal(out[0].cpu().numpy(), exp)


@pytest.mark.parametrize("inline_max", [0, 10 ** 9])
def test_constant_shape_overflow_is_a_load_error(monkeypatch, inline_max):
    """Dims whose product overflows 64 bits are rejected as a load error
    (checked count * 4), not a wrapped bounds check or a C++ exception."""
    m = ModelSpec("huge")
    x = m.value("x")
    m.inputs = ["x"]
    big = m.const("big", np.zeros((7, 7), np.float32))
    m.outputs = [m.op("Add", [x, big], name="add")]
    orig = rten_file._u32v
    monkeypatch.setattr(rten_file, "_u32v",
                        lambda v: orig([0xFFFFFFFF] * 3) if tuple(v) == (7, 7) else orig(v))
    with pytest.raises(OpError, match="constant shape is too large"):
        rten_file.describe_model(_model_bytes(m, inline_max=inline_max))
