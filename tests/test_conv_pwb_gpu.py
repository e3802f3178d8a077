"""B-stationary pointwise GEMM (csrc/gemm_pwb.hip, latency-GEMM variants
61 / 62 / 64: a workgroup keeps its 64 columns' B panel in LDS and walks 1, 2
or 4 chunks of 64 output rows) against the CPU oracle.  Same contract as every
conv configuration: the reference's conv = im2col GEMM with KC = 256 blocks,
each an fma chain from +0, then the bias and the fused tail
(src/gemm.rs:733-1050, src/ops/conv.rs:243-270).  Bar: bit-exact, for each
variant, at K = 256, K ragged against the 16-deep groups, M not a multiple
of 16 or 64, column tiles crossing image boundaries and a ragged last tile,
strided 1x1, no bias, fused residual / Clip / BatchNormalization, a conv
writing a zero-bordered output that a padded 3x3 conv reads, and whole
ResNet-50 / MobileNetV2 forwards with the variant forced where it applies.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rh():
    import torch
    import rten_hip
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    return rten_hip


def _bits_equal(a, b):
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


# (N, C, H, W, O, stride, tail, bias)
CASES = [
    (4, 64, 14, 14, 256, 1, "add_relu", True),   # N*P = 784: 12 full column tiles + a tail
    (2, 256, 28, 28, 64, 1, "relu", True),       # K = 256, one row chunk
    (3, 37, 9, 7, 100, 1, "clip", False),        # K = 37 ragged, M = 100, P = 63
    (2, 128, 14, 14, 96, 2, "none", True),       # strided 1x1 (downsample-shaped)
    (1, 24, 56, 56, 144, 1, "clip", True),       # MobileNetV2 expand
    (8, 160, 7, 7, 960, 1, "clip", True),        # M = 960: 15 chunks, P = 49
    (2, 96, 10, 10, 40, 1, "bn_relu", False),    # Conv -> BatchNormalization -> Relu
]


def _case_id(c):
    return "x".join(map(str, c[:5])) + f"s{c[5]}-{c[6]}"


@pytest.mark.parametrize("mode", ["61", "62", "64"])
@pytest.mark.parametrize("case", CASES, ids=_case_id)
def test_pwb_conv_bitexact(rh, monkeypatch, mode, case):
    import torch
    import graph_runner
    from rten_hip.graph import ModelSpec

    N, C, H, W, O, st, tail, bias = case
    monkeypatch.setenv("RTENHIP_LAT", mode)
    rng = np.random.default_rng(C * 17 + O + N)
    m = ModelSpec("pwb")
    x = m.value("x")
    m.inputs = ["x"]
    ins = {"x": rng.uniform(-1, 1, (N, C, H, W)).astype(np.float32)}
    args = [x, m.const("w", rng.uniform(-0.5, 0.5, (O, C, 1, 1)).astype(np.float32))]
    if bias:
        args.append(m.const("b", rng.uniform(-0.2, 0.2, (O,)).astype(np.float32)))
    y = m.op("Conv", args, {"pads": [0, 0, 0, 0], "strides": [st, st]})
    oh, ow = (H - 1) // st + 1, (W - 1) // st + 1
    if tail == "add_relu":
        r = m.value("r")
        m.inputs.append("r")
        ins["r"] = rng.uniform(-1, 1, (N, O, oh, ow)).astype(np.float32)
        y = m.op("Relu", [m.op("Add", [y, r])])
    elif tail == "relu":
        y = m.op("Relu", [y])
    elif tail == "clip":
        y = m.op("Clip", [y, m.const("lo", np.array(0, np.float32)), m.const("hi", np.array(6, np.float32))])
    elif tail == "bn_relu":
        bn = [m.const(nm, v.astype(np.float32)) for nm, v in (
            ("scale", rng.uniform(0.5, 1.5, O)), ("beta", rng.uniform(-0.2, 0.2, O)),
            ("mean", rng.uniform(-0.3, 0.3, O)), ("var", rng.uniform(0.5, 2.0, O)))]
        y = m.op("Relu", [m.op("BatchNormalization", [y] + bn, {"epsilon": 1e-5})])
    m.outputs = [y]
    exp = graph_runner.run(m, ins)[y]
    g = m.to_graph()
    dev = {g.input_ids[i]: torch.from_numpy(ins[n]).cuda() for i, n in enumerate(m.inputs)}
    out = None
    for _ in range(3):  # eager, capture, replay
        out = g.run(dev, g.output_ids, out=out)
        torch.cuda.synchronize()
        o = out[0].cpu().numpy()
        assert _bits_equal(o, exp), np.abs(o - exp).max()
    g.set_timing(True)
    g.run(dev, g.output_ids, out=out)
    torch.cuda.synchronize()
    assert f"cfg=lat{mode}" in g.timing_report()


@pytest.mark.parametrize("mode", ["61", "64"])
def test_pwb_padded_handoff(rh, monkeypatch, mode):
    """1x1 (B-stationary) -> Relu -> 3x3 pad 1 -> Add -> Relu at batch 4: the
    pointwise conv writes straight into the 3x3 conv's zero-bordered input."""
    import torch
    import graph_runner
    from rten_hip.graph import ModelSpec

    monkeypatch.setenv("RTENHIP_LAT", mode)
    rng = np.random.default_rng(78)
    m = ModelSpec("pwbchain")
    x = m.value("x")
    m.inputs = ["x"]
    w1 = m.const("w1", rng.uniform(-0.3, 0.3, (48, 96, 1, 1)).astype(np.float32))
    b1 = m.const("b1", rng.uniform(-0.2, 0.2, (48,)).astype(np.float32))
    w2 = m.const("w2", rng.uniform(-0.2, 0.2, (96, 48, 3, 3)).astype(np.float32))
    b2 = m.const("b2", rng.uniform(-0.2, 0.2, (96,)).astype(np.float32))
    h = m.op("Relu", [m.op("Conv", [x, w1, b1], {"pads": [0, 0, 0, 0], "strides": [1, 1]})])
    y = m.op("Relu", [m.op("Add", [m.op("Conv", [h, w2, b2], {"pads": [1, 1, 1, 1], "strides": [1, 1]}), x])])
    m.outputs = [y]
    ins = {"x": rng.uniform(-1, 1, (4, 96, 14, 14)).astype(np.float32)}
    exp = graph_runner.run(m, ins)[y]
    g = m.to_graph()
    dev = {g.input_ids[0]: torch.from_numpy(ins["x"]).cuda()}
    out = None
    for _ in range(3):
        out = g.run(dev, g.output_ids, out=out)
        torch.cuda.synchronize()
        assert _bits_equal(out[0].cpu().numpy(), exp)
    g.set_timing(True)
    g.run(dev, g.output_ids, out=out)
    torch.cuda.synchronize()
    assert g.timing_report().count(f"cfg=lat{mode}") == 1


@pytest.mark.parametrize("model,mode,batch", [("resnet50", "62", 4), ("resnet50_bn", "64", 2),
                                              ("mobilenet_v2", "61", 4)])
def test_model_forced_pwb(rh, monkeypatch, model, mode, batch):
    """Whole forwards with every eligible 1x1 conv on the B-stationary kernel
    (the rest tuned as usual): oracle bits, eager and replayed."""
    import torch
    import graph_runner
    from rten_hip import models

    monkeypatch.setenv("RTENHIP_LAT", mode)
    spec = models.resnet50(unfolded_bn=True) if model == "resnet50_bn" else getattr(models, model)()
    x = np.random.default_rng(13).random((batch, 3, 224, 224), dtype=np.float32)
    exp = graph_runner.run(spec, {spec.inputs[0]: x})[spec.outputs[0]]
    g = spec.to_graph()
    xd = torch.from_numpy(x).cuda()
    out = None
    for _ in range(3):
        out = g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
        torch.cuda.synchronize()
        assert _bits_equal(out[0].cpu().numpy(), exp)
    g.set_timing(True)
    g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
    torch.cuda.synchronize()
    assert g.timing_report().count(f"cfg=lat{mode}") >= 10
