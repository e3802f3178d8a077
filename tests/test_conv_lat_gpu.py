"""Latency GEMM convs (csrc/gemm_lat.hip: one wave per 16x16 output tile and
KC block, the K blocks folded in order by the last to arrive) against the CPU
oracle.  Same contract as the DMA kernel: the reference's conv = im2col GEMM
with KC = 256 blocks, each an fma chain from +0, folded in K order after the
bias (src/gemm.rs:733-1050, src/ops/conv.rs:243-270), then the fused
Add / Relu / Clip.  Bar: bit-exact, for every variant (RTENHIP_LAT forces
one), at K below, at and far above one KC block, K not a multiple of the
kernel's 16-deep groups, M not a multiple of 16, N tails, strided and grouped
convs, no bias, fused residuals, and a conv writing a zero-bordered output
that the next (padded) conv reads.
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


# (N, C, H, W, O, kh, stride, pads, groups, tail, bias)
CASES = [
    (1, 64, 14, 14, 64, 3, 1, [1, 1, 1, 1], 1, "relu", True),        # K = 576: 3 KC blocks
    (1, 64, 28, 28, 256, 1, 1, [0, 0, 0, 0], 1, "add_relu", True),    # pointwise K = 64, residual
    (1, 256, 28, 28, 128, 1, 2, [0, 0, 0, 0], 1, "none", True),       # strided 1x1, K = 256
    (1, 3, 30, 30, 64, 7, 2, [3, 3, 3, 3], 1, "relu", True),          # stem: K = 147
    (2, 20, 9, 11, 40, 3, 1, [1, 1, 1, 1], 2, "clip", False),         # groups, M = 20, no bias
    (1, 1030, 7, 7, 24, 1, 1, [0, 0, 0, 0], 1, "none", True),         # K = 1030: ragged last block
    (1, 512, 7, 7, 512, 3, 1, [1, 1, 1, 1], 1, "relu", True),         # K = 4608: 18 blocks, N = 49
    (1, 128, 7, 7, 2048, 1, 1, [0, 0, 0, 0], 1, "add_relu", True),    # M = 2048
    # 3x3 windows (offsets formed in the kernel, no K table):
    (1, 37, 12, 10, 24, 3, 2, [1, 1, 1, 1], 1, "relu", True),         # strided, K = 333 ragged
    (1, 30, 13, 11, 20, 3, 1, [2, 2, 2, 2], 1, "none", True, 2),      # dilation 2, K = 270
    (1, 3, 9, 9, 16, 3, 1, [0, 1, 2, 0], 1, "none", False),           # K = 27, asymmetric pads
]


def _case_id(c):
    return "x".join(map(str, c[:6])) + f"s{c[6]}g{c[8]}-{c[9]}" + (f"d{c[11]}" if len(c) > 11 else "")


@pytest.mark.parametrize("mode", ["41", "22", "12", "91", "92", "71", "72", "74", "85", "86", "61", "62", "63", "66"])
@pytest.mark.parametrize("case", CASES, ids=_case_id)
def test_lat_conv_bitexact(rh, monkeypatch, mode, case):
    import torch
    import graph_runner
    from rten_hip.graph import ModelSpec

    N, C, H, W, O, kh, st, pads, groups, tail, bias = case[:11]
    dil = case[11] if len(case) > 11 else 1
    monkeypatch.setenv("RTENHIP_LAT", mode)
    rng = np.random.default_rng(C * 31 + O + kh + groups)
    m = ModelSpec("lat")
    x = m.value("x")
    m.inputs = ["x"]
    ins = {"x": rng.uniform(-1, 1, (N, C, H, W)).astype(np.float32)}
    w = m.const("w", rng.uniform(-0.5, 0.5, (O, C // groups, kh, kh)).astype(np.float32))
    args = [x, w]
    if bias:
        args.append(m.const("b", rng.uniform(-0.2, 0.2, (O,)).astype(np.float32)))
    y = m.op("Conv", args, {"pads": pads, "strides": [st, st], "groups": groups, "dilations": [dil, dil]})
    if tail == "add_relu":
        oh = (H + pads[0] + pads[2] - dil * (kh - 1) - 1) // st + 1
        ow = (W + pads[1] + pads[3] - dil * (kh - 1) - 1) // st + 1
        r = m.value("r")
        m.inputs.append("r")
        ins["r"] = rng.uniform(-1, 1, (N, O, oh, ow)).astype(np.float32)
        y = m.op("Relu", [m.op("Add", [y, r])])
    elif tail == "relu":
        y = m.op("Relu", [y])
    elif tail == "clip":
        y = m.op("Clip", [y, m.const("lo", np.array(0, np.float32)), m.const("hi", np.array(6, np.float32))])
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
    slab_ok = (N == 1 and groups == 1 and kh in (1, 3) and
               min(C, 30 if kh == 3 else 256) * (H + pads[0] + pads[2]) * (W + pads[1] + pads[3]) + 8 <= 13312)
    if not (mode[0] in "78" and kh not in (1, 3)) and not (mode[0] == "6" and not slab_ok):
        # (the LDS variants take 1x1 / 3x3 windows, the slab variants one image whose planes fit)
        assert f"cfg=lat{mode}" in g.timing_report()


@pytest.mark.parametrize("mode", ["41", "12", "86", "62"])
def test_lat_conv_chain_padded_handoff(rh, monkeypatch, mode):
    """1x1 -> Relu -> 3x3 (pad 1) -> Add -> Relu, both convs on the latency
    kernel: the first writes straight into the second's zero-bordered input."""
    import torch
    import graph_runner
    from rten_hip.graph import ModelSpec

    monkeypatch.setenv("RTENHIP_LAT", mode)
    rng = np.random.default_rng(77)
    m = ModelSpec("chain")
    x = m.value("x")
    m.inputs = ["x"]
    w1 = m.const("w1", rng.uniform(-0.3, 0.3, (48, 96, 1, 1)).astype(np.float32))
    b1 = m.const("b1", rng.uniform(-0.2, 0.2, (48,)).astype(np.float32))
    w2 = m.const("w2", rng.uniform(-0.2, 0.2, (96, 48, 3, 3)).astype(np.float32))
    b2 = m.const("b2", rng.uniform(-0.2, 0.2, (96,)).astype(np.float32))
    h = m.op("Relu", [m.op("Conv", [x, w1, b1], {"pads": [0, 0, 0, 0], "strides": [1, 1]})])
    y = m.op("Relu", [m.op("Add", [m.op("Conv", [h, w2, b2], {"pads": [1, 1, 1, 1], "strides": [1, 1]}), x])])
    m.outputs = [y]
    ins = {"x": rng.uniform(-1, 1, (1, 96, 14, 14)).astype(np.float32)}
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
    # (the slab variant takes the 3x3 conv only: the 1x1's 96 planes of 196 do not fit)
    assert g.timing_report().count(f"cfg=lat{mode}") == (1 if mode == "62" else 2)


def test_resnet50_batch1_all_latency_convs(rh, monkeypatch):
    """Whole ResNet-50 at batch 1 with every DMA-eligible conv forced onto the
    latency kernel: bit-exact against the oracle (eager and replayed)."""
    import torch
    import graph_runner
    from rten_hip import models

    monkeypatch.setenv("RTENHIP_LAT", "41")
    spec = models.resnet50()
    x = np.random.default_rng(11).random((1, 3, 224, 224), dtype=np.float32)
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
    assert g.timing_report().count("cfg=lat41") >= 50




@pytest.mark.parametrize("mode", ["71", "72", "74", "85", "86", "61", "62", "63", "66", "91", "92", "22", "12", "11", "21", "42"])
def test_resnet50_batch1_forced_variant(rh, monkeypatch, mode):
    """ResNet-50 at batch 1 with one latency-GEMM variant forced on every conv
    it takes (the tuner may pick any of them per layer): oracle bits."""
    import torch
    import graph_runner
    from rten_hip import models

    monkeypatch.setenv("RTENHIP_LAT", mode)
    spec = models.resnet50()
    x = np.random.default_rng(12).random((1, 3, 224, 224), dtype=np.float32)
    exp = graph_runner.run(spec, {spec.inputs[0]: x})[spec.outputs[0]]
    g = spec.to_graph()
    xd = torch.from_numpy(x).cuda()
    out = None
    for _ in range(3):
        out = g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
        torch.cuda.synchronize()
        assert _bits_equal(out[0].cpu().numpy(), exp)


@pytest.mark.parametrize("pair", ["72/72", "74/74", "71/71", "72/74", "74/72", "0"])
def test_resnet50_batch1_conv1_downsample_pair(rh, monkeypatch, pair):
    """ResNet-50 at batch 1 with each bottleneck's conv1 and downsample in one
    gemm_lat2_pair_kernel launch (RTENHIP_LAT_PAIR="v0/v1" forces that
    variant pair; "0" plans none): the oracle's bits, eager and replayed, and
    the downsample ops run inside their conv1's launch."""
    import torch
    import graph_runner
    from rten_hip import models

    monkeypatch.setenv("RTENHIP_LAT_PAIR", pair)
    spec = models.resnet50()
    x = np.random.default_rng(13).random((1, 3, 224, 224), dtype=np.float32)
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
    rep = g.timing_report()
    if pair == "0":
        assert "lat_pair" not in rep, rep
    else:
        v0, v1 = pair.split("/")
        # (a downsample the tuner put on a non-latency kernel is not paired)
        assert rep.count(f"cfg=lat{v0}/lat{v1}") >= 1, rep
        assert rep.count("(in its conv1's latency pair launch)") == rep.count(f"cfg=lat{v0}/lat{v1}"), rep
