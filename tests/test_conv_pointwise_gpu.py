"""Pointwise convs on the VALU kernel (csrc/conv_pointwise.hip) against the CPU
oracle: conv_2d_pointwise (src/ops/conv.rs:24-68) = per-image
gemm_uninit_bias with one KC block (K <= 256), then the fused Add / Relu /
Clip in the graph.  Bar: bit-exact, for every kernel variant (channel-chunk
width, streamed or register-resident x column) the tuner
can pick (RTENHIP_PW_VALU forces one), including partial chunks (M not a
multiple of it), K not a multiple of the kernel's 8-deep load group, K = 1,
no bias, and a fused residual.
"""
import re

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rh():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import rten_hip

    rten_hip.default_context()
    return rten_hip


def _bits_equal(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


# (N, C=K, H, W, O, bias, tail): tail in {"clip", "relu", "add_relu", "add", "none"}
CASES = [
    (2, 20, 12, 12, 24, True, "clip"),
    (3, 16, 28, 28, 96, True, "relu"),
    (2, 144, 8, 8, 24, True, "add"),
    (2, 32, 10, 10, 40, False, "add_relu"),
    (1, 256, 4, 4, 40, True, "none"),
    (2, 1, 8, 8, 16, True, "none"),
    (2, 13, 6, 6, 7, True, "clip"),
]


@pytest.mark.parametrize("mode", ["8", "16", "32", "108", "116", "208", "216"])
@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c[:5])) + f"-{c[6]}")
def test_pointwise_valu_bitexact(rh, monkeypatch, mode, case):
    import torch
    import graph_runner
    from rten_hip.graph import ModelSpec

    N, C, H, W, O, has_bias, tail = case
    if int(mode) >= 100 and C > int(mode) // 100 * 16:
        pytest.skip("x-resident variant needs K <= KX")
    monkeypatch.setenv("RTENHIP_PW_VALU", mode)
    rng = np.random.default_rng(C * 131 + O)
    m = ModelSpec("pw")
    x = m.value("x")
    m.inputs = ["x"]
    ins = {"x": rng.uniform(-1, 1, (N, C, H, W)).astype(np.float32)}
    w = m.const("w", rng.uniform(-0.5, 0.5, (O, C, 1, 1)).astype(np.float32))
    args = [x, w]
    if has_bias:
        args.append(m.const("b", rng.uniform(-0.2, 0.2, (O,)).astype(np.float32)))
    y = m.op("Conv", args, {"pads": [0, 0, 0, 0], "strides": [1, 1]})
    if tail.startswith("add"):
        r = m.value("r")
        m.inputs.append("r")
        ins["r"] = rng.uniform(-1, 1, (N, O, H, W)).astype(np.float32)
        y = m.op("Add", [y, r])
    if tail.endswith("relu"):
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
    assert f"cfg=valu{mode}" in g.timing_report()


@pytest.mark.parametrize("mode", ["16", "-1"])
def test_mobilenet_v2_pointwise_valu(rh, monkeypatch, mode):
    """MobileNetV2 (batch 2) with every eligible 1x1 conv forced onto the
    VALU kernel, and with the tuner choosing per layer: oracle bits."""
    import torch
    import graph_runner
    from rten_hip import models

    monkeypatch.setenv("RTENHIP_PW_VALU", mode)
    spec = models.mobilenet_v2()
    x = np.random.default_rng(5).random((2, 3, 224, 224), dtype=np.float32)
    exp = graph_runner.run(spec, {"input": x})[spec.outputs[0]]
    g = spec.to_graph()
    xd = torch.from_numpy(x).cuda()
    out = None
    for _ in range(3):
        out = g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
        torch.cuda.synchronize()
        o = out[0].cpu().numpy()
        assert _bits_equal(o, exp), np.abs(o - exp).max()
    if mode == "16":
        g.set_timing(True)
        g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
        torch.cuda.synchronize()
        # the expand convs that run fused with their depthwise conv
        # (mbconv.hip) no longer appear as pointwise convs
        rep = g.timing_report()
        m = re.search(r"Conv\(expand\+dw\)\s+[\d.]+ ms \([^)]*\)\s+x(\d+)", rep)
        fused = int(m.group(1)) if m else 0
        # and the depthwise -> projection pair (dw_project.hip), features.1
        # (with the stem, features.0, in the same kernel by default)
        m2 = re.search(r"Conv\((?:stem\+)?dw\+project\)\s+[\d.]+ ms \([^)]*\)\s+x(\d+)", rep)
        assert m2 and int(m2.group(1)) == 1, rep
        fused += 1
        # bench.py's HBM bytes (models.conv_io_bytes) assume the executor's pairs
        from rten_hip import models as _m
        assert fused - 1 == _m.expand_dw_pairs(spec), (fused, _m.expand_dw_pairs(spec))
        assert rep.count("cfg=valu16") + fused >= 20, rep


# Direct VALU conv (3-wide kernels): (N, C, H, W, O, kh, stride, pads, tail)
DIRECT_CASES = [
    (2, 3, 16, 16, 32, 3, 2, [1, 1, 1, 1], "clip"),  # MobileNetV2 stem shape, small
    (2, 3, 17, 15, 24, 3, 2, [1, 1, 1, 1], "relu"),  # odd input, OW = 8
    (1, 4, 12, 12, 40, 3, 1, [1, 1, 1, 1], "none"),  # stride 1, partial chunk
    (2, 2, 9, 12, 16, 1, 1, [0, 1, 0, 1], "add"),   # 1x3 kernel, residual
    (1, 7, 10, 14, 8, 3, 2, [0, 2, 1, 1], "clip"),  # asymmetric pads, K = 63
    (2, 3, 224, 224, 32, 3, 2, [1, 1, 1, 1], "clip"),  # MobileNetV2 stem, full width (LDS rows: 8-row tiles)
    (1, 3, 62, 40, 24, 2, 2, [0, 0, 1, 1], "relu"),  # no left pad, stride 2, partial last row tile
    (1, 5, 20, 24, 20, 3, 1, [1, 0, 1, 2], "add"),   # no left pad, stride 1
]


def _direct_lds_eligible(case):
    N, C, H, W, O, kh, st, pads, tail = case
    return kh <= 3 and pads[1] <= 1


# 316 / 332: one lane per 4 outputs reading x directly; 416 / 432: the same
# with the block's input rows staged in LDS (conv_direct_lds_kernel).
@pytest.mark.parametrize("mode", ["316", "332", "416", "432"])
@pytest.mark.parametrize("case", DIRECT_CASES, ids=lambda c: "x".join(map(str, c[:6])) + f"s{c[6]}-{c[8]}")
def test_direct_valu_bitexact(rh, monkeypatch, mode, case):
    import torch
    import graph_runner
    from rten_hip.graph import ModelSpec

    N, C, H, W, O, kh, st, pads, tail = case
    if mode.startswith("4") and not _direct_lds_eligible(case):
        pytest.skip("LDS-row variant needs kh <= 3 and a left pad <= 1")
    monkeypatch.setenv("RTENHIP_PW_VALU", mode)
    rng = np.random.default_rng(C * 17 + O + kh)
    m = ModelSpec("direct")
    x = m.value("x")
    m.inputs = ["x"]
    ins = {"x": rng.uniform(-1, 1, (N, C, H, W)).astype(np.float32)}
    w = m.const("w", rng.uniform(-0.5, 0.5, (O, C, kh, 3)).astype(np.float32))
    b = m.const("b", rng.uniform(-0.2, 0.2, (O,)).astype(np.float32))
    y = m.op("Conv", [x, w, b], {"pads": pads, "strides": [st, st]})
    if tail == "add":
        oh = (H + pads[0] + pads[2] - kh) // st + 1
        ow = (W + pads[1] + pads[3] - 3) // st + 1
        r = m.value("r")
        m.inputs.append("r")
        ins["r"] = rng.uniform(-1, 1, (N, O, oh, ow)).astype(np.float32)
        y = m.op("Add", [y, r])
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
    assert f"cfg=valu{mode}" in g.timing_report()


def _offset_view(arr, torch):
    """A contiguous device copy of ``arr`` starting 4 bytes past a 16-byte
    boundary (as an ``out=`` slice or a sliced graph input would be)."""
    base = torch.empty(arr.size + 1, dtype=torch.float32, device="cuda")
    v = base[1:].view(arr.shape)
    v.copy_(torch.from_numpy(arr))
    assert v.data_ptr() % 16 == 4
    return v


@pytest.mark.parametrize("mode,kh,pads", [("16", 1, [0, 0, 0, 0]), ("316", 3, [1, 1, 1, 1])])
def test_valu_conv_rebound_to_misaligned_views(rh, monkeypatch, mode, kh, pads):
    """A plan tuned onto a VALU conv kernel (16-byte operands) and later bound
    to 4-byte-offset input / residual / output views runs its DMA fallback
    instead of failing, with the same bits (eager and replayed)."""
    import torch
    import graph_runner
    from rten_hip.graph import ModelSpec

    monkeypatch.setenv("RTENHIP_PW_VALU", mode)
    rng = np.random.default_rng(404 + kh)
    N, C, H, W, O = 2, 3 if kh == 3 else 24, 16, 16, 32
    m = ModelSpec("misaligned")
    x = m.value("x")
    r = m.value("r")
    m.inputs = ["x", "r"]
    w = m.const("w", rng.uniform(-0.5, 0.5, (O, C, kh, kh)).astype(np.float32))
    b = m.const("b", rng.uniform(-0.2, 0.2, (O,)).astype(np.float32))
    y = m.op("Relu", [m.op("Add", [m.op("Conv", [x, w, b], {"pads": pads, "strides": [1, 1]}), r])])
    m.outputs = [y]
    ins = {"x": rng.uniform(-1, 1, (N, C, H, W)).astype(np.float32),
           "r": rng.uniform(-1, 1, (N, O, H, W)).astype(np.float32)}
    exp = graph_runner.run(m, ins)[y]
    g = m.to_graph()
    aligned = {g.input_ids[i]: torch.from_numpy(ins[n]).cuda() for i, n in enumerate(m.inputs)}
    out = g.run(aligned, g.output_ids)  # eager: the forced VALU kernel
    torch.cuda.synchronize()
    assert _bits_equal(out[0].cpu().numpy(), exp)
    off = {g.input_ids[i]: _offset_view(ins[n], torch) for i, n in enumerate(m.inputs)}
    y_off = _offset_view(np.zeros(exp.shape, np.float32), torch)
    for feed in (off, off, aligned, off):  # capture + replays, rebinding each time
        res = g.run(feed, g.output_ids, out=[y_off])
        torch.cuda.synchronize()
        assert _bits_equal(res[0].cpu().numpy(), exp)


# Expand (1x1) -> depthwise (3x3) pairs run as one kernel (csrc/mbconv.hip):
# (N, C_in, H, W, hidden, stride, expand act, dw act, biases)
EXPAND_DW = [
    (2, 16, 112, 112, 96, 2, "clip", "clip", True),   # MobileNetV2 features.2
    (2, 24, 56, 56, 144, 1, "clip", "clip", True),    # features.3
    (3, 24, 56, 56, 144, 2, "clip", "clip", True),    # features.4
    (2, 32, 28, 28, 192, 1, "relu", "none", False),   # features.5/6 shape, other acts, no biases
    (2, 32, 28, 28, 192, 2, "none", "relu", True),    # features.7 shape
    (1, 16, 9, 20, 40, 1, "clip", "clip", True),      # odd H, partial band
    (2, 64, 14, 14, 384, 1, "clip", "clip", True),    # features.8-11 (whole-plane kernel)
    (2, 96, 14, 14, 576, 2, "clip", "clip", True),    # features.14, stride 2
    (3, 160, 7, 7, 960, 1, "clip", "clip", True),     # features.15-17 (four planes per block)
    (2, 24, 14, 14, 40, 1, "relu", "none", False),    # whole-plane kernel, partial channel pass
    (1, 48, 20, 20, 64, 1, "clip", "clip", True),     # neither kernel: both convs run apart
]


@pytest.mark.parametrize("case", EXPAND_DW, ids=lambda c: "x".join(map(str, c[:6])) + f"-{c[6]}-{c[7]}")
@pytest.mark.parametrize("policy", ["all", "default"])
def test_expand_depthwise_fused_bitexact(rh, monkeypatch, case, policy):
    """The fused expand -> depthwise kernel gives the two operators' bits
    (conv_2d_pointwise then conv_2d_depthwise_block, with the graph's Clip /
    Relu after each), eager and replayed; shapes it does not take run unfused.
    RTENHIP_EXPAND_DW=all fuses every pair a fused kernel can take; the
    default the C_in = 16 / 24 pairs and C_in = 32 at stride 2 (see
    expand_dw_eligible)."""
    import torch
    import graph_runner
    from rten_hip.graph import ModelSpec

    N, C, H, W, M, s, act_e, act_d, biases = case
    if policy == "all":
        monkeypatch.setenv("RTENHIP_EXPAND_DW", "all")
    else:
        monkeypatch.delenv("RTENHIP_EXPAND_DW", raising=False)
    rng = np.random.default_rng(C * 7 + M + s)
    m = ModelSpec("mbconv")
    x = m.value("x")
    m.inputs = ["x"]
    lo, hi = m.const("lo", np.array(0.0, np.float32)), m.const("hi", np.array(6.0, np.float32))

    def act(v, a):
        if a == "clip":
            return m.op("Clip", [v, lo, hi])
        return m.op("Relu", [v]) if a == "relu" else v

    we = m.const("we", rng.uniform(-0.5, 0.5, (M, C, 1, 1)).astype(np.float32))
    args = [x, we] + ([m.const("be", rng.uniform(-0.2, 0.2, (M,)).astype(np.float32))] if biases else [])
    e = act(m.op("Conv", args, {"pads": [0, 0, 0, 0], "strides": [1, 1]}, name="expand"), act_e)
    wd = m.const("wd", rng.uniform(-0.5, 0.5, (M, 1, 3, 3)).astype(np.float32))
    args = [e, wd] + ([m.const("bd", rng.uniform(-0.2, 0.2, (M,)).astype(np.float32))] if biases else [])
    m.outputs = [act(m.op("Conv", args, {"pads": [1, 1, 1, 1], "strides": [s, s], "groups": M}, name="dw"), act_d)]
    ins = {"x": rng.uniform(-1, 2, (N, C, H, W)).astype(np.float32)}
    exp = graph_runner.run(m, ins)[m.outputs[0]]
    g = m.to_graph()
    xd = torch.from_numpy(ins["x"]).cuda()
    out = None
    for _ in range(3):
        out = g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
        torch.cuda.synchronize()
        assert _bits_equal(out[0].cpu().numpy(), exp)
    g.set_timing(True)
    g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
    torch.cuda.synchronize()
    fused = "Conv(expand+dw)" in g.timing_report()
    if policy == "all":
        assert fused == ((C in (16, 24, 32) and W % 4 == 0) or H * W <= 256), g.timing_report()
    else:
        assert fused == ((C in (16, 24) or (C == 32 and s == 2)) and W % 4 == 0), g.timing_report()



# Network stems on MFMA (csrc/conv_stem.hip), forced with RTENHIP_PW_VALU=800:
# (N, C, H, W, O, k, pads, tail, bias)
STEM_CASES = [
    (2, 3, 32, 32, 64, 7, [3, 3, 3, 3], "relu", True),      # ResNet-50 stem, small
    (1, 3, 224, 224, 64, 7, [3, 3, 3, 3], "relu", True),    # ResNet-50 stem, batch 1 (one row per band)
    (20, 3, 224, 224, 64, 7, [3, 3, 3, 3], "relu", True),   # enough bands for the 4-row, 7-item variant
    (20, 3, 202, 200, 64, 7, [3, 3, 3, 3], "relu", True),   # 7-item variant, last band of 1 row, partial tile
    (3, 3, 200, 200, 64, 7, [3, 3, 3, 3], "relu", True),    # 2-item variant, 100-pixel bands (partial tile)
    (2, 3, 224, 224, 32, 3, [1, 1, 1, 1], "clip", True),    # MobileNetV2 stem, full size
    (3, 3, 19, 23, 24, 3, [1, 1, 1, 1], "none", False),     # odd sizes, M < 32, no bias
    (2, 3, 30, 17, 48, 7, [2, 3, 3, 1], "clip", True),      # asymmetric pads, partial 32-row tile
    (2, 3, 4, 4, 64, 7, [3, 3, 3, 3], "relu", True),        # 2x2 output
    (1, 3, 150, 250, 16, 3, [0, 0, 1, 1], "relu", True),    # OW = 125: partial column tile
]


@pytest.mark.parametrize("case", STEM_CASES, ids=lambda c: "x".join(map(str, c[:6])) + f"-{c[7]}")
def test_stem_mfma_bitexact(rh, monkeypatch, case):
    """The stem kernel gives the oracle's bits (one KC block, k in im2col
    order from +0, then bias and the fused Relu / Clip), eager and replayed."""
    import torch
    import graph_runner
    from rten_hip.graph import ModelSpec

    N, C, H, W, O, k, pads, tail, bias = case
    monkeypatch.setenv("RTENHIP_PW_VALU", "800")
    rng = np.random.default_rng(H * 7 + O + k)
    m = ModelSpec("stem")
    x = m.value("x")
    m.inputs = ["x"]
    ins = {"x": rng.uniform(-1, 1, (N, C, H, W)).astype(np.float32)}
    args = [x, m.const("w", rng.uniform(-0.5, 0.5, (O, C, k, k)).astype(np.float32))]
    if bias:
        args.append(m.const("b", rng.uniform(-0.2, 0.2, (O,)).astype(np.float32)))
    y = m.op("Conv", args, {"pads": pads, "strides": [2, 2]})
    if tail == "relu":
        y = m.op("Relu", [y])
    elif tail == "clip":
        y = m.op("Clip", [y, m.const("lo", np.array(0, np.float32)), m.const("hi", np.array(6, np.float32))])
    m.outputs = [y]
    exp = graph_runner.run(m, ins)[y]
    g = m.to_graph()
    dev = {g.input_ids[0]: torch.from_numpy(ins["x"]).cuda()}
    out = None
    for _ in range(3):  # eager, capture, replay
        out = g.run(dev, g.output_ids, out=out)
        torch.cuda.synchronize()
        o = out[0].cpu().numpy()
        assert _bits_equal(o, exp), np.abs(o - exp).max()
    g.set_timing(True)
    g.run(dev, g.output_ids, out=out)
    torch.cuda.synchronize()
    assert "cfg=stem" in g.timing_report(), g.timing_report()


@pytest.mark.parametrize("model", ["resnet50", "mobilenet_v2"])
def test_model_stem_mfma(rh, monkeypatch, model):
    """ResNet-50 / MobileNetV2 (batch 2) with the stem forced onto the MFMA
    stem kernel (every other conv tuned as usual): oracle bits.  (MobileNetV2's
    stem runs inside the stem -> depthwise -> projection kernel by default;
    RTENHIP_STEM_DWPW=0 keeps it a conv of its own here.)"""
    import torch
    import graph_runner
    from rten_hip import models

    monkeypatch.setenv("RTENHIP_PW_VALU", "800")
    monkeypatch.setenv("RTENHIP_STEM_DWPW", "0")
    spec = getattr(models, model)()
    x = np.random.default_rng(21).random((2, 3, 224, 224), dtype=np.float32)
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
    assert g.timing_report().count("cfg=stem") == 1, g.timing_report()


# Depthwise 3x3 -> 1x1 projection pairs run as one kernel (csrc/dw_project.hip):
# (N, C, H, W, M, dw act, projection tail, biases)
DW_PROJECT = [
    (2, 32, 112, 112, 16, "clip", "none", True),       # MobileNetV2 features.1
    (1, 32, 9, 112, 24, "relu", "relu", False),        # partial band, M not a multiple of 16
    (3, 32, 6, 112, 32, "none", "add_clip", True),     # residual, two channel tiles
    (1, 32, 1, 112, 16, "clip", "add", True),          # one row: both window rows skipped
    (2, 48, 8, 112, 16, "clip", "none", True),         # C = 48: runs unfused
]


@pytest.mark.parametrize("case", DW_PROJECT, ids=lambda c: "x".join(map(str, c[:5])) + f"-{c[5]}-{c[6]}")
@pytest.mark.parametrize("policy", ["on", "off"])
def test_dw_project_fused_bitexact(rh, monkeypatch, case, policy):
    """The fused depthwise -> projection kernel gives the two operators'
    bits (conv_2d_depthwise_block then conv_2d_pointwise, with the graph's
    Clip / Relu / Add after each), eager and replayed; RTENHIP_DW_PROJECT=0
    and shapes it does not take run the two convs apart."""
    import torch
    import graph_runner
    from rten_hip.graph import ModelSpec

    N, C, H, W, M, act_d, tail, biases = case
    if policy == "off":
        monkeypatch.setenv("RTENHIP_DW_PROJECT", "0")
    else:
        monkeypatch.delenv("RTENHIP_DW_PROJECT", raising=False)
    rng = np.random.default_rng(C * 5 + M + H)
    m = ModelSpec("dwpw")
    x = m.value("x")
    m.inputs = ["x"]
    lo, hi = m.const("lo", np.array(0.0, np.float32)), m.const("hi", np.array(6.0, np.float32))
    ins = {"x": rng.uniform(-1, 2, (N, C, H, W)).astype(np.float32)}
    wd = m.const("wd", rng.uniform(-0.5, 0.5, (C, 1, 3, 3)).astype(np.float32))
    args = [x, wd] + ([m.const("bd", rng.uniform(-0.2, 0.2, (C,)).astype(np.float32))] if biases else [])
    dv = m.op("Conv", args, {"pads": [1, 1, 1, 1], "strides": [1, 1], "groups": C}, name="dw")
    if act_d == "clip":
        dv = m.op("Clip", [dv, lo, hi])
    elif act_d == "relu":
        dv = m.op("Relu", [dv])
    wp = m.const("wp", rng.uniform(-0.5, 0.5, (M, C, 1, 1)).astype(np.float32))
    args = [dv, wp] + ([m.const("bp", rng.uniform(-0.2, 0.2, (M,)).astype(np.float32))] if biases else [])
    y = m.op("Conv", args, {"pads": [0, 0, 0, 0], "strides": [1, 1]}, name="project")
    if tail.startswith("add"):
        r = m.value("r")
        m.inputs.append("r")
        ins["r"] = rng.uniform(-1, 1, (N, M, H, W)).astype(np.float32)
        y = m.op("Add", [y, r])
    if tail.endswith("clip"):
        y = m.op("Clip", [y, lo, hi])
    elif tail.endswith("relu"):
        y = m.op("Relu", [y])
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
    fused = "Conv(dw+project)" in g.timing_report()
    assert fused == (policy == "on" and C == 32), g.timing_report()


# MobileNetV2's stem (3 -> 32, 3x3 / 2, pads 1) feeding the depthwise ->
# projection pair, all three in one kernel (dw_project.hip
# stem_dw_project_kernel): (N, H0, stem act, dw act, M, projection tail,
# stem bias, input scale)
STEM_DW_PROJECT = [
    (2, 224, "clip", "clip", 16, "none", True, 1.0),     # MobileNetV2 features.0 + features.1
    (1, 29, "relu", "relu", 24, "relu", False, 1.0),     # 15 rows: a partial band, zero bottom pad row; M = 24
    (3, 30, "none", "clip", 32, "add_clip", True, 1.0),  # 15 rows, residual, two channel tiles
    (1, 2, "clip", "none", 16, "add", True, 1.0),        # one output row
    (2, 56, "clip", "clip", 16, "none", True, 1e30),     # huge sums, clamped; 2 bands
]


@pytest.mark.parametrize("case", STEM_DW_PROJECT, ids=lambda c: f"n{c[0]}h{c[1]}-{c[2]}-{c[3]}-m{c[4]}-{c[5]}")
@pytest.mark.parametrize("policy", ["on", "off"])
def test_stem_dw_project_fused_bitexact(rh, monkeypatch, case, policy):
    """The stem -> depthwise -> projection kernel gives the three operators'
    bits (the stem's im2col GEMM chain + bias + act, conv_2d_depthwise_block,
    conv_2d_pointwise), eager and replayed; RTENHIP_STEM_DWPW=0 runs the stem
    apart (and the depthwise -> projection pair fused)."""
    import torch
    import graph_runner
    from rten_hip.graph import ModelSpec

    N, H0, act_s, act_d, M, tail, biases, scale = case
    if policy == "off":
        monkeypatch.setenv("RTENHIP_STEM_DWPW", "0")
    else:
        monkeypatch.delenv("RTENHIP_STEM_DWPW", raising=False)
    monkeypatch.delenv("RTENHIP_DW_PROJECT", raising=False)
    rng = np.random.default_rng(H0 * 7 + M)
    m = ModelSpec("stemdwpw")
    x = m.value("x")
    m.inputs = ["x"]
    lo, hi = m.const("lo", np.array(0.0, np.float32)), m.const("hi", np.array(6.0, np.float32))

    def act(v, a):
        if a == "clip":
            return m.op("Clip", [v, lo, hi])
        if a == "relu":
            return m.op("Relu", [v])
        return v

    ins = {"x": (rng.uniform(-1, 1, (N, 3, H0, 224)) * scale).astype(np.float32)}
    ws = m.const("ws", rng.uniform(-0.5, 0.5, (32, 3, 3, 3)).astype(np.float32))
    args = [x, ws] + ([m.const("bs", rng.uniform(-0.2, 0.2, (32,)).astype(np.float32))] if biases else [])
    sv = act(m.op("Conv", args, {"pads": [1, 1, 1, 1], "strides": [2, 2]}, name="stem"), act_s)
    wd = m.const("wd", rng.uniform(-0.5, 0.5, (32, 1, 3, 3)).astype(np.float32))
    args = [sv, wd] + ([m.const("bd", rng.uniform(-0.2, 0.2, (32,)).astype(np.float32))] if biases else [])
    dv = act(m.op("Conv", args, {"pads": [1, 1, 1, 1], "strides": [1, 1], "groups": 32}, name="dw"), act_d)
    wp = m.const("wp", rng.uniform(-0.5, 0.5, (M, 32, 1, 1)).astype(np.float32))
    args = [dv, wp] + ([m.const("bp", rng.uniform(-0.2, 0.2, (M,)).astype(np.float32))] if biases else [])
    y = m.op("Conv", args, {"pads": [0, 0, 0, 0], "strides": [1, 1]}, name="project")
    OH = (H0 - 1) // 2 + 1
    if tail.startswith("add"):
        r = m.value("r")
        m.inputs.append("r")
        ins["r"] = rng.uniform(-1, 1, (N, M, OH, 112)).astype(np.float32)
        y = m.op("Add", [y, r])
    y = act(y, tail.split("_")[-1] if "_" in tail or tail in ("relu", "clip") else "none")
    m.outputs = [y]
    exp = graph_runner.run(m, ins)[y]
    g = m.to_graph()
    dev = {g.input_ids[i]: torch.from_numpy(ins[n]).cuda() for i, n in enumerate(m.inputs)}
    out = None
    for _ in range(3):  # eager, capture, replay
        out = g.run(dev, g.output_ids, out=out)
        torch.cuda.synchronize()
        o = out[0].cpu().numpy()
        bad = np.count_nonzero(o.view(np.uint32) != exp.view(np.uint32))
        assert bad == 0, f"{bad} of {o.size} differ, max |d| {np.nanmax(np.abs(o - exp))}"
    g.set_timing(True)
    g.run(dev, g.output_ids, out=out)
    torch.cuda.synchronize()
    rep = g.timing_report()
    assert ("Conv(stem+dw+project)" in rep) == (policy == "on"), rep
    assert "Conv(dw+project)" in rep or policy == "on", rep
