"""The fused inverted residual block (csrc/mbconv_block.hip): 1x1 expand
(+ bias, Clip / Relu; or none, MobileNetV2's features.1) -> 3x3 depthwise (+ bias, Clip / Relu) -> 1x1 project
(+ bias) [+ Add], bit-identical to the three operators run apart by the
oracle (conv_2d_pointwise, conv_2d_depthwise_block, conv_2d_pointwise:
src/ops/conv.rs:24-68, src/ops/conv/depthwise.rs:49-120, the KC = 256 block
fold of gemm.rs:733-1050 for hidden widths above 256), eager, captured and
replayed.  Covers both strides, every instantiated (C_in, C_out) shape,
hidden widths of 1-3 KC blocks, partial pixel tiles and bands, no biases,
Relu, the block's own residual (read from the staged band) and a residual
from another tensor."""
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


# (N, C_in, H, W, hidden, C_out, stride, act_e, act_d, biases, residual)
CASES = [
    (2, 16, 20, 20, 96, 24, 2, "clip", "clip", True, None),      # features.2-like
    (1, 16, 112, 112, 96, 24, 2, "clip", "clip", True, None),    # features.2 at full size
    (2, 24, 14, 14, 144, 24, 1, "clip", "clip", True, "x"),      # features.3-like
    (1, 24, 56, 56, 144, 24, 1, "clip", "clip", True, "x"),      # features.3 at full size (several bands)
    (2, 24, 14, 14, 144, 32, 2, "clip", "clip", True, None),     # features.4-like
    (2, 32, 9, 9, 192, 32, 1, "relu", "clip", False, "x"),       # no biases, Relu, partial tiles
    (1, 32, 28, 28, 192, 32, 1, "clip", "clip", True, "x"),      # features.5 at full size
    (1, 32, 12, 10, 192, 64, 2, "clip", "clip", True, None),     # features.7-like (512 threads)
    (2, 64, 7, 7, 384, 64, 1, "clip", "clip", True, "x"),        # hidden 384: two KC blocks
    (1, 64, 14, 14, 384, 96, 1, "clip", "relu", True, None),     # C_out 96
    (1, 96, 14, 14, 576, 96, 1, "clip", "clip", True, "x"),      # hidden 576: three KC blocks
    (1, 24, 10, 10, 144, 32, 2, "clip", "clip", True, "other"),  # residual from another tensor
    # hidden 0: no expand conv (features.1: depthwise -> project)
    (2, 32, 20, 20, 0, 16, 1, None, "clip", True, None),
    (1, 32, 112, 112, 0, 16, 1, None, "clip", True, None),        # features.1 at full size
    (2, 32, 9, 11, 0, 16, 1, None, "relu", False, None),
]


def _case_id(c):
    return f"n{c[0]}c{c[1]}_{c[2]}x{c[3]}_h{c[4]}o{c[5]}s{c[6]}_{c[7]}{c[8]}{'b' if c[9] else 'nb'}_{c[10]}"


def _block_spec(case, rng):
    from rten_hip.graph import ModelSpec

    N, C, H, W, M, O, s, act_e, act_d, biases, res = case
    m = ModelSpec("ir_block")
    x = m.value("x")
    m.inputs = ["x"]
    lo, hi = m.const("lo", np.array(0.0, np.float32)), m.const("hi", np.array(6.0, np.float32))

    def act(v, a):
        if a == "clip":
            return m.op("Clip", [v, lo, hi])
        return m.op("Relu", [v]) if a == "relu" else v

    def bias(name, n):
        return [m.const(name, rng.uniform(-0.2, 0.2, (n,)).astype(np.float32))] if biases else []

    if M:
        we = m.const("we", rng.uniform(-0.4, 0.4, (M, C, 1, 1)).astype(np.float32))
        e = act(m.op("Conv", [x, we] + bias("be", M), {"pads": [0, 0, 0, 0], "strides": [1, 1]}, name="expand"),
                act_e)
    else:  # no expand: the depthwise conv reads the block input
        M, e = C, x
    wd = m.const("wd", rng.uniform(-0.5, 0.5, (M, 1, 3, 3)).astype(np.float32))
    d = act(m.op("Conv", [e, wd] + bias("bd", M), {"pads": [1, 1, 1, 1], "strides": [s, s], "groups": M},
                 name="dw"), act_d)
    wp = m.const("wp", rng.uniform(-0.1, 0.1, (O, M, 1, 1)).astype(np.float32))
    y = m.op("Conv", [d, wp] + bias("bp", O), {"pads": [0, 0, 0, 0], "strides": [1, 1]}, name="project")
    ins = {"x": rng.uniform(-1, 2, (N, C, H, W)).astype(np.float32)}
    if res == "x":
        y = m.op("Add", [y, x])
    elif res == "other":
        oh, ow = (H - 1) // s + 1, (W - 1) // s + 1
        m.value("r")
        m.inputs.append("r")
        ins["r"] = rng.uniform(-1, 1, (N, O, oh, ow)).astype(np.float32)
        y = m.op("Add", [y, "r"])
    m.outputs = [y]
    return m, ins


@pytest.mark.parametrize("case", CASES, ids=_case_id)
def test_mbconv_block_bitexact(rh, monkeypatch, case):
    import torch
    import graph_runner

    monkeypatch.setenv("RTENHIP_MBCONV", "all")
    rng = np.random.default_rng(sum(case[1:6]) * 13 + case[6])
    m, ins = _block_spec(case, rng)
    exp = graph_runner.run(m, ins)[m.outputs[0]]
    g = m.to_graph()
    dev = {g.input_ids[i]: torch.from_numpy(ins[n]).cuda() for i, n in enumerate(m.inputs)}
    out = None
    for _ in range(3):  # eager, capture, replay
        out = g.run(dev, g.output_ids, out=out)
        torch.cuda.synchronize()
        got = out[0].cpu().numpy()
        if not _bits_equal(got, exp):
            diff = np.abs(got.astype(np.float64) - exp)
            pytest.fail(f"block differs: max abs {diff.max():.3g}, {(diff > 0).sum()} of {diff.size} elements")
    g.set_timing(True)
    g.run(dev, g.output_ids, out=out)
    torch.cuda.synchronize()
    assert "Conv(mbconv_block)" in g.timing_report(), g.timing_report()


def test_mbconv_block_default_policy(rh, monkeypatch):
    """By default (measured slower) no block fuses."""
    import torch

    monkeypatch.delenv("RTENHIP_MBCONV", raising=False)
    m, ins = _block_spec(CASES[4], np.random.default_rng(6))
    g = m.to_graph()
    dev = {g.input_ids[0]: torch.from_numpy(ins["x"]).cuda()}
    g.set_timing(True)
    g.run(dev, g.output_ids)
    torch.cuda.synchronize()
    assert "Conv(mbconv_block)" not in g.timing_report(), g.timing_report()


def test_mbconv_block_off_switch(rh, monkeypatch):
    """RTENHIP_MBCONV=0 runs the three convs apart (same bits)."""
    import torch
    import graph_runner

    monkeypatch.setenv("RTENHIP_MBCONV", "0")
    case = CASES[2]
    m, ins = _block_spec(case, np.random.default_rng(5))
    exp = graph_runner.run(m, ins)[m.outputs[0]]
    g = m.to_graph()
    dev = {g.input_ids[0]: torch.from_numpy(ins["x"]).cuda()}
    g.set_timing(True)
    out = g.run(dev, g.output_ids)
    torch.cuda.synchronize()
    assert _bits_equal(out[0].cpu().numpy(), exp)
    assert "Conv(mbconv_block)" not in g.timing_report()


def test_mbconv_block_nonfinite_depthwise_weight_unfused(rh, monkeypatch):
    """A non-finite depthwise weight keeps the block apart (the fused kernel's
    skipped taps rely on w * copysign(0, -w) == -0)."""
    import torch

    monkeypatch.setenv("RTENHIP_MBCONV", "all")
    case = CASES[2]
    m, ins = _block_spec(case, np.random.default_rng(7))
    wd = next(n for n in m.nodes if n.kind == "const" and n.name == "wd")
    wd.data[0, 0, 0, 0] = np.inf
    g = m.to_graph()
    dev = {g.input_ids[0]: torch.from_numpy(ins["x"]).cuda()}
    g.set_timing(True)
    g.run(dev, g.output_ids)
    torch.cuda.synchronize()
    assert "Conv(mbconv_block)" not in g.timing_report()
