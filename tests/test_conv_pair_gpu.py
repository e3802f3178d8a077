"""A bottleneck's conv3 (1x1 64 -> 256, + bias, + residual, Relu) and the next
block's conv1 (1x1 256 -> 64, + bias, Relu) run as one kernel
(csrc/conv_pair.hip) against the CPU oracle: the two convs are
conv_2d_pointwise (src/ops/conv.rs:24-68) with the GEMM's one-KC-block
summation (src/gemm.rs:733-1050), the graph's Add / Relu fused after.  Bar:
bit-exact for both outputs (conv3's is still written: the next residual),
eager and replayed, with conv1's output feeding a padded 3x3 conv, without
biases, and with RTENHIP_CONV_PAIR=0 (the two convs apart)."""
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


# (N, H, W, M1, biases, conv1 act)
CASES = [
    (8, 16, 16, 64, True, "relu"),     # layer1.x -> layer1.x+1
    (8, 8, 24, 128, True, "relu"),     # layer1.2 -> layer2.0 (M1 = 128): runs apart
    (9, 16, 12, 64, False, "none"),    # no biases, no conv1 activation
]


@pytest.mark.parametrize("policy", ["on", "off"])
@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c[:4])) + f"-{c[5]}")
def test_conv_pair_bitexact(rh, monkeypatch, case, policy):
    import torch
    import graph_runner
    from rten_hip.graph import ModelSpec

    N, H, W, M1, biases, act1 = case
    if policy == "off":
        monkeypatch.setenv("RTENHIP_CONV_PAIR", "0")
    else:
        monkeypatch.delenv("RTENHIP_CONV_PAIR", raising=False)
    rng = np.random.default_rng(N * 31 + H + M1)
    m = ModelSpec("pair")
    x, r = m.value("x"), m.value("r")
    m.inputs = ["x", "r"]
    ins = {"x": rng.uniform(-1, 1, (N, 64, H, W)).astype(np.float32),
           "r": rng.uniform(-1, 1, (N, 256, H, W)).astype(np.float32)}
    w3 = m.const("w3", rng.uniform(-0.2, 0.2, (256, 64, 1, 1)).astype(np.float32))
    args = [x, w3] + ([m.const("b3", rng.uniform(-0.2, 0.2, (256,)).astype(np.float32))] if biases else [])
    y3 = m.op("Relu", [m.op("Add", [m.op("Conv", args, {"pads": [0, 0, 0, 0], "strides": [1, 1]}, name="conv3"), r])])
    w1 = m.const("w1", rng.uniform(-0.1, 0.1, (M1, 256, 1, 1)).astype(np.float32))
    args = [y3, w1] + ([m.const("b1", rng.uniform(-0.2, 0.2, (M1,)).astype(np.float32))] if biases else [])
    y1 = m.op("Conv", args, {"pads": [0, 0, 0, 0], "strides": [1, 1]}, name="conv1")
    if act1 == "relu":
        y1 = m.op("Relu", [y1])
    w2 = m.const("w2", rng.uniform(-0.1, 0.1, (16, M1, 3, 3)).astype(np.float32))
    z = m.op("Conv", [y1, w2], {"pads": [1, 1, 1, 1], "strides": [1, 1]}, name="conv2")
    keep = m.op("Relu", [y3])  # conv3's output is read by something else too
    m.outputs = [z, keep]
    res = graph_runner.run(m, ins)
    g = m.to_graph()
    dev = {g.input_ids[i]: torch.from_numpy(ins[n]).cuda() for i, n in enumerate(m.inputs)}
    out = None
    for _ in range(3):  # eager, capture, replay
        out = g.run(dev, g.output_ids, out=out)
        torch.cuda.synchronize()
        for o, name in zip(out, m.outputs):
            got = o.cpu().numpy()
            assert _bits_equal(got, res[name]), (name, np.abs(got - res[name]).max())
    g.set_timing(True)
    g.run(dev, g.output_ids, out=out)
    torch.cuda.synchronize()
    assert ("Conv(conv3+conv1)" in g.timing_report()) == (policy == "on" and M1 == 64), g.timing_report()
