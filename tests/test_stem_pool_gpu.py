"""The stem (Conv 7x7 / 2, pads 3, + bias, Relu) and its MaxPool 3x3 / 2
/ pads 1 as one pass (csrc/conv_stem.hip POOL + stem_pool_finish_kernel)
against the CPU oracle running the two operators apart: conv_2d (src/ops/
conv.rs:86-280, one KC block) then pool_impl's (ky, kx) f32::max fold
(src/ops/pooling.rs:104-238).  The stem's output is never written; pooled row
2b takes the band's two rows and band b - 1's halo row.  Bar: bit-exact,
eager and replayed, with and without bias, with NaN / inf / large negative
inputs (Relu maps them to +0 / +inf, so every pooled value is a max over
non-negative, non-NaN numbers), and with RTENHIP_STEM_POOL=0 (apart)."""
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


def _stem_net(bias, seed=3):
    from rten_hip.graph import ModelSpec

    rng = np.random.default_rng(seed)
    m = ModelSpec("stem_pool")
    x = m.value("x")
    m.inputs = ["x"]
    w = m.const("w", rng.uniform(-0.1, 0.1, (64, 3, 7, 7)).astype(np.float32))
    ins = [x, w]
    if bias:
        ins.append(m.const("b", rng.uniform(-0.2, 0.2, (64,)).astype(np.float32)))
    h = m.op("Relu", [m.op("Conv", ins, {"pads": [3, 3, 3, 3], "strides": [2, 2]})])
    m.outputs = [m.op("MaxPool", [h], {"kernel_size": [3, 3], "strides": [2, 2], "pads": [1, 1, 1, 1]})]
    return m


@pytest.mark.parametrize("batch,bias,special,policy", [(20, True, False, "on"), (24, False, True, "on"),
                                                       (20, True, True, "off")])
def test_stem_pool_bitexact(rh, monkeypatch, batch, bias, special, policy):
    import torch
    import graph_runner

    if policy == "off":
        monkeypatch.setenv("RTENHIP_STEM_POOL", "0")
    spec = _stem_net(bias)
    rng = np.random.default_rng(batch)
    x = rng.uniform(-1, 1, (batch, 3, 224, 224)).astype(np.float32)
    if special:
        x[0, 0, 10:14, 20:30] = np.nan
        x[1, 1, 100, :] = np.inf
        x[2, 2, 50:60, 50:60] = -1e30
        x[3, :, 0:8, :] = -np.inf
    exp = graph_runner.run(spec, {"x": x})[spec.outputs[0]]
    assert exp.shape == (batch, 64, 56, 56)
    g = spec.to_graph()
    xd = torch.from_numpy(x).cuda()
    out = None
    for r in range(3):  # eager, capture + replay, replay
        out = g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
        torch.cuda.synchronize()
        got = out[0].cpu().numpy()
        if not _bits_equal(got, exp):
            bad = np.argwhere(got.view(np.uint32) != exp.view(np.uint32))
            pytest.fail(f"run {r}: {len(bad)} pooled values differ, first {bad[:4].tolist()}")
    g.set_timing(True)
    g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
    torch.cuda.synchronize()
    assert ("Conv(stem+pool)" in g.timing_report()) == (policy == "on")


def test_stem_pool_not_taken_off_shape(rh):
    """A 232 x 232 input (116 x 116 stem output) and a small batch (one-row
    bands) keep the two operators apart, still bit-exact."""
    import torch
    import graph_runner

    spec = _stem_net(True)
    for shape in ((20, 3, 232, 232), (2, 3, 224, 224)):
        x = np.random.default_rng(5).uniform(-1, 1, shape).astype(np.float32)
        exp = graph_runner.run(spec, {"x": x})[spec.outputs[0]]
        g = spec.to_graph()
        xd = torch.from_numpy(x).cuda()
        out = None
        for _ in range(2):
            out = g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
            torch.cuda.synchronize()
            assert _bits_equal(out[0].cpu().numpy(), exp)
        g.set_timing(True)
        g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
        torch.cuda.synchronize()
        assert "Conv(stem+pool)" not in g.timing_report()

