"""Conv chain (csrc/conv_chain.hip): a run of small-batch convs as one
persistent launch with a grid-wide arrival barrier between phases and the
next phase's weights loaded before it.  Bar: bit-exact against the oracle
(the chain's items are gemm_lat2's, whose bits are the reference's), on the
eager first run, the chain's build run and hipGraph replays.  RTENHIP_CHAIN=1
keeps the chain whatever its build-time timing says, -1 (default) only when
it is faster; the timing report names the launch ("Conv(chain)").
"""
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


def _check(spec, x, runs=4):
    import torch
    import graph_runner

    exp = graph_runner.run(spec, {spec.inputs[0]: x})[spec.outputs[0]]
    g = spec.to_graph()
    xd = torch.from_numpy(x).cuda()
    out = None
    for r in range(runs):  # eager (tuning), chain build + capture, replays
        out = g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
        torch.cuda.synchronize()
        got = out[0].cpu().numpy()
        if not _bits_equal(got, exp):
            d = np.abs(got.astype(np.float64) - exp)
            pytest.fail(f"run {r}: max abs {d.max():.3g}, {(d > 0).sum()} of {d.size} differ")
    g.set_timing(True)
    out = g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
    torch.cuda.synchronize()
    assert _bits_equal(out[0].cpu().numpy(), exp)
    rep = g.timing_report()
    g.set_timing(False)
    return rep


@pytest.mark.parametrize("unfolded_bn", [False, True])
def test_resnet50_batch1_chain_forced(rh, monkeypatch, unfolded_bn):
    """The whole ResNet-50 body (52 convs, 48 phases) as one chain launch."""
    from rten_hip import models

    monkeypatch.setenv("RTENHIP_CHAIN", "1")
    spec = models.resnet50(unfolded_bn=unfolded_bn)
    x = np.random.default_rng(5).random((1, 3, 224, 224), dtype=np.float32)
    rep = _check(spec, x)
    assert "Conv(chain)" in rep, rep
    assert "chain of 52 convs" in rep, rep


def test_resnet50_batch2_chain_forced(rh, monkeypatch):
    """Two images per column range (the B gather's image offsets)."""
    from rten_hip import models

    monkeypatch.setenv("RTENHIP_CHAIN", "1")
    monkeypatch.setenv("RTENHIP_LAT", "72")  # every conv on the latency GEMM at batch 2
    x = np.random.default_rng(6).random((2, 3, 224, 224), dtype=np.float32)
    rep = _check(models.resnet50(), x, runs=3)
    assert "Conv(chain)" in rep, rep


def _small_net(C=24, O=40, H=17, seed=3):
    """Bottleneck-shaped chain with ragged channel and pixel counts: 1x1,
    padded 3x3 (stride 1 and 2), a 1x1 stride-2 downsample in the same phase
    as its block's conv1, residual adds, Relu, and K > 256 (split-K folds)."""
    from rten_hip.graph import ModelSpec

    rng = np.random.default_rng(seed)
    s = ModelSpec("chain_small")
    x = s.value("input")
    s.inputs = [x]

    def conv(name, inp, cin, cout, k, stride=1, pad=0, res=None, relu=True):
        w = s.const(name + "_w", ((rng.random((cout, cin, k, k), dtype=np.float32) - 0.5) * (2.0 / np.sqrt(cin * k * k))))
        b = s.const(name + "_b", (rng.random(cout, dtype=np.float32) - 0.5) * 0.1)
        h = s.op("Conv", [inp, w, b], {"pads": [pad] * 4, "strides": [stride, stride]}, name=name)
        if res is not None:
            h = s.op("Add", [h, res], name=name + "_add")
        if relu:
            h = s.op("Relu", [h], name=name + "_relu")
        return h

    stem = conv("stem", x, 3, C, 3, pad=1)  # small-C 3x3 (DMA / direct), before the chain
    h1 = conv("b1c1", stem, C, O, 1)
    h2 = conv("b1c2", h1, O, O, 3, stride=2, pad=1)
    ds = conv("b1ds", stem, C, 3 * O, 1, stride=2, relu=False)
    h3 = conv("b1c3", h2, O, 3 * O, 1, res=ds)
    h4 = conv("b2c1", h3, 3 * O, 2 * O, 1)
    h5 = conv("b2c2", h4, 2 * O, 2 * O, 3, pad=1)          # K = 720: three KC blocks
    h6 = conv("b2c3", h5, 2 * O, 3 * O, 1, res=h3)
    gap = s.op("GlobalAveragePool", [h6], name="gap")
    s.outputs = [gap]
    return s


@pytest.mark.parametrize("batch", [1, 3])
def test_chain_small_net_forced(rh, monkeypatch, batch):
    monkeypatch.setenv("RTENHIP_CHAIN", "1")
    monkeypatch.setenv("RTENHIP_LAT", "72")
    spec = _small_net()
    x = np.random.default_rng(9).random((batch, 3, 17, 17), dtype=np.float32)
    rep = _check(spec, x)
    assert "Conv(chain)" in rep, rep


@pytest.mark.parametrize("variant", ["71", "74"])
def test_chain_small_net_geometries(rh, monkeypatch, variant):
    """Items of 1 x 4 and 4 x 1 tiles (the chain takes each conv's tuned
    gemm_lat2 geometry)."""
    monkeypatch.setenv("RTENHIP_CHAIN", "1")
    monkeypatch.setenv("RTENHIP_LAT", variant)
    spec = _small_net(C=16, O=36, H=15, seed=4)
    x = np.random.default_rng(10).random((1, 3, 15, 15), dtype=np.float32)
    rep = _check(spec, x)
    assert "Conv(chain)" in rep, rep
