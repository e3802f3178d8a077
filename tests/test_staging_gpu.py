"""Host-resident inputs and outputs (rten_hip/staging.py) and the executor's
capture cache (one hipGraph per input/output binding, Plan::captures): the
staged pipeline returns, for every step, the bits a device-resident run gives
for that step's images (the oracle's), while the uploads overlap earlier
steps' forwards; bindings beyond the cache's four entries re-capture without
changing results.
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


def _small_net():
    from rten_hip.graph import ModelSpec

    rng = np.random.default_rng(21)
    s = ModelSpec("staging_net")
    x = s.value("input")
    s.inputs = [x]
    w1 = s.const("w1", (rng.random((16, 3, 3, 3), dtype=np.float32) - 0.5) * 0.5)
    b1 = s.const("b1", (rng.random(16, dtype=np.float32) - 0.5) * 0.1)
    h = s.op("Relu", [s.op("Conv", [x, w1, b1], {"pads": [1, 1, 1, 1], "strides": [2, 2]})])
    w2 = s.const("w2", (rng.random((32, 16, 1, 1), dtype=np.float32) - 0.5) * 0.5)
    h = s.op("Relu", [s.op("Conv", [h, w2], {"pads": [0, 0, 0, 0]})])
    h = s.op("Flatten", [s.op("GlobalAveragePool", [h])], {"axis": 1})
    fw = s.const("fc_w", (rng.random((10, 32), dtype=np.float32) - 0.5))
    fb = s.const("fc_b", (rng.random(10, dtype=np.float32) - 0.5) * 0.1)
    s.outputs = [s.op("Gemm", [h, fw, fb], {"transB": 1})]
    return s


def test_host_staging_matches_oracle_every_step(rh):
    import torch
    import graph_runner
    from rten_hip.staging import HostStaging

    spec = _small_net()
    g = spec.to_graph()
    B = 4
    imgs = [np.random.default_rng(100 + k).random((B, 3, 32, 32), dtype=np.float32) for k in range(6)]
    exps = [graph_runner.run(spec, {"input": x})[spec.outputs[0]] for x in imgs]
    outs = [torch.empty((B, 10), device="cuda") for _ in range(2)]

    def fwd(xb, slot):
        g.run({g.input_ids[0]: xb}, g.output_ids, out=[outs[slot]])
        return outs[slot]

    st = HostStaging(fwd, (B, 3, 32, 32), torch.device("cuda", torch.cuda.current_device()))
    hin = [HostStaging.pinned((B, 3, 32, 32)) for _ in imgs]
    hout = [HostStaging.pinned((B, 10)) for _ in imgs]
    for k, x in enumerate(imgs):
        hin[k].copy_(torch.from_numpy(x))
    for k in range(len(imgs)):  # eager, capture per slot binding, replays
        st.submit(hin[k], hout[k])
    st.synchronize()
    for k in range(len(imgs)):
        assert _bits_equal(hout[k].numpy(), exps[k]), f"step {k}"
    with pytest.raises(ValueError):
        st.submit(HostStaging.pinned((B + 1, 3, 32, 32)), hout[0])


def test_capture_cache_many_bindings(rh):
    """Six input buffers in turn (more than the four cached captures): every
    run gives the oracle's bits for its own input."""
    import torch
    import graph_runner

    spec = _small_net()
    g = spec.to_graph()
    xs = [np.random.default_rng(200 + k).random((2, 3, 32, 32), dtype=np.float32) for k in range(6)]
    exps = [graph_runner.run(spec, {"input": x})[spec.outputs[0]] for x in xs]
    dev = [torch.from_numpy(x).cuda() for x in xs]
    for rep in range(3):
        for k in range(len(xs)):
            (out,) = g.run({g.input_ids[0]: dev[k]}, g.output_ids)
            torch.cuda.synchronize()
            assert _bits_equal(out.cpu().numpy(), exps[k]), (rep, k)
