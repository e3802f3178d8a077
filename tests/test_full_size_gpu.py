"""Full-size parity for every single-GPU BASELINE config (BASELINE.json
``configs``), bit-exact against the oracle running the same graph with RTen's
semantics (the pattern of the reference's whole-model check,
src/model.rs:1078-... ``test_all_op_types``: build the model, run it, compare).

- configs[0] / the metric's batch=1: ResNet-50 loaded from a ``.rten`` file,
  batch 1 (the FC runs the reference's gemv order, gemm.rs:651-704);
- configs[1]: ResNet-50 batch 64 (tests/test_model_gpu.py);
- configs[2]: MobileNetV2 batch 128;
- configs[3]: BERT-base encoder, seq 128, batch 32, from int32 ids with a
  padded attention-mask tail (the embedding and mask subgraph included).

Each runs eager (first run: plan-time tuning), then hipGraph capture and
replay, and every run must give the oracle's bits.
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


def _check_runs(g, feed, exp, runs=3):
    import torch

    out = None
    for r in range(runs):  # eager, capture + replay, replay
        out = g.run(feed, g.output_ids, out=out)
        torch.cuda.synchronize()
        got = out[0].cpu().numpy()
        if not _bits_equal(got, exp):
            d = np.abs(got.astype(np.float64) - exp)
            pytest.fail(f"run {r}: max abs {d.max():.3g}, {(d > 0).sum()} of {d.size} elems differ")


def test_resnet50_batch1_from_rten_file(rh, tmp_path):
    """configs[0] (ResNet-50 .rten, 1x3x224x224) on the device."""
    import torch
    import graph_runner
    from rten_hip import models, rten_file

    spec = models.resnet50()
    path = tmp_path / "resnet50.rten"
    rten_file.write_rten(spec, str(path))
    g = rten_file.load_model(str(path))
    x = np.random.default_rng(1234).random((1, 3, 224, 224), dtype=np.float32)
    exp = graph_runner.run(spec, {"input": x})[spec.outputs[0]]
    assert exp.shape == (1, 1000) and np.isfinite(exp).all()
    _check_runs(g, {g.input_ids[0]: torch.from_numpy(x).cuda()}, exp)


def test_mobilenet_v2_batch128_full_size(rh):
    """configs[2] (MobileNetV2 f32, batch 128)."""
    import torch
    import graph_runner
    from rten_hip import models

    spec = models.mobilenet_v2()
    x = np.random.default_rng(77).random((128, 3, 224, 224), dtype=np.float32)
    exp = graph_runner.run(spec, {"input": x})[spec.outputs[0]]
    assert np.isfinite(exp).all()
    g = spec.to_graph()
    _check_runs(g, {g.input_ids[0]: torch.from_numpy(x).cuda()}, exp)


def test_bert_base_batch32_full_size(rh):
    """configs[3] (BERT-base encoder, seq 128, batch 32) from int32 inputs:
    random token ids, and a padded tail on a quarter of the sequences."""
    import torch
    import graph_runner
    from rten_hip import models

    B, S = 32, 128
    spec = models.bert_encoder(seq=S, embeddings=True)
    rng = np.random.default_rng(32)
    ids = rng.integers(0, 30522, (B, S)).astype(np.int32)
    tt = rng.integers(0, 2, (B, S)).astype(np.int32)
    am = np.ones((B, S), np.int32)
    for b in range(0, B, 4):
        am[b, S - 1 - 3 * b:] = 0
    feed = {"input_ids": ids, "token_type_ids": tt, "attention_mask": am}
    exp = graph_runner.run(spec, feed)[spec.outputs[0]]
    assert exp.shape == (B, S, 768) and np.isfinite(exp).all()
    g = spec.to_graph()
    dev = {g.input_ids[i]: torch.from_numpy(feed[n]).cuda() for i, n in enumerate(spec.inputs)}
    _check_runs(g, dev, exp)
