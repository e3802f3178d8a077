"""Whole-model parity on the GPU: the device graph executor (fused, hipGraph
replayed) against the CPU oracle running the same ModelSpec op by op with
RTen's semantics.  Bar: bit-exact logits.
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


def _run_both(rh, spec, batch, optimize=True, runs=3, seed=1234):
    import torch
    import graph_runner

    x = np.random.default_rng(seed).random((batch, 3, 224, 224), dtype=np.float32)
    exp = graph_runner.run(spec, {"input": x})[spec.outputs[0]]
    g = spec.to_graph(optimize=optimize)
    xd = torch.from_numpy(x).cuda()
    outs = []
    out = None
    for _ in range(runs):  # run 1 eager, later runs replay the captured hipGraph
        out = g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
        torch.cuda.synchronize()
        outs.append(out[0].cpu().numpy())
    return exp, outs


@pytest.mark.parametrize("optimize", [True, False])
def test_resnet50_bitexact(rh, optimize):
    from rten_hip import models

    exp, outs = _run_both(rh, models.resnet50(), batch=2, optimize=optimize)
    for o in outs:
        if not _bits_equal(o, exp):
            d = np.abs(o.astype(np.float64) - exp)
            pytest.fail(f"ResNet-50 logits differ: max abs {d.max():.3g}, "
                        f"rel {d.max() / np.abs(exp).max():.3g}, {(d > 0).sum()} elems")


@pytest.mark.parametrize("batch", [1, 2, 64])
def test_resnet50_unfolded_bn_bitexact(rh, batch):
    """ResNet-50 exported without BN folding (bias-free convs, each followed by
    BatchNormalization): the BN runs in the conv epilogue on the rounded conv
    output, with the reference's per-channel formula (norm.rs:45-49), on the
    latency GEMM (batch 1) and the DMA GEMM (batch 2, 64): bit-exact against
    the oracle running every BatchNormalization op, and no BN launch is left
    in the plan."""
    import torch
    from rten_hip import models

    spec = models.resnet50(unfolded_bn=True)
    exp, outs = _run_both(rh, spec, batch=batch, runs=3, seed=11)
    assert np.isfinite(exp).all()
    for o in outs:
        if not _bits_equal(o, exp):
            d = np.abs(o.astype(np.float64) - exp)
            pytest.fail(f"logits differ: max abs {d.max():.3g}, {(d > 0).sum()} elems")
    g = spec.to_graph()
    x = torch.from_numpy(np.random.default_rng(11).random((batch, 3, 224, 224), dtype=np.float32)).cuda()
    g.set_timing(True)
    out = g.run({g.input_ids[0]: x}, g.output_ids)
    g.run({g.input_ids[0]: x}, g.output_ids, out=out)
    torch.cuda.synchronize()
    rep = g.timing_report()
    assert "BatchNormalization" not in rep, rep
    assert _bits_equal(out[0].cpu().numpy(), exp)


def test_mobilenet_v2_bitexact(rh):
    from rten_hip import models

    exp, outs = _run_both(rh, models.mobilenet_v2(), batch=2)
    for o in outs:
        assert _bits_equal(o, exp), np.abs(o - exp).max()


def test_resnet50_batch64_full_size(rh, monkeypatch):
    """BASELINE config 2 (ResNet-50 f32, batch 64) end to end, bit-exact, with
    the DMA GEMM's launches tuned, all persistent (work queues) and none."""
    import torch
    from rten_hip import models

    spec = models.resnet50()
    exp, outs = _run_both(rh, spec, batch=64, runs=2, seed=7)
    assert np.isfinite(exp).all()
    for o in outs:
        assert _bits_equal(o, exp), np.abs(o - exp).max()
    x = torch.from_numpy(np.random.default_rng(7).random((64, 3, 224, 224), dtype=np.float32)).cuda()
    for mode in ("3", "0"):
        monkeypatch.setenv("RTENHIP_PERSIST", mode)
        g = spec.to_graph()
        out = None
        for _ in range(3):  # eager (tuning), capture, replay
            out = g.run({g.input_ids[0]: x}, g.output_ids, out=out)
            torch.cuda.synchronize()
            assert _bits_equal(out[0].cpu().numpy(), exp), f"RTENHIP_PERSIST={mode}"


@pytest.mark.parametrize("mode", ["2", "3", "0"])
def test_resnet50_persistent_modes(rh, monkeypatch, mode):
    """Persistent (per-XCD work queue) and one-block-per-tile DMA launches give
    the oracle's bits at batch 2 (few tiles: queues shorter than the grid)."""
    from rten_hip import models

    monkeypatch.setenv("RTENHIP_PERSIST", mode)
    exp, outs = _run_both(rh, models.resnet50(), batch=2, runs=4)
    for o in outs:
        assert _bits_equal(o, exp), np.abs(o - exp).max()


_CFG_EXP = {}


@pytest.mark.parametrize("cfg", [7, 14, 17, 19, 20, 21, 22])
def test_dma_forced_config_persistent(rh, monkeypatch, cfg):
    """Every DMA GEMM conv of ResNet-50 at batch 3 under one forced tile
    configuration (3- and 4-stage rings, 64- and 32-row tiles), launched
    persistent (RTENHIP_PERSIST=4: blocks walking several items, ragged last
    tiles, KC-split units after whole tiles), untuned: the oracle's bits in the
    eager, captured and replayed runs."""
    import ctypes as C

    import torch
    import graph_runner
    from rten_hip import models

    spec = models.resnet50()
    x = np.random.default_rng(5).random((3, 3, 224, 224), dtype=np.float32)
    if "exp" not in _CFG_EXP:
        _CFG_EXP["exp"] = graph_runner.run(spec, {"input": x})[spec.outputs[0]]
    exp = _CFG_EXP["exp"]
    monkeypatch.setenv("RTENHIP_TUNE", "0")
    monkeypatch.setenv("RTENHIP_PERSIST", "4")
    lib = rh.lib()
    lib.rtenhip_debug_set_dma_config.argtypes = [C.c_int]
    lib.rtenhip_debug_set_dma_config(cfg)
    try:
        g = spec.to_graph()
        xd = torch.from_numpy(x).cuda()
        out = None
        for _ in range(3):  # eager, capture, replay
            out = g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
            torch.cuda.synchronize()
            o = out[0].cpu().numpy()
            assert _bits_equal(o, exp), (cfg, np.abs(o - exp).max())
    finally:
        lib.rtenhip_debug_set_dma_config(-1)


def test_graph_errors(rh):
    import torch
    from rten_hip.graph import Graph

    g = Graph()
    x = g.add_value("x")
    w = g.add_constant("w", np.zeros((4, 3, 3, 3), np.float32))
    y = g.add_value("y")
    g.add_op("conv", "Conv", [x, w], [y], {"pads": [0, 0, 0, 0], "strides": [1, 1]})
    with pytest.raises(rh.OpError) as e:
        g.run({x: torch.zeros(1, 3, 2, 2, device="cuda")}, [y])
    assert "Input too small for kernel size" in str(e.value)
    z = g.add_value("z")
    with pytest.raises(rh.OpError) as e:
        g.run({}, [y])
    assert e.value.kind == "MissingInputs"


def _run_bert(rh, spec, batch, seq, hidden=768, runs=2, seed=99):
    import torch
    import graph_runner

    rng = np.random.default_rng(seed)
    x = (rng.random((batch, seq, hidden), dtype=np.float32) - np.float32(0.5))
    mask = np.zeros((batch, 1, 1, seq), np.float32)
    # a padded tail on the last sequence: additive mask -10000 (rten-cli style)
    mask[-1, :, :, seq - seq // 4:] = -10000.0
    exp = graph_runner.run(spec, {"hidden_states": x, "attention_mask": mask})[spec.outputs[0]]
    g = spec.to_graph()
    xd, md = torch.from_numpy(x).cuda(), torch.from_numpy(mask).cuda()
    outs, out = [], None
    for _ in range(runs):
        out = g.run({g.input_ids[0]: xd, g.input_ids[1]: md}, g.output_ids, out=out)
        torch.cuda.synchronize()
        outs.append(out[0].cpu().numpy())
    return exp, outs


@pytest.mark.parametrize("persist", [None, "3"])
def test_bert_two_layers_bitexact(rh, monkeypatch, persist):
    """BERT encoder (MatMul / Softmax / LayerNormalization / Gelu / Transpose)
    at a small size: batch 2, seq 32, 2 layers (MatMul launches tuned, and all
    persistent)."""
    from rten_hip import models

    if persist:
        monkeypatch.setenv("RTENHIP_PERSIST", persist)

    exp, outs = _run_bert(rh, models.bert_encoder(layers=2, seq=32), batch=2, seq=32)
    for o in outs:
        if not _bits_equal(o, exp):
            d = np.abs(o.astype(np.float64) - exp)
            pytest.fail(f"BERT output differs: max abs {d.max():.3g}, {(d > 0).sum()} elems")


@pytest.mark.parametrize("mask_op", ["mul", "where"])
def test_bert_embeddings_bitexact(rh, mask_op):
    """BERT with its embedding and mask subgraph in the device graph: int32
    input_ids / token_type_ids / attention_mask -> word, position and type
    Gathers, Unsqueeze, Cast or Where, Sub / Mul -> the encoder; eager, then
    hipGraph capture and replay, bit-exact vs the oracle."""
    import torch
    import graph_runner
    from rten_hip import models

    spec = models.bert_encoder(layers=2, seq=32, embeddings=True, vocab=1000, mask_op=mask_op)
    rng = np.random.default_rng(11)
    ids = rng.integers(0, 1000, (2, 32)).astype(np.int32)
    tt = rng.integers(0, 2, (2, 32)).astype(np.int32)
    am = np.ones((2, 32), np.int32)
    am[-1, 24:] = 0
    feed = {"input_ids": ids, "token_type_ids": tt, "attention_mask": am}
    exp = graph_runner.run(spec, feed)[spec.outputs[0]]
    g = spec.to_graph()
    dev = {g.input_ids[i]: torch.from_numpy(feed[n]).cuda() for i, n in enumerate(spec.inputs)}
    out = None
    for _ in range(3):
        out = g.run(dev, g.output_ids, out=out)
        torch.cuda.synchronize()
        assert _bits_equal(out[0].cpu().numpy(), exp)


def _gather_graph(width=3):
    from rten_hip.graph import ModelSpec

    m = ModelSpec("gather")
    ids = m.value("ids")
    m.inputs = ["ids"]
    table = m.const("table", np.arange(4 * width, dtype=np.float32).reshape(4, width))
    y = m.op("Gather", [table, ids], {"axis": 0}, name="gather")
    c = m.op("Cast", [ids], {"to": 1}, name="cast")
    m.outputs = [y, c, m.op("Relu", [y], name="relu")]
    return m


@pytest.mark.parametrize("width", [3, 8])  # 8: the float4 row-gather path (embeddings)
def test_graph_gather_index_error_and_types(rh, width):
    """Gather in the captured plan reports an out-of-range index with the
    reference's error (gather.rs:52-60) from the run that had it (eager,
    captured and replayed runs); the next valid run succeeds; negative indices
    count from the end; Cast of an int32 value; int32 data into an f32-only
    operator is IncorrectInputType."""
    import torch
    from rten_hip import OpError
    from rten_hip.graph import ModelSpec

    g = _gather_graph(width).to_graph()
    good = torch.tensor([[0, 3], [-1, 2]], dtype=torch.int32).cuda()
    bad = torch.tensor([[0, 4], [1, 2]], dtype=torch.int32).cuda()
    table = np.arange(4 * width, dtype=np.float32).reshape(4, width)
    exp = table[np.array([[0, 3], [3, 2]])]
    outs = None
    # eager (bad first), capture, replays
    for feed in ("bad", good, good, good, "bad", good, "bad", "bad", good):
        if isinstance(feed, str):
            with pytest.raises(OpError, match="Entry in `indices` is out of range") as e:
                g.run({g.input_ids[0]: bad}, g.output_ids, out=outs)
            assert e.value.kind == "InvalidValue"
            g.synchronize()  # nothing left to report
            continue
        outs = g.run({g.input_ids[0]: feed}, g.output_ids, out=outs)
        torch.cuda.synchronize()
        assert _bits_equal(outs[0].cpu().numpy(), exp)
        assert outs[1].dtype == torch.float32
        assert np.array_equal(outs[1].cpu().numpy(), feed.cpu().numpy().astype(np.float32))
    # int32 into Relu (f32 only on the device)
    m = ModelSpec("relu_int")
    x = m.value("x")
    m.inputs = ["x"]
    m.outputs = [m.op("Relu", [x], name="relu")]
    g2 = m.to_graph()
    with pytest.raises(OpError) as e:
        g2.run({g2.input_ids[0]: good}, g2.output_ids)
    assert e.value.kind == "IncorrectInputType"


@pytest.mark.parametrize("width", [3, 8])
def test_graph_gather_deferred_checks(rh, width):
    """rtenhip_graph_set_deferred_checks: runs queue without a host round trip;
    an index error is raised by synchronize() only (the earliest failing run's),
    never by a later run -- also when more runs than the check ring holds (4)
    follow the bad one, and when the later runs' own indices are valid."""
    import torch
    from rten_hip import OpError

    g = _gather_graph(width).to_graph()
    good = torch.tensor([[0, 3], [-1, 2]], dtype=torch.int32).cuda()
    bad = torch.tensor([[0, 4], [1, 2]], dtype=torch.int32).cuda()
    table = np.arange(4 * width, dtype=np.float32).reshape(4, width)
    exp = table[np.array([[0, 3], [3, 2]])]
    outs = g.run({g.input_ids[0]: good}, g.output_ids)  # eager, synchronous
    g.set_deferred_checks(True)
    for n_after in (0, 1, 6):
        g.run({g.input_ids[0]: bad}, g.output_ids, out=outs)  # no raise
        for _ in range(n_after):
            outs = g.run({g.input_ids[0]: good}, g.output_ids, out=outs)  # no raise
        with pytest.raises(OpError, match="Entry in `indices` is out of range") as e:
            g.synchronize()
        assert e.value.kind == "InvalidValue"
        g.synchronize()  # reported once
        outs = g.run({g.input_ids[0]: good}, g.output_ids, out=outs)
        g.synchronize()
        torch.cuda.synchronize()
        assert _bits_equal(outs[0].cpu().numpy(), exp)
    # back to synchronous checks: a pending deferred error is kept for synchronize()
    g.run({g.input_ids[0]: bad}, g.output_ids, out=outs)
    g.set_deferred_checks(False)
    with pytest.raises(OpError, match="out of range"):
        g.synchronize()
    with pytest.raises(OpError, match="out of range"):
        g.run({g.input_ids[0]: bad}, g.output_ids, out=outs)
    outs = g.run({g.input_ids[0]: good}, g.output_ids, out=outs)
    torch.cuda.synchronize()
    assert _bits_equal(outs[0].cpu().numpy(), exp)


def test_bert_base_seq128_bitexact(rh):
    """BASELINE config 4's model (BERT-base encoder, 12 layers, seq 128) at
    batch 2, bit-exact vs the oracle."""
    from rten_hip import models

    exp, outs = _run_bert(rh, models.bert_encoder(), batch=2, seq=128)
    assert np.isfinite(exp).all()
    for o in outs:
        assert _bits_equal(o, exp), np.abs(o - exp).max()


def _attention_spec(S, D, H=3, scale_op="Div", mask_shape="b11s", out_transpose=True):
    """q, k, v [B, H, S, D] -> MatMul(q, Transpose(k)) -> Div|Mul -> [Add(mask)]
    -> Softmax -> MatMul(., v) -> [Transpose]: the pattern Graph::optimize
    collapses into FusedAttention."""
    from rten_hip.graph import ModelSpec

    m = ModelSpec(f"attn_s{S}_d{D}")
    q, k, v = m.value("q"), m.value("k"), m.value("v")
    m.inputs = ["q", "k", "v"]
    kt = m.op("Transpose", [k], {"perm": [0, 1, 3, 2]}, name="kt")
    s = m.op("MatMul", [q, kt], name="qk")
    c = m.const("scale", np.array([np.sqrt(D)] if scale_op == "Div" else [1.0 / np.sqrt(D)], np.float32))
    s = m.op(scale_op, [s, c], name="scale")
    if mask_shape:
        m.value("mask")
        m.inputs.append("mask")
        s = m.op("Add", [s, "mask"], name="mask_add")
    s = m.op("Softmax", [s], {"axis": -1}, name="softmax")
    o = m.op("MatMul", [s, v], name="av")
    if out_transpose:
        o = m.op("Transpose", [o], {"perm": [0, 2, 1, 3]}, name="out_t")
    m.outputs = [o]
    return m


@pytest.mark.parametrize("S,D,scale_op,mask_shape,out_t", [
    (40, 64, "Div", "b11s", True),     # attention.hip
    (2, 64, "Div", "b11s", True),      # attention.hip, one key pair
    (96, 64, "Mul", "b1ss", True),     # attention.hip, three 32-key tiles
    (128, 64, "Mul", "b1ss", False),   # attention.hip, full mask, no transpose
    (64, 16, "Div", "b11s", True),     # head dim 16: unfused sequence
    (130, 64, "Mul", None, True),      # S > 128: unfused sequence
    (33, 64, "Div", "b11s", False),    # odd S: unfused sequence
])
def test_fused_attention_bitexact(rh, S, D, scale_op, mask_shape, out_t):
    import torch
    import graph_runner

    B, H = 2, 3
    spec = _attention_spec(S, D, H, scale_op, mask_shape, out_t)
    rng = np.random.default_rng(S * 100 + D)
    ins = {n: (rng.random((B, H, S, D), dtype=np.float32) - np.float32(0.5)) * 2 for n in ("q", "k", "v")}
    if mask_shape:
        shape = (B, 1, 1, S) if mask_shape == "b11s" else (B, 1, S, S)
        mask = np.zeros(shape, np.float32)
        mask[-1, ..., S - S // 4:] = -10000.0
        ins["mask"] = mask
    exp = graph_runner.run(spec, ins)[spec.outputs[0]]
    g = spec.to_graph()
    dev = {g.input_ids[i]: torch.from_numpy(ins[name]).cuda() for i, name in enumerate(spec.inputs)}
    out = None
    for _ in range(2):  # eager, then hipGraph replay
        out = g.run(dev, g.output_ids, out=out)
        torch.cuda.synchronize()
        got = out[0].cpu().numpy()
        if not _bits_equal(got, exp):
            d = np.abs(got.astype(np.float64) - exp)
            pytest.fail(f"attention differs: max abs {d.max():.3g}, {(d > 0).sum()} elems")


@pytest.mark.parametrize("mask_shape", ["b1ss", "b11s"])
def test_fused_attention_extreme_scores_bitexact(rh, mask_shape):
    """attention.hip's softmax exp (vm_exp2_nonpos) and division over the
    ranges BERT's inputs never reach: scores of a few hundred, so x - max falls
    below the -104 clamp (e = +0) and into (-104, -41) (e below 2^-60, where
    the divide takes __fdiv_rn), keys masked with -inf and -1e30 (every row
    keeps key 0 finite, so no row is all -inf): bit-exact vs the oracle."""
    import torch
    import graph_runner

    B, H, S, D = 2, 3, 128, 64
    spec = _attention_spec(S, D, H, "Mul", mask_shape, True)
    rng = np.random.default_rng(77)
    ins = {n: rng.uniform(-8, 8, (B, H, S, D)).astype(np.float32) for n in ("q", "k", "v")}
    shape = (B, 1, 1, S) if mask_shape == "b11s" else (B, 1, S, S)
    u = rng.random(shape)
    mask = np.where(u < 0.1, -np.inf, np.where(u < 0.15, -1e30, 0.0)).astype(np.float32)
    mask[..., 0] = 0.0
    ins["mask"] = mask
    exp = graph_runner.run(spec, ins)[spec.outputs[0]]
    assert np.isfinite(exp).all()
    g = spec.to_graph()
    dev = {g.input_ids[i]: torch.from_numpy(ins[name]).cuda() for i, name in enumerate(spec.inputs)}
    out = None
    for _ in range(2):  # eager, then hipGraph replay
        out = g.run(dev, g.output_ids, out=out)
        torch.cuda.synchronize()
        got = out[0].cpu().numpy()
        if not _bits_equal(got, exp):
            d = np.abs(got.astype(np.float64) - exp)
            pytest.fail(f"attention differs: max abs {d.max():.3g}, {(d > 0).sum()} elems")


def test_conv_transpose_graph_and_file_bitexact(rh):
    """A decoder-style graph (Conv -> Relu -> ConvTranspose s2 -> Relu ->
    ConvTranspose Same), run from a ModelSpec and from its .rten file."""
    import torch
    import graph_runner
    from rten_hip import rten_file
    from rten_hip.graph import ModelSpec

    rng = np.random.default_rng(21)
    m = ModelSpec("decoder")
    x = m.value("x")
    m.inputs = ["x"]
    w0 = m.const("w0", rng.uniform(-0.2, 0.2, (32, 16, 3, 3)).astype(np.float32))
    b0 = m.const("b0", rng.uniform(-0.1, 0.1, (32,)).astype(np.float32))
    h = m.op("Relu", [m.op("Conv", [x, w0, b0], {"pads": [1, 1, 1, 1], "strides": [1, 1]})])
    w1 = m.const("w1", rng.uniform(-0.2, 0.2, (32, 16, 2, 2)).astype(np.float32))
    b1 = m.const("b1", rng.uniform(-0.1, 0.1, (16,)).astype(np.float32))
    h = m.op("Relu", [m.op("ConvTranspose", [h, w1, b1], {"strides": [2, 2], "pads": [0, 0, 0, 0]})])
    w2 = m.const("w2", rng.uniform(-0.2, 0.2, (16, 8, 3, 3)).astype(np.float32))
    m.outputs = [m.op("ConvTranspose", [h, w2], {"strides": [2, 2], "auto_pad": "same"})]
    xin = rng.random((2, 16, 20, 20), dtype=np.float32)
    exp = graph_runner.run(m, {"x": xin})[m.outputs[0]]
    assert exp.shape == (2, 8, 80, 80)
    for g in (m.to_graph(), rten_file.load_model(rten_file.to_rten_bytes(m))):
        out = None
        for _ in range(2):
            out = g.run({g.input_ids[0]: torch.from_numpy(xin).cuda()}, g.output_ids, out=out)
            torch.cuda.synchronize()
            assert _bits_equal(out[0].cpu().numpy(), exp)


@pytest.mark.parametrize("B,K,O,c_kind", [
    (2, 2048, 1000, "vec"),   # ResNet-50 classifier at batch 2
    (64, 2048, 1000, "row"),  # bench batch, C as [1, O]
    (3, 17, 10, None),        # short K, no C
    (5, 300, 130, "vec"),     # two KC blocks, the second partial
    (1, 2048, 1000, "vec"),   # batch 1: the reference's gemv order (general path)
    (1, 300, 130, "row"),     # batch 1, C as [1, O], read by the gemv in place of a copy
])
def test_gemm_fc_bitexact(rh, B, K, O, c_kind):
    """Gemm with a constant transposed weight (the classifier layer): batch >= 2
    runs on the DMA GEMM as a pointwise conv over B images of [K, 1, 1], with C
    folded like a conv bias (C + block 0, then the later KC blocks)."""
    import torch
    import graph_runner
    from rten_hip.graph import ModelSpec

    rng = np.random.default_rng(B * 7919 + K)
    m = ModelSpec(f"fc_{B}_{K}_{O}")
    x = m.value("x")
    m.inputs = ["x"]
    ins = [x, m.const("w", rng.uniform(-0.05, 0.05, (O, K)).astype(np.float32))]
    if c_kind:
        shape = (O,) if c_kind == "vec" else (1, O)
        ins.append(m.const("c", rng.uniform(-0.1, 0.1, shape).astype(np.float32)))
    m.outputs = [m.op("Gemm", ins, {"alpha": 1.0, "beta": 1.0, "transA": 0, "transB": 1})]
    xin = rng.random((B, K), dtype=np.float32) - np.float32(0.5)
    exp = graph_runner.run(m, {"x": xin})[m.outputs[0]]
    g = m.to_graph()
    out = None
    for _ in range(2):  # eager (tuning), then hipGraph replay
        out = g.run({g.input_ids[0]: torch.from_numpy(xin).cuda()}, g.output_ids, out=out)
        torch.cuda.synchronize()
        got = out[0].cpu().numpy()
        assert _bits_equal(got, exp), f"max abs {np.abs(got.astype(np.float64) - exp).max():.3g}"


def _pad_conv_spec(C=3, O=32):
    """Conv 3x3 pad 1 on a graph input (padded through the context's scratch
    slot) -> Relu."""
    from rten_hip.graph import ModelSpec

    rng = np.random.default_rng(5)
    m = ModelSpec("padconv")
    x = m.value("x")
    m.inputs = ["x"]
    w = m.const("w", rng.uniform(-0.3, 0.3, (O, C, 3, 3)).astype(np.float32))
    b = m.const("b", rng.uniform(-0.1, 0.1, (O,)).astype(np.float32))
    m.outputs = [m.op("Relu", [m.op("Conv", [x, w, b], {"pads": [1, 1, 1, 1], "strides": [1, 1]})])]
    return m


def test_replay_after_scratch_grows(rh):
    """A captured plan that baked in a context scratch buffer is re-captured
    when another plan grows (and frees) that buffer: batch 1 twice (eager,
    capture), batch 8 (grows the padded-input scratch), batch 1 again with the
    same input/output buffers -- bit-exact every time."""
    import torch
    import graph_runner

    spec = _pad_conv_spec()
    g = spec.to_graph()
    rng = np.random.default_rng(11)
    x1 = rng.random((1, 3, 40, 40), dtype=np.float32)
    x8 = rng.random((8, 3, 40, 40), dtype=np.float32)
    e1 = graph_runner.run(spec, {"x": x1})[spec.outputs[0]]
    e8 = graph_runner.run(spec, {"x": x8})[spec.outputs[0]]
    d1 = torch.from_numpy(x1).cuda()
    out1 = None
    for _ in range(2):
        out1 = g.run({g.input_ids[0]: d1}, g.output_ids, out=out1)
        torch.cuda.synchronize()
        assert _bits_equal(out1[0].cpu().numpy(), e1)
    out8 = g.run({g.input_ids[0]: torch.from_numpy(x8).cuda()}, g.output_ids)
    torch.cuda.synchronize()
    assert _bits_equal(out8[0].cpu().numpy(), e8)
    # fresh allocations that may land on the freed scratch memory
    junk = [torch.full((1 << 20,), float("nan"), device="cuda") for _ in range(8)]
    for _ in range(2):
        out1 = g.run({g.input_ids[0]: d1}, g.output_ids, out=out1)
        torch.cuda.synchronize()
        assert _bits_equal(out1[0].cpu().numpy(), e1)
    del junk


@pytest.mark.parametrize("other", ["const_c11", "input_c11", "scalar"])
def test_conv_add_broadcast_unfused(rh, other):
    """Conv -> Add(x) -> Relu where x broadcasts ([1, C, 1, 1] constant or
    input, or a scalar): the Add runs unfused after the conv, as in the
    reference, instead of failing the plan."""
    import torch
    import graph_runner
    from rten_hip.graph import ModelSpec

    rng = np.random.default_rng(17)
    m = ModelSpec("conv_add_bcast")
    x = m.value("x")
    m.inputs = ["x"]
    w = m.const("w", rng.uniform(-0.3, 0.3, (16, 8, 1, 1)).astype(np.float32))
    c = m.op("Conv", [x, w], {"pads": [0, 0, 0, 0], "strides": [1, 1]})
    ins = {"x": rng.random((2, 8, 12, 12), dtype=np.float32)}
    if other == "const_c11":
        o = m.const("bias", rng.uniform(-1, 1, (1, 16, 1, 1)).astype(np.float32))
    elif other == "scalar":
        o = m.const("s", np.array(0.25, np.float32))
    else:
        o = m.value("bias")
        m.inputs.append("bias")
        ins["bias"] = rng.uniform(-1, 1, (1, 16, 1, 1)).astype(np.float32)
    m.outputs = [m.op("Relu", [m.op("Add", [c, o])])]
    exp = graph_runner.run(m, ins)[m.outputs[0]]
    g = m.to_graph()
    dev = {g.input_ids[i]: torch.from_numpy(ins[n]).cuda() for i, n in enumerate(m.inputs)}
    out = None
    for _ in range(2):
        out = g.run(dev, g.output_ids, out=out)
        torch.cuda.synchronize()
        assert _bits_equal(out[0].cpu().numpy(), exp)


def test_transpose_invalid_perm(rh):
    import torch
    from rten_hip.graph import Graph

    for perm in ([0, 0, 1], [0, 1, 3], [2, 1]):
        g = Graph()
        x = g.add_value("x")
        y = g.add_value("y")
        g.add_op("t", "Transpose", [x], [y], {"perm": perm})
        with pytest.raises(rh.OpError, match="Permutation is invalid"):
            g.run({x: torch.zeros(2, 3, 4, device="cuda")}, [y])


@pytest.mark.parametrize("case", [(300, 256, 520, 132, True), (256, 128, 512, 256, False)],
                         ids=["ragged-gelu", "even-plain"])
@pytest.mark.parametrize("pk_out", ["1", "0"])
def test_matmul_chain_packed_a_bitexact(rh, monkeypatch, case, pk_out):
    """MatMul -> (Add bias, Gelu) -> MatMul, the producer's output read only as
    the consumer's A (BERT's FFN1 -> FFN2): from the second run on the
    producer stores its output in the consumer's packed-A layout and the
    consumer skips its pack (Plan::mm_next).  Ragged M and a consumer K that is
    not a whole number of its k tiles check the zero padding.  Bit-exact
    against the oracle, eager, captured and replayed; RTENHIP_NO_PK_OUT=1 is
    the unfused reference path."""
    import torch
    import graph_runner
    from rten_hip.graph import ModelSpec

    M, K1, N1, N2, gelu = case
    if pk_out == "0":
        monkeypatch.setenv("RTENHIP_NO_PK_OUT", "1")
    else:
        monkeypatch.delenv("RTENHIP_NO_PK_OUT", raising=False)
    rng = np.random.default_rng(M + N1)
    m = ModelSpec("mmchain")
    x = m.value("x")
    m.inputs = ["x"]
    w1 = m.const("w1", rng.uniform(-0.1, 0.1, (K1, N1)).astype(np.float32))
    b1 = m.const("b1", rng.uniform(-0.1, 0.1, (N1,)).astype(np.float32))
    w2 = m.const("w2", rng.uniform(-0.1, 0.1, (N1, N2)).astype(np.float32))
    h = m.op("Add", [m.op("MatMul", [x, w1]), b1])
    if gelu:
        h = m.op("Gelu", [h])
    m.outputs = [m.op("MatMul", [h, w2])]
    ins = {"x": rng.uniform(-1, 1, (2, M // 2, K1)).astype(np.float32)}
    exp = graph_runner.run(m, ins)[m.outputs[0]]
    g = m.to_graph()
    xd = torch.from_numpy(ins["x"]).cuda()
    out = None
    for r in range(4):  # eager (tuning), capture, replays
        out = g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
        torch.cuda.synchronize()
        got = out[0].cpu().numpy()
        assert _bits_equal(got, exp), f"run {r}: max abs {np.abs(got - exp).max():.3g}"


@pytest.mark.parametrize("K", [256, 768])
@pytest.mark.parametrize("pk_out", ["1", "0"])
def test_layernorm_packed_a_bitexact(rh, monkeypatch, pk_out, K):
    """LayerNormalization -> two MatMuls reading it as A (BERT's LN -> Q / K)
    with the LN output also the second MatMul's fused residual: from the
    second run on the LN stores its rows both row-major and in the MatMuls'
    packed-A layout, and neither MatMul packs A (Plan::pk_cons).  Ragged M
    (300 rows: a partial last block of rows, for the runtime-length kernel
    and for BERT's 768-wide instance).  Bit-exact, eager, captured and
    replayed."""
    import torch
    import graph_runner
    from rten_hip.graph import ModelSpec

    if pk_out == "0":
        monkeypatch.setenv("RTENHIP_NO_PK_OUT", "1")
    else:
        monkeypatch.delenv("RTENHIP_NO_PK_OUT", raising=False)
    rng = np.random.default_rng(5)
    M, N = 300, K  # (N = K: the second MatMul adds h as its residual)
    m = ModelSpec("lnmm")
    x = m.value("x")
    m.inputs = ["x"]
    sc = m.const("sc", rng.uniform(0.5, 1.5, (K,)).astype(np.float32))
    bi = m.const("bi", rng.uniform(-0.1, 0.1, (K,)).astype(np.float32))
    h = m.op("LayerNormalization", [x, sc, bi], {"axis": -1, "epsilon": 1e-12})
    w1 = m.const("w1", rng.uniform(-0.1, 0.1, (K, N)).astype(np.float32))
    w2 = m.const("w2", rng.uniform(-0.1, 0.1, (K, N)).astype(np.float32))
    q = m.op("MatMul", [h, w1])
    k = m.op("Add", [m.op("MatMul", [h, w2]), h])
    m.outputs = [q, k]
    ins = {"x": rng.uniform(-1, 1, (3, M // 3, K)).astype(np.float32)}
    res = graph_runner.run(m, ins)
    g = m.to_graph()
    xd = torch.from_numpy(ins["x"]).cuda()
    out = None
    for r in range(4):  # eager (tuning), capture, replays
        out = g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
        torch.cuda.synchronize()
        for i, name in enumerate(m.outputs):
            got = out[i].cpu().numpy()
            assert _bits_equal(got, res[name]), f"run {r} output {i}: max abs {np.abs(got - res[name]).max():.3g}"


# conv3 + downsample pairs as one dual DMA GEMM (Plan::conv_dual):
# (N, C_in, H, W, C_mid, C_out, stride)
DUAL_BLOCKS = [
    (2, 64, 20, 20, 64, 256, 1),     # layer1.0 shape family, K = 64 + 64
    (2, 256, 18, 18, 128, 512, 2),   # layer2.0: strided downsample, K = 128 + 256
    (1, 512, 9, 9, 256, 1024, 2),    # layer3.0: K = 256 + 512 (downsample folds 2 KC blocks)
    (1, 96, 7, 11, 48, 136, 1),      # ragged M (136), K not a multiple of 16, N = 77
    (2, 48, 12, 12, 32, 128, 1),     # K1 = 48: no single K loop, so 4-byte B copies
    (1, 512, 8, 8, 256, 512, 1),     # 16-byte B copies, K = 256 + 512 (segment 1 folds 2 KC blocks)
]


@pytest.mark.parametrize("case", DUAL_BLOCKS, ids=lambda c: "x".join(map(str, c)))
@pytest.mark.parametrize("mode", ["force", "force-two-pass", "off"])
def test_bottleneck_dual_gemm_bitexact(rh, monkeypatch, case, mode):
    """ResNet bottleneck with a downsample branch: relu(conv3(h) + b3 +
    downsample(x)) with conv3 and the downsample in one dual GEMM launch
    (RTENHIP_DUAL=1 forces it; the default takes it when faster) -- one K
    loop over both segments by default, two passes with
    RTENHIP_DMA_DUAL1=0 -- or apart (RTENHIP_NO_DUAL=1).  Bit-exact against
    the oracle, eager and replayed."""
    import torch
    import graph_runner
    from rten_hip.graph import ModelSpec

    N, C, H, W, Cm, Co, s = case
    monkeypatch.delenv("RTENHIP_DUAL", raising=False)
    monkeypatch.delenv("RTENHIP_NO_DUAL", raising=False)
    monkeypatch.delenv("RTENHIP_DMA_DUAL1", raising=False)
    if mode.startswith("force"):
        monkeypatch.setenv("RTENHIP_DUAL", "1")
        if mode == "force-two-pass":
            monkeypatch.setenv("RTENHIP_DMA_DUAL1", "0")
    else:
        monkeypatch.setenv("RTENHIP_NO_DUAL", "1")
    rng = np.random.default_rng(C + Cm + Co)
    m = ModelSpec("block")
    x = m.value("x")
    m.inputs = ["x"]

    def conv(v, ci, co, k, st, name, pad):
        w = m.const(name + ".w", rng.uniform(-0.3, 0.3, (co, ci, k, k)).astype(np.float32))
        b = m.const(name + ".b", rng.uniform(-0.1, 0.1, (co,)).astype(np.float32))
        return m.op("Conv", [v, w, b], {"pads": [pad] * 4, "strides": [st, st]}, name=name)

    h = m.op("Relu", [conv(x, C, Cm, 1, 1, "c1", 0)])
    h = m.op("Relu", [conv(h, Cm, Cm, 3, s, "c2", 1)])
    y = conv(h, Cm, Co, 1, 1, "c3", 0)
    d = conv(x, C, Co, 1, s, "ds", 0)
    m.outputs = [m.op("Relu", [m.op("Add", [y, d])])]
    ins = {"x": rng.uniform(-1, 1, (N, C, H, W)).astype(np.float32)}
    exp = graph_runner.run(m, ins)[m.outputs[0]]
    g = m.to_graph()
    xd = torch.from_numpy(ins["x"]).cuda()
    out = None
    for r in range(3):  # eager (tuning + the dual decision), capture, replay
        out = g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
        torch.cuda.synchronize()
        got = out[0].cpu().numpy()
        assert _bits_equal(got, exp), f"run {r}: max abs {np.abs(got - exp).max():.3g}"
    g.set_timing(True)
    g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
    torch.cuda.synchronize()
    rep = g.timing_report()
    assert ("Conv(dual)" in rep) == mode.startswith("force"), rep


@pytest.mark.parametrize("group", ["on", "off"])
def test_grouped_matmuls_bitexact(rh, monkeypatch, group):
    """MatMuls sharing A with constant weights (BERT's Q / K / V projections)
    run as one GEMM over stacked weight / bias / output segments
    (MatMulExec::nseg; RTENHIP_MM_GROUP=0 keeps them apart): every output
    element keeps its own K chain, so the bits are the unfused graph's."""
    import torch
    import graph_runner
    from rten_hip.graph import ModelSpec

    if group == "off":
        monkeypatch.setenv("RTENHIP_MM_GROUP", "0")
    else:
        monkeypatch.delenv("RTENHIP_MM_GROUP", raising=False)
    rng = np.random.default_rng(77)
    B, S, K, N = 4, 64, 256, 256
    m = ModelSpec("qkv")
    a = m.value("a")
    m.inputs = ["a"]
    outs = []
    for name, bias in (("q", True), ("k", True), ("v", True)):
        w = m.const(name + ".w", rng.uniform(-0.1, 0.1, (K, N)).astype(np.float32))
        y = m.op("MatMul", [a, w], name=name)
        if bias:
            y = m.op("Add", [y, m.const(name + ".b", rng.uniform(-0.1, 0.1, (N,)).astype(np.float32))])
        outs.append(y)
    m.outputs = [m.op("Mul", [m.op("Add", [outs[0], outs[1]]), outs[2]])]
    ins = {"a": rng.uniform(-1, 1, (B, S, K)).astype(np.float32)}
    exp = graph_runner.run(m, ins)[m.outputs[0]]
    g = m.to_graph()
    ad = torch.from_numpy(ins["a"]).cuda()
    out = None
    for _ in range(3):
        out = g.run({g.input_ids[0]: ad}, g.output_ids, out=out)
        torch.cuda.synchronize()
        got = out[0].cpu().numpy()
        assert _bits_equal(got, exp), np.abs(got - exp).max()
    g.set_timing(True)
    g.run({g.input_ids[0]: ad}, g.output_ids, out=out)
    torch.cuda.synchronize()
    rep = g.timing_report()
    g.set_timing(False)
    # The grouping is actually taken (or not) -- not a pass on the ungrouped path.
    assert ("MatMul(in_group)" in rep) == (group == "on"), rep
    # (q reads k's output as its fused residual, so k and v form the group)
    assert (" group2" in rep) == (group == "on"), rep

    # Knob change after planning: with the DMA GEMM disabled the graph makes a
    # new plan (Plan::dma_mm) without groups, and every output is still written.
    import ctypes

    lib = rh.lib()
    lib.rtenhip_debug_set_dma.argtypes = [ctypes.c_void_p, ctypes.c_int]
    ctx = rh.default_context()
    lib.rtenhip_debug_set_dma(ctypes.c_void_p(ctx.ptr), 0)
    try:
        for _ in range(3):
            out = g.run({g.input_ids[0]: ad}, g.output_ids, out=out)
            torch.cuda.synchronize()
            got = out[0].cpu().numpy()
            assert _bits_equal(got, exp), np.abs(got - exp).max()
    finally:
        lib.rtenhip_debug_set_dma(ctypes.c_void_p(ctx.ptr), 1)


@pytest.mark.parametrize("attn_pk", ["on", "off"])
@pytest.mark.parametrize("extra_reader", [False, True])
def test_attention_packed_a_store_bitexact(rh, monkeypatch, attn_pk, extra_reader):
    """FusedAttention -> Reshape -> MatMul (BERT's output projection): the
    attention kernel stores the MatMul's packed A (Plan::attn_pk), alone when
    nothing else reads its output (Plan::attn_pk_only), both layouts when the
    reshaped output has another reader.  The layout is fixed by the MatMul's
    tile on the first run, so the eager run, the capture and the replays are
    all checked; RTENHIP_ATTN_PK=0 turns the packed store off."""
    import torch
    import graph_runner

    if attn_pk == "off":
        monkeypatch.setenv("RTENHIP_ATTN_PK", "0")
    else:
        monkeypatch.delenv("RTENHIP_ATTN_PK", raising=False)
    B, H, S, D, N = 4, 4, 64, 64, 256  # M * N * K = 2^24: the dense DMA GEMM
    m = _attention_spec(S, D, H, "Div", "b11s", True)
    o = m.outputs[0]
    shape_merge = m.const("shape.merge", np.array([0, 0, H * D], np.float32))
    c = m.op("Reshape", [o, shape_merge], name="ctx.reshape")
    rng = np.random.default_rng(5)
    w = m.const("proj.w", rng.uniform(-0.1, 0.1, (H * D, N)).astype(np.float32))
    b = m.const("proj.b", rng.uniform(-0.1, 0.1, (N,)).astype(np.float32))
    y = m.op("Add", [m.op("MatMul", [c, w], name="proj"), b], name="proj.add")
    m.outputs = [y] + ([m.op("Relu", [c], name="other")] if extra_reader else [])
    ins = {n: (rng.random((B, H, S, D), dtype=np.float32) - np.float32(0.5)) * 2 for n in ("q", "k", "v")}
    mask = np.zeros((B, 1, 1, S), np.float32)
    mask[-1, ..., S - S // 4:] = -10000.0
    ins["mask"] = mask
    res = graph_runner.run(m, ins)
    g = m.to_graph()
    dev = {g.input_ids[i]: torch.from_numpy(ins[name]).cuda() for i, name in enumerate(m.inputs)}
    out = None
    for r in range(4):  # eager (tuning fixes the layout), capture, replays
        out = g.run(dev, g.output_ids, out=out)
        torch.cuda.synchronize()
        for i, name in enumerate(m.outputs):
            got = out[i].cpu().numpy()
            assert _bits_equal(got, res[name]), f"run {r} output {i}: max abs {np.abs(got - res[name]).max():.3g}"
