"""Host-resident and batch-sharded runs through the C ABI (csrc/graph_io.cpp),
driven with ctypes and numpy host arrays only -- the surface a Rust
``Model::run`` caller binds (src/model.rs:580-592; rten-cli times that call
in a loop, rten-cli/src/main.rs:296-317).

- ``rtenhip_graph_run_host`` / ``rtenhip_graph_wait``: every queued run's
  outputs are the oracle's bits for that run's inputs, with the inputs changing
  from run to run (so a slot that was uploaded too late, or a download that
  raced the next forward, shows up as wrong bits); the plan's eager, capture
  and replay runs are all inside the pipeline.
- Gather index errors of host runs come back from ``rtenhip_graph_wait``.
- ``rtenhip_sharded_*``: a ResNet-50 ``.rten`` replicated as two shards on the
  one GPU (gather by host copies; RCCL needs distinct devices), even and
  ragged batches, each shard bit-exact against the oracle run on that shard
  (DESIGN.md §5 on per-shard bits).
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

    rng = np.random.default_rng(5)
    m = ModelSpec("small")
    x = m.value("x")
    m.inputs = ["x"]
    w1 = m.const("w1", rng.uniform(-0.3, 0.3, (32, 8, 3, 3)).astype(np.float32))
    b1 = m.const("b1", rng.uniform(-0.1, 0.1, (32,)).astype(np.float32))
    w2 = m.const("w2", rng.uniform(-0.2, 0.2, (10, 32)).astype(np.float32))
    b2 = m.const("b2", rng.uniform(-0.1, 0.1, (10,)).astype(np.float32))
    h = m.op("Relu", [m.op("Conv", [x, w1, b1], {"pads": [1, 1, 1, 1], "strides": [1, 1]})])
    p = m.op("Flatten", [m.op("GlobalAveragePool", [h])], {"axis": 1})
    m.outputs = [m.op("Gemm", [p, w2, b2], {"transB": 1})]
    return m


@pytest.mark.parametrize("model,batch,pinned_io", [("small", 4, True), ("small", 4, False),
                                                   ("resnet50", 8, True)])
def test_graph_run_host_pipeline_bitexact(rh, model, batch, pinned_io):
    import graph_runner
    from rten_hip import models
    from rten_hip.host import pinned

    spec = _small_net() if model == "small" else models.resnet50()
    shape = (batch, 8, 12, 12) if model == "small" else (batch, 3, 224, 224)
    g = spec.to_graph()
    rng = np.random.default_rng(11)
    xs = [rng.random(shape, dtype=np.float32) for _ in range(3)]
    exps = [graph_runner.run(spec, {spec.inputs[0]: x})[spec.outputs[0]] for x in xs]
    alloc = pinned if pinned_io else (lambda s: np.empty(s, np.float32))
    hin = []
    for x in xs:
        h = alloc(shape)
        h[...] = x
        hin.append(h)
    steps = 7
    outs = [alloc(exps[0].shape) for _ in range(steps)]
    ids = [g.run_host({g.input_ids[0]: hin[k % 3]}, g.output_ids, [outs[k]]) for k in range(steps)]
    assert ids == sorted(ids) and len(set(ids)) == steps
    g.wait(ids[2])  # run 2 (and every earlier one) is on the host now
    for k in range(3):
        assert _bits_equal(outs[k], exps[k % 3]), f"run {k} (waited for by id)"
    g.wait()
    for k in range(steps):
        assert _bits_equal(outs[k], exps[k % 3]), f"run {k}"
    # A new input shape re-sizes the slots; Model::run semantics (run + wait).
    x1 = np.ascontiguousarray(xs[0][:1])
    o1 = np.empty((1,) + exps[0].shape[1:], np.float32)
    g.wait(g.run_host({g.input_ids[0]: x1}, g.output_ids, [o1]))
    assert _bits_equal(o1, graph_runner.run(spec, {spec.inputs[0]: x1})[spec.outputs[0]])


def test_graph_run_host_errors(rh):
    """Output shape mismatch fails at submission; a Gather index error of a
    host run is reported by wait (gather.rs:52-60), and the next runs are
    clean."""
    from rten_hip import OpError
    from rten_hip.graph import ModelSpec

    m = ModelSpec("gather")
    ids = m.value("ids")
    m.inputs = ["ids"]
    table = m.const("table", np.arange(4 * 8, dtype=np.float32).reshape(4, 8))
    m.outputs = [m.op("Gather", [table, ids], {"axis": 0}, name="gather")]
    g = m.to_graph()
    tab = np.arange(4 * 8, dtype=np.float32).reshape(4, 8)
    good = np.array([[0, 3], [-1, 2]], np.int32)
    bad = np.array([[0, 4], [1, 2]], np.int32)
    with pytest.raises(OpError, match="wrong shape"):
        g.run_host({g.input_ids[0]: good}, g.output_ids, [np.empty((2, 3), np.float32)])
    outs = [np.empty((2, 2, 8), np.float32) for _ in range(4)]
    for k, feed in enumerate((good, good, bad, good)):
        g.run_host({g.input_ids[0]: feed}, g.output_ids, [outs[k]])
    with pytest.raises(OpError, match="Entry in `indices` is out of range"):
        g.wait()
    g.wait()  # reported once
    for k in (0, 1, 3):
        assert _bits_equal(outs[k], tab[np.array([[0, 3], [3, 2]])])
    o = np.empty((2, 2, 8), np.float32)
    g.wait(g.run_host({g.input_ids[0]: good}, g.output_ids, [o]))
    assert _bits_equal(o, tab[np.array([[0, 3], [3, 2]])])


@pytest.mark.parametrize("batch", [5, 4, 1])
def test_sharded_two_shards_one_gpu_bitexact(rh, batch):
    """rtenhip_sharded_* over two shards on cuda:0 (host-copy gather): each
    shard's rows are the oracle's bits for that shard (5 -> 3 + 2, 4 -> 2 + 2,
    1 -> 1 + 0), repeated runs replay the captured plans."""
    import graph_runner
    from rten_hip import models, rten_file
    from rten_hip.host import ShardedModel, pinned
    from rten_hip.parallel import shard_bounds

    spec = models.resnet50()
    sm = ShardedModel(rten_file.to_rten_bytes(spec), [0, 0])
    assert sm.gather_mode == "host"
    x = pinned((batch, 3, 224, 224))
    x[...] = np.random.default_rng(1234).random((batch, 3, 224, 224), dtype=np.float32)
    parts = []
    for r in range(2):
        a, b = shard_bounds(batch, r, 2)
        if b > a:
            parts.append(graph_runner.run(spec, {"input": np.ascontiguousarray(x[a:b])})[spec.outputs[0]])
    exp = np.concatenate(parts)
    for run in range(3):  # eager (tuning), capture + replay, replay
        out = np.full((batch, 1000), np.nan, np.float32)
        sm.run(x, out)
        bad = sorted({int(i) for i in np.nonzero(out.view(np.uint32) != exp.view(np.uint32))[0]})
        assert not bad, f"run {run}: images {bad} of {batch} differ"
    sm.close()


def test_sharded_errors(rh):
    from rten_hip import OpError, models, rten_file
    from rten_hip.host import ShardedModel

    with pytest.raises(OpError):
        ShardedModel(b"not a model", [0])
    sm = ShardedModel(rten_file.to_rten_bytes(_small_net()), [0])
    with pytest.raises(OpError, match="wrong shape"):
        sm.run(np.zeros((2, 8, 12, 12), np.float32), np.zeros((3, 10), np.float32))
    out = np.zeros((0, 10), np.float32)
    sm.run(np.zeros((0, 8, 12, 12), np.float32), out)  # empty batch: nothing to do
    sm.close()


def test_runs_on_the_executor_stream(rh):
    """rtenhip_set_exec_stream: a caller issuing runs from the executor stream
    itself (no cross-stream events between runs) gets the oracle's bits through
    eager, capture and replay runs, and can go back to a library-owned
    executor."""
    import torch
    import graph_runner
    from rten_hip import Context, models

    spec = models.resnet50()
    x = np.random.default_rng(3).random((1, 3, 224, 224), dtype=np.float32)
    exp = graph_runner.run(spec, {"input": x})[spec.outputs[0]]
    ctx = Context(0)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        ctx.use_stream(s)
        g = spec.to_graph(ctx)
        xd = torch.from_numpy(x).cuda()
        out = None
        for r in range(4):
            out = g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
            s.synchronize()
            assert _bits_equal(out[0].cpu().numpy(), exp), f"run {r}"
    from rten_hip import check, lib
    import ctypes as C

    check(lib().rtenhip_set_exec_stream(C.c_void_p(ctx.ptr), None))  # back to a library-owned executor
    out = g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
    torch.cuda.synchronize()
    assert _bits_equal(out[0].cpu().numpy(), exp)
    g.close()
    ctx.close()
