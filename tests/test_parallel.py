"""N>1 path on the CPU: world_size-2 gloo process groups.

Each rank runs a small conv net (ResNet bottleneck shaped: 3x3 conv + ReLU,
1x1 conv + residual Add + ReLU, global pool, FC) on its contiguous batch
slice through the oracle graph runner (CPU stand-in for the device graph),
then BatchShardRunner all-gathers the logits.  The gathered result must be
bit-identical to one process running the whole batch -- items are independent
and sharding must not change any arithmetic.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rten-fork_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from rten_hip.parallel import shard_bounds, shard_sizes  # noqa: E402


def test_shard_bounds_cover_batch():
    for total in (0, 1, 7, 64, 65, 512):
        for world in (1, 2, 3, 4, 8):
            spans = [shard_bounds(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            for (a, b), (c, _) in zip(spans, spans[1:]):
                assert b == c and b >= a
            sizes = shard_sizes(total, world)
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_bounds(4, 2, 2)


def tiny_spec():
    from rten_hip.graph import ModelSpec

    rng = np.random.default_rng(7)
    s = ModelSpec("tiny")
    x = s.value("input")
    s.inputs = [x]
    w1 = s.const("w1", (rng.random((8, 4, 3, 3), dtype=np.float32) - 0.5) * 0.4)
    b1 = s.const("b1", (rng.random(8, dtype=np.float32) - 0.5) * 0.1)
    w2 = s.const("w2", (rng.random((8, 8, 1, 1), dtype=np.float32) - 0.5) * 0.4)
    h = s.op("Conv", [x, w1, b1], {"pads": [1, 1, 1, 1], "strides": [1, 1]})
    h = s.op("Relu", [h])
    r = s.op("Conv", [h, w2], {"pads": [0, 0, 0, 0]})
    h = s.op("Add", [r, h])
    h = s.op("Relu", [h])
    h = s.op("GlobalAveragePool", [h])
    h = s.op("Flatten", [h], {"axis": 1})
    fw = s.const("fc_w", (rng.random((10, 8), dtype=np.float32) - 0.5))
    fb = s.const("fc_b", (rng.random(10, dtype=np.float32) - 0.5) * 0.1)
    out = s.op("Gemm", [h, fw, fb], {"transB": 1})
    s.outputs = [out]
    return s


def _worker(rank, world, port, total, q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import graph_runner
        from rten_hip.parallel import BatchShardRunner

        spec = tiny_spec()
        x = np.random.default_rng(1234).random((total, 4, 6, 6), dtype=np.float32)

        def fn(xb):
            y = graph_runner.run(spec, {"input": xb.numpy()})[spec.outputs[0]]
            return torch.from_numpy(np.ascontiguousarray(y))

        runner = BatchShardRunner(fn)
        a, b = runner.local_slice(total)
        got = runner.run(torch.from_numpy(x[a:b]), total)
        if rank == 0:
            q.put(got.numpy())
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("total", [6, 5])
def test_gloo_world2_matches_single_process(total):
    import torch.multiprocessing as mp

    import graph_runner

    spec = tiny_spec()
    x = np.random.default_rng(1234).random((total, 4, 6, 6), dtype=np.float32)
    expect = graph_runner.run(spec, {"input": x})[spec.outputs[0]]

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, total, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got.shape == expect.shape
    assert (got.view(np.uint32) == np.ascontiguousarray(expect).view(np.uint32)).all()


def _bench_cmd(world, extra=()):
    port = _free_port()
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
            "--steps", "3", "--warmup", "1", "--batch", "5", "--cpu-logic-test", *extra]


def test_bench_world2_launch_logic_gloo():
    """bench.py as the driver launches it for N > 1 (torch.distributed.run, one
    process per rank), with the CPU stand-in forward over gloo: one JSON line
    from rank 0 with n_gpus = world, per-rank step times, the all-gather time,
    and the gathered [world * B, ...] logits."""
    import json
    import subprocess

    r = subprocess.run(_bench_cmd(2, ("--gpus", "2")), capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    js = json.loads(lines[0])
    assert js["n_gpus"] == 2 and js["config"]["global_batch"] == 10
    assert len(js["ranks"]["ms_per_step"]) == 2
    assert js["ms_per_step"] == max(js["ranks"]["ms_per_step"])
    assert js["ranks"]["allgather_us"] > 0
    assert js["gathered_shape"] == [10, 10]


def test_bench_rejects_world_mismatch():
    """--gpus must equal the launched WORLD_SIZE (a driver misconfiguration
    must fail loudly, not print a line for the wrong N)."""
    import subprocess

    r = subprocess.run(_bench_cmd(2, ("--gpus", "4")), capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr + r.stdout
