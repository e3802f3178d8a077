"""RTen's thread-count semantics (src/threading.rs:41-62, num_cpus 1.16):
the pool is the physical core count, or RTEN_NUM_THREADS clamped to
[1, logical].  The count changes results only through the gemv column blocks
(src/gemm.rs:676: ceil(N / threads), at least 128), so the batch-1 FC layer is
checked bit-exact at thread counts that give different blockings.
"""
import os

import numpy as np
import pytest


def _num_cpus():
    """Independent restatement of num_cpus::get / get_physical on Linux."""
    logical = len(os.sched_getaffinity(0))
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            logical = min(logical, -(-int(q) // int(p)))
    except (OSError, ValueError):
        pass
    per_socket, pid, cores, seen = {}, 0, 0, 0
    for line in open("/proc/cpuinfo"):
        if ":" not in line:
            continue
        k, v = (t.strip() for t in line.split(":", 1))
        if k == "physical id":
            pid, seen = int(v), seen + 1
        elif k == "cpu cores":
            cores, seen = int(v), seen + 1
        if seen == 2:
            per_socket[pid], seen = cores, 0
    return max(1, logical), (sum(per_socket.values()) or max(1, logical))


def test_cpu_counts_match_num_cpus(oracle):
    import rten_hip

    assert rten_hip.cpu_counts() == _num_cpus()
    assert oracle.cpu_counts() == _num_cpus()


@pytest.mark.parametrize("val,expect", [("1", "1"), ("3", "3"), ("0", "1"), ("100000", "logical"),
                                        ("+2", "2"), ("x", "physical"), ("-1", "physical"), ("", "physical")])
def test_oracle_thread_count_rule(oracle, monkeypatch, val, expect):
    logical, physical = _num_cpus()
    monkeypatch.setenv("RTEN_NUM_THREADS", val)
    try:
        n = oracle.reset_num_threads()
        want = {"logical": logical, "physical": physical}.get(expect)
        assert n == (want if want is not None else min(int(expect), logical))
    finally:
        monkeypatch.setenv("RTEN_NUM_THREADS", os.environ.get("RTEN_NUM_THREADS", "8"))
    monkeypatch.undo()
    oracle.reset_num_threads()


@pytest.mark.gpu
@pytest.mark.parametrize("val", ["1", "3", "8", "100000"])
def test_batch1_fc_bitexact_per_thread_count(oracle, monkeypatch, val):
    """ResNet-50's classifier at batch 1 (gemv, transposed B) with the context
    and the oracle resolving the same RTEN_NUM_THREADS."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import rten_hip

    monkeypatch.setenv("RTEN_NUM_THREADS", val)
    n_or = oracle.reset_num_threads()
    ctx = rten_hip.Context(0)
    try:
        assert ctx.num_threads == n_or
        rng = np.random.default_rng(int(val) % 1000)
        x = rng.random((1, 2048), dtype=np.float32)
        w = rng.uniform(-0.05, 0.05, (1000, 2048)).astype(np.float32)
        c = rng.uniform(-0.01, 0.01, (1000,)).astype(np.float32)
        exp = oracle.gemm_op(x, w, c, 1.0, 1.0, False, True)
        got = rten_hip.gemm_op(torch.from_numpy(x).cuda(), torch.from_numpy(w).cuda(),
                               torch.from_numpy(c).cuda(), 1.0, 1.0, False, True, ctx=ctx)
        torch.cuda.synchronize()
        got = got.cpu().numpy()
        assert np.array_equal(got.view(np.uint32), exp.view(np.uint32))
    finally:
        ctx.close()
        monkeypatch.undo()
        oracle.reset_num_threads()
