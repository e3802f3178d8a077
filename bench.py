#!/usr/bin/env python3
"""Benchmark: RTen's f32 operator path on MI355X (BASELINE.json).

Headline: ResNet-50 f32, batch 64 per GPU (BASELINE.json configs[1]; with
N > 1 the batch-sharded configs[4] path), one step = one forward pass through
the device graph executor (librten_hip.so: fused conv epilogues, hipGraph
replay) plus -- for N > 1 -- the RCCL all-gather of every rank's [64, 1000]
logits (the one exchange step of the batch-sharded path).

At N = 1 the same JSON line also carries ``secondary``: the other single-GPU
configurations the metric and BASELINE.json name, each timed the same way in
this run (the reference's CLI times whichever model it is given,
rten-cli/src/main.rs:296-317):
  - ResNet-50 batch 1 (the metric's "batch=1"; replicas only for N > 1),
  - MobileNetV2 batch 128 (configs[2], HBM roofline),
  - BERT-base encoder batch 32, seq 128 (configs[3]).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--model M]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line.  ``value`` = images/s of the whole job (all
ranks' images / max-over-ranks wall time of the K timed steps).  ``roofline``
prices the dominant kernel family (the f32 MFMA implicit-GEMM engine: every
Conv / Gemm / MatMul / FusedAttention launch) by per-op hipEvent times on the
executor's stream over eager runs of the same plan, capped at the replayed
step's wall time (a dominant-kernel time per step cannot exceed the step);
``cpu_baseline`` times the CPU oracle (RTen's algorithm restated in C++,
"port") on a bounded sample of the headline workload on the host.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "rten-fork_amd"))

F32_MFMA_PEAK_TFLOPS = 157.3   # MI355X dense f32 matrix peak (MI355X_MICROARCH.md)
HBM_PEAK_GBPS = 8000.0


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=64, help="images per GPU")
    p.add_argument("--model", default="resnet50", choices=["resnet50", "mobilenet_v2", "bert"])
    p.add_argument("--seq", type=int, default=128, help="BERT sequence length")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-secondary", action="store_true",
                   help="skip the other single-GPU configs (b1, MobileNetV2 b128, BERT b32)")
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--timing-report", action="store_true")
    p.add_argument("--host-input", action="store_true",
                   help="headline with host-resident inputs/outputs (pinned staging, rten_hip/staging.py)")
    p.add_argument("--cpu-logic-test", action="store_true",
                   help="tests only: run the launch / sharding / timing / JSON logic with a torch CPU "
                        "stand-in forward under gloo (no GPU, not a measurement)")
    return p.parse_args()


def _git_head():
    """HEAD of the tree, or the commit __graft_entry__.build() recorded in
    BUILD_COMMIT when the tree arrived without .git (the GPU box)."""
    try:
        head = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                              text=True, timeout=5).stdout.strip()
        if head:
            return head
    except (OSError, subprocess.SubprocessError):
        pass
    try:
        return open(os.path.join(ROOT, "BUILD_COMMIT")).read().split()[0] + " (BUILD_COMMIT)"
    except (OSError, IndexError):
        return None


def _source_commit():
    """The last commit that changed the product sources (__graft_entry__.
    SOURCE_PATHS), or the one build() recorded in BUILD_COMMIT: a committed
    rocprof summary taken at it describes this build's kernels."""
    try:
        from __graft_entry__ import SOURCE_PATHS

        src = subprocess.run(["git", "-C", ROOT, "log", "-1", "--format=%h", "--abbrev=12", "--"] + SOURCE_PATHS,
                             capture_output=True, text=True, timeout=5).stdout.strip()
        if src:
            return src
    except (OSError, ImportError, subprocess.SubprocessError):
        pass
    try:
        parts = open(os.path.join(ROOT, "BUILD_COMMIT")).read().split()
        return parts[1] if len(parts) > 1 else None
    except OSError:
        return None


def cpu_baseline(spec, seconds: float, batch: int, feed_fn):
    """Time the CPU oracle (RTen's CPU algorithm restated in C++: BLIS 6x16
    AVX2-FMA GEMM with the reference's x4 k-unroll and next-B prefetch,
    KC = 256, per-image conv parallelism, VirtualIm2Col offset tables with
    masked gathers) on the benchmark's own config and batch.

    RTen sizes its pool to num_cpus::get_physical() (src/threading.rs:41-62),
    which counts the whole machine's cores, not this process's CPU share: on a
    box leased 16 CPUs of a 128-core host it would start 128 threads on 16
    CPUs.  RTEN_NUM_THREADS (an RTen-supported override) is therefore set to
    the share (OMP_NUM_THREADS when the box sets it, else the logical count)
    and all three counts are reported."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import rten_oracle

    logical, physical = rten_oracle.cpu_counts()
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or logical
    os.environ["RTEN_NUM_THREADS"] = str(min(share, logical))
    threads = rten_oracle.reset_num_threads()
    import graph_runner

    feed = feed_fn()
    graph_runner.run(spec, feed)  # warm-up (also builds the optimized graph)
    times = []
    t_end = time.time() + seconds
    while time.time() < t_end or len(times) < 2:
        t0 = time.perf_counter()
        graph_runner.run(spec, feed)
        times.append(time.perf_counter() - t0)
    times.sort()
    med = times[len(times) // 2]
    # Per-core rate of the oracle's GEMM micro-kernel at the reference's
    # bench_gemm shapes (src/gemm.rs:1782-1903), one thread.
    gflops_1t = gflops_mt = None
    try:
        gflops_1t = round(rten_oracle.gemm_gflops_1t(1024, 1024, 1024, 0.5), 1)
        gflops_mt = round(rten_oracle.gemm_gflops(1024, 1024, 1024, 0.5, threads=threads), 1)
    except Exception:  # noqa: BLE001 -- informative only
        pass
    topo = {}
    try:
        topo = rten_oracle.cpu_topology()
    except Exception:  # noqa: BLE001 -- informative only
        pass
    cpu_model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    unit = "sequences/s" if spec.name.startswith("bert") else "images/s"
    return {
        "value": round(batch / med, 3),
        "unit": unit,
        "cores": threads,
        "kind": "port",
        "logical_cpus": logical,
        "physical_cores": physical,
        "gemm_gflops_per_core": gflops_1t,
        "gemm_gflops_all_threads": gflops_mt,
        "topology": topo,
        "sample": f"{spec.name} batch {batch} (the benchmark config), {len(times)} runs in ~{seconds:.0f}s, "
                  f"median {med * 1e3:.1f} ms per batch; restated RTen algorithm (C++ BLIS 6x16 "
                  f"AVX2-FMA with x4 unroll + B prefetch, KC=256, im2col offset tables + masked gathers), "
                  f"not the Rust binary; {threads} threads (RTEN_NUM_THREADS = the box's CPU share; RTen's own "
                  f"rule, num_cpus::get_physical(), would start {physical} on this {logical}-CPU lease); "
                  f"GEMM 1024^3: {gflops_1t} GFLOP/s on 1 thread, {gflops_mt} GFLOP/s on {threads} "
                  f"({(gflops_mt or 0) / max(gflops_1t or 1, 1e-9):.1f}x); the {topo.get('affinity_cpus')} "
                  f"CPUs of this lease are {topo.get('physical_cores_in_affinity')} physical cores "
                  f"(SMT {'on' if topo.get('smt_active') else 'off' if topo.get('smt_active') is False else 'unknown'}); "
                  f"host: {cpu_model}",
    }


# Kernel families the roofline's dominant-kernel time covers, per model (the
# ops bench.py sums: Conv / Gemm / MatMul / FusedAttention).
_ROOF_KERNELS = {
    "resnet50": ("gemm_dma_kernel", "gemm_lat", "gemv", "conv_stem_kernel", "conv_pair_kernel"),
    "bert": ("gemm_dma_kernel", "pack_a_kernel", "attention_kernel"),
    "mobilenet_v2": ("gemm_dma_kernel", "gemm_lat", "gemv", "conv_pw_valu_kernel", "conv_direct",
                     "depthwise", "dw_stream_kernel", "expand_dw_kernel", "dw_project_kernel", "conv_stem_kernel"),
}


def traffic_bytes(model, batch, all_kernels=False):
    """HBM bytes per step of the roofline's kernels, from the newest committed
    rocprofv3 PMC summary of this workload (scripts/gpu_prof.sh ->
    tools/pmc_traffic.py --marker): FETCH_SIZE x2 (gfx950) + WRITE_SIZE,
    eager forwards.  (None, None) when no summary exists for this workload."""
    for rnd in ("r6", "r5", "r4", "r3"):
        path = os.path.join(ROOT, "profiles", f"{rnd}_pmc_traffic_{model}_b{batch}.json")
        if not os.path.exists(path):
            continue
        try:
            js = json.load(open(path))
            by = js["by_kernel"]
        except (OSError, ValueError, KeyError):
            continue
        fams = _ROOF_KERNELS[model]
        if all_kernels:
            return round(js.get("all_kernels_bytes_per_forward") or sum(by.values())), path
        return round(sum(v for k, v in by.items() if any(f in k for f in fams))), \
            f"profiles/{os.path.basename(path)} (commit {js.get('commit', 'unrecorded')})"
    return None, None


def rocprof_kernel_ms(model, batch):
    """Dominant-kernel time per forward from the newest committed rocprofv3
    per-forward summary of this workload (scripts/gpu_evidence.sh ->
    tools/rocprof_per_forward.py): the sum of the _ROOF_KERNELS families'
    ms/forward, the commit the summary was taken at, and its path.  None when
    no summary exists."""
    import re

    for rnd in ("r6", "r5", "r4"):
        path = os.path.join(ROOT, "profiles", f"{rnd}_rocprof_{model}_b{batch}_per_forward.txt")
        if not os.path.exists(path):
            continue
        commit, ms = None, 0.0
        for line in open(path):
            if line.startswith("# commit"):
                commit = line.split()[2]
            m = re.match(r"\s+(\S+)\s+([0-9.]+) ms/forward", line)
            if m and any(f in m.group(1) for f in _ROOF_KERNELS[model]):
                ms += float(m.group(2))
        if ms > 0:
            return {"kernel_ms_per_step": round(ms, 4), "commit": commit,
                    "source": f"profiles/{os.path.basename(path)}"}
    return None


class Workload:
    """One configuration on the device graph: builds the spec and its
    synthetic inputs, plans + tunes it on the first run, then steps it."""

    def __init__(self, ctx, model, B, seq, rank, world, backend):
        import numpy as np
        import torch

        from rten_hip import models

        self.model, self.B, self.seq, self.world, self.backend = model, B, seq, world, backend
        rng = np.random.default_rng(1234 + rank)
        if model == "bert":
            # rten-cli's inputs for a BERT .rten (rten-cli/src/main.rs:250-259):
            # *_ids -> zeros, *_mask -> ones; the embedding Gathers and the mask
            # subgraph run inside the timed step.
            self.spec = models.bert_encoder(seq=seq, embeddings=True)
            self.flops_per_img = models.bert_flops(seq=seq)
            self.feed_np = {"input_ids": np.zeros((B, seq), np.int32),
                            "token_type_ids": np.zeros((B, seq), np.int32),
                            "attention_mask": np.ones((B, seq), np.int32)}
        else:
            self.spec = models.resnet50() if model == "resnet50" else models.mobilenet_v2()
            self.flops_per_img = models.conv_flops(self.spec, 1)
            self.feed_np = {"input": rng.random((B, 3, 224, 224), dtype=np.float32)}
        self.io_bytes = models.conv_io_bytes(self.spec, B) if model == "mobilenet_v2" else None
        g = self.g = self.spec.to_graph(ctx)
        if model == "bert":
            # The embedding Gathers check their indices on the device; a run
            # normally waits for that check (Model::run returns the error).
            # Queued back to back, the check of every step is collected at the
            # end of the timed region instead (sync() -> rtenhip_graph_synchronize
            # raises any index error), so the GPU is not idle between steps.
            g.set_deferred_checks(True)
        dev = [torch.from_numpy(self.feed_np[n]).cuda() for n in self.spec.inputs]
        self.x = dev[0]
        self.extra = {g.input_ids[i]: dev[i] for i in range(1, len(dev))}
        (self.out,) = g.run({g.input_ids[0]: self.x, **self.extra}, g.output_ids)  # plans + tunes

        from rten_hip.parallel import BatchShardRunner

        def forward(xb):
            g.run({g.input_ids[0]: xb, **self.extra}, g.output_ids, out=[self.out])
            return self.out

        # Rank r holds images [r*B, (r+1)*B) of the world*B job; the only
        # exchange is the all-gather of logits (RCCL) inside runner.run.
        self.runner = BatchShardRunner(forward)
        self.staging = None

    def step(self):
        self.runner.run(self.x, self.world * self.B)

    def enable_host_input(self):
        """Host-resident inputs and outputs (the drop-in Model::run case,
        src/model.rs:580-592): every step uploads this rank's images from
        pinned host memory and downloads the (gathered) logits, pipelined by
        rten_hip/staging.py -- step k+1's upload overlaps step k's forward."""
        import torch

        from rten_hip.staging import HostStaging

        if self.extra:
            raise ValueError("host-input mode covers single-input image models")
        g = self.g
        total = self.world * self.B
        if self.world == 1:
            # Through the C ABI (rtenhip_graph_run_host / rtenhip_graph_wait,
            # csrc/graph_io.cpp): pinned host arrays in and out, the staging
            # pipeline inside librten_hip.so -- what a Rust Model::run caller
            # binds.  No torch tensor is involved in the step.
            from rten_hip.host import pinned

            self.host_in = pinned(self.feed_np["input"].shape)
            self.host_in[...] = self.feed_np["input"]
            out_shape = tuple(self.out.shape)
            self.host_out = [pinned(out_shape), pinned(out_shape)]
            self.k_host = 0
            self.capi_host = True
            return
        outs = [self.out, torch.empty_like(self.out)]

        def fwd(xb, slot):
            g.run({g.input_ids[0]: xb}, g.output_ids, out=[outs[slot]])
            return self.runner.gather(outs[slot], total)

        self.staging = HostStaging(fwd, tuple(self.x.shape), self.x.device, slots=2)
        self.host_in = torch.from_numpy(self.feed_np["input"]).pin_memory()
        out_shape = (total,) + tuple(self.out.shape[1:])
        self.host_out = [HostStaging.pinned(out_shape), HostStaging.pinned(out_shape)]
        self.k_host = 0

    def host_step(self):
        if getattr(self, "capi_host", False):
            g = self.g
            g.run_host({g.input_ids[0]: self.host_in}, g.output_ids, [self.host_out[self.k_host % 2]])
        else:
            self.staging.submit(self.host_in, self.host_out[self.k_host % 2])
        self.k_host += 1

    def sync(self):
        import torch

        if getattr(self, "capi_host", False):
            self.g.wait()
        if self.staging is not None:
            self.staging.synchronize()
        self.g.synchronize()  # (raises a deferred Gather index error)
        torch.cuda.synchronize()

    def timed(self, steps, warmup, dist, host=False):
        """Wall time of `steps` steps between barriers: the max over ranks,
        and every rank's own time (rank order)."""
        import torch

        step = self.host_step if host else self.step
        for _ in range(warmup):
            step()
        self.sync()
        if dist is not None:
            dist.barrier()
        self.sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        self.sync()
        if dist is not None:
            dist.barrier()
        self.sync()
        elapsed = time.perf_counter() - t0
        per_rank = [elapsed]
        if dist is not None:
            dev = self.x.device if self.backend == "nccl" else "cpu"
            t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
            parts = [torch.zeros_like(t) for _ in range(self.world)]
            dist.all_gather(parts, t)
            per_rank = [float(p.item()) for p in parts]
        return max(per_rank), per_rank

    def gather_us(self, reps, dist):
        """Mean time of the logits all-gather alone (µs, max over ranks);
        None with one rank."""
        import torch

        if dist is None:
            return None
        total = self.world * self.B
        self.runner.gather(self.out, total)
        self.sync()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            self.runner.gather(self.out, total)
        self.sync()
        us = (time.perf_counter() - t0) / reps * 1e6
        t = torch.tensor([us], device=self.x.device if self.backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return round(float(t.item()), 1)

    def kernel_ms(self, runs):
        """Per-op hipEvent time of the dominant family per step (eager runs of
        the same plan, events on the executor's stream), and the report."""
        import torch

        g = self.g
        g.set_timing(True)
        ms, report = 0.0, ""
        self.hold_timeouts = 0
        for _ in range(runs):
            g.run({g.input_ids[0]: self.x, **self.extra}, g.output_ids, out=[self.out])
            torch.cuda.synchronize()
            report = g.timing_report()
            # (the stream hold gave up before the plan was queued: that run's
            # event pairs include host launch time, graph.cpp launch_hold)
            self.hold_timeouts += "hold timed out" in report.splitlines()[0]
            for line in report.splitlines()[1:]:
                name = line.split()[0]
                if name.startswith(("Conv", "MatMul", "FusedAttention", "Gemm")):
                    ms += float(line.split()[1])
        g.set_timing(False)
        self.report = report
        return ms / runs, report

    def describe(self):
        B, model = self.B, self.model
        if model == "bert":
            workload = (f"{self.spec.name} encoder f32 batch={B} per GPU, seq {self.seq}, hidden 768, "
                        f"12 heads, FFN 3072, embeddings + mask subgraph (BASELINE.json configs[3])")
            kernel_desc = "MatMul GEMM launches (gemm_dma_kernel) + FusedAttention"
            data = ("synthetic (rten-cli inputs: input_ids / token_type_ids zeros, attention_mask ones, "
                    "resident in HBM; seeded U(+-0.05) weights)")
            metric = "sequences/sec BERT-base encoder f32"
        else:
            if model == "mobilenet_v2":
                cfg = "BASELINE.json configs[2]"
            elif B == 64:
                cfg = "BASELINE.json configs[1]" if self.world == 1 else "BASELINE.json configs[4]: 64 per GPU"
            elif B == 1:
                cfg = "BASELINE.json metric batch=1 on the GPU path; replicas only for N > 1"
            else:
                cfg = "not a BASELINE.json config"
            workload = f"{self.spec.name} f32 batch={B} per GPU, 224x224 NCHW, BN folded ({cfg})"
            kernel_desc = ("all Conv launches (DMA / latency implicit GEMM) + FC Gemm" if model == "resnet50"
                           else "all Conv launches (DMA GEMM / VALU pointwise / depthwise) + FC Gemm")
            data = "synthetic (U[0,1) images resident in HBM; seeded He-uniform weights)"
            metric = ({"resnet50": f"images/sec ResNet-50 f32 batch={B} per GPU",
                       "mobilenet_v2": "images/sec MobileNetV2 f32"})[model]
        return metric, workload, kernel_desc, data

    def fused_io_bytes(self, report):
        """Algorithmic HBM bytes of one ResNet step as the executor fused it:
        models.conv_io_bytes (each conv / pool reads its input and weights and
        writes its output once, fused residual reads once) minus what the
        fused kernels the plan took never move -- a dual conv3 + downsample
        GEMM neither writes nor re-reads the downsample output (2 x M x N
        floats), a conv3 -> conv1 pair kernel reads conv1's input from LDS (K1
        x N floats), the stem + MaxPool kernel never writes the stem's output
        (2 x its floats: the write and the pool's read).  Parsed from the plan's per-op report lines."""
        import re

        from rten_hip import models

        total = models.conv_io_bytes(self.spec, self.B)
        for line in report.splitlines():
            m = re.search(r"  dual M=(\d+) N=(\d+) K=(\d+)\+(\d+)", line)
            if m:
                # the downsample's M equals conv3's (both produce the residual sum's operands)
                total -= 2 * 4.0 * int(m.group(1)) * int(m.group(2))
            m = re.search(r"  pair conv3 M=(\d+) K=(\d+) \+ conv1 M=(\d+) K=(\d+) N=(\d+)", line)
            if m:
                total -= 4.0 * int(m.group(4)) * int(m.group(5))
            m = re.search(r"  stem\+pool M=\d+ N=\d+ K=\d+ stem_out=(\d+)", line)
            if m:
                # the stem's output is neither written nor read back by the pool
                total -= 2 * 4.0 * int(m.group(1))
        return total

    def roofline(self, kernel_ms_eager, ms_per_step, value):
        # The eager per-op event pairs bracket each op's launches (the stream
        # is held until the whole plan is queued, graph.cpp launch_hold, so
        # host launch pace is not in them, but each pair still spans its
        # op's dispatch); when their sum exceeds the replayed step the step
        # time is used instead and the line says so ("capped").
        capped = kernel_ms_eager > ms_per_step
        kms = min(kernel_ms_eager, ms_per_step)
        _, _, kernel_desc, _ = self.describe()
        gemm_flops = self.flops_per_img * self.B
        achieved = gemm_flops / (kms * 1e-3) / 1e12 if kms > 0 else 0.0
        traffic, traffic_src = traffic_bytes(self.model, self.B)
        common = {"traffic": traffic, "traffic_source": traffic_src, "kernel": kernel_desc,
                  "kernel_ms_per_step": round(kms, 4), "kernel_ms_eager_events": round(kernel_ms_eager, 4),
                  "capped": capped, "hold_timeouts": getattr(self, "hold_timeouts", 0),
                  "timing": "per-op hipEvents on the executor stream over eager runs (stream held until the "
                            "plan is queued), capped at ms_per_step when larger (capped: true)"}
        rp = rocprof_kernel_ms(self.model, self.B)
        if rp:
            # (the summary's commit vs the last commit that changed the sources)
            head = _source_commit() or ""
            rp["matches_head"] = bool(head and rp["commit"] and (head.startswith(rp["commit"]) or
                                                                 rp["commit"].startswith(head)))
            if self.model == "mobilenet_v2":
                rp["achieved_gbs"] = round(self.io_bytes / (rp["kernel_ms_per_step"] * 1e-3) / 1e9, 1)
                rp["frac"] = round(rp["achieved_gbs"] / HBM_PEAK_GBPS, 4)
            else:
                rp["achieved"] = round(gemm_flops / (rp["kernel_ms_per_step"] * 1e-3) / 1e12, 2)
                rp["frac"] = round(rp["achieved"] / F32_MFMA_PEAK_TFLOPS, 4)
            common["rocprof"] = rp
        if self.model == "mobilenet_v2":
            gbs = self.io_bytes / (kms * 1e-3) / 1e9 if kms > 0 else 0.0
            return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(gbs / HBM_PEAK_GBPS, 4), "bytes_per_step": self.io_bytes,
                    "mfma_tflops": round(achieved, 2), **common}
        if self.model == "resnet50" and getattr(self, "report", ""):
            # All kernels' PMC bytes (pooling included, as in the algorithmic
            # figure) over the fused path's algorithmic bytes.
            io = self.fused_io_bytes(self.report)
            all_bytes = traffic_bytes(self.model, self.B, all_kernels=True)[0]
            common["bytes_per_step"] = round(io)
            common["traffic_all_kernels"] = all_bytes
            common["traffic_ratio"] = round(all_bytes / io, 3) if all_bytes else None
        return {"bound": "mfma", "achieved": round(achieved, 2), "peak": F32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / F32_MFMA_PEAK_TFLOPS, 4), "flops_per_step": gemm_flops,
                "model_frac": round(value / self.world * self.flops_per_img / 1e12 / F32_MFMA_PEAK_TFLOPS, 4),
                **common}


def secondary_entry(ctx, model, B, seq, steps, warmup, cpu_seconds=0.0):
    """One extra single-GPU configuration, timed like the headline: W warmup
    steps, then K steps between synchronisations (K raised so the timed
    region is >= ~0.15 s for short steps)."""
    w = Workload(ctx, model, B, seq, 0, 1, "nccl")
    est = w.timed(3, 1, None)[0] / 3
    k = max(steps, min(2000, int(0.15 / max(est, 1e-5))))
    elapsed, _ = w.timed(k, warmup, None)
    ms = elapsed / k * 1e3
    value = B * k / elapsed
    kms, _ = w.kernel_ms(max(1, min(steps, 10)))
    metric, workload, _, _ = w.describe()
    ent = {"metric": metric, "value": round(value, 2),
           "unit": "sequences/s" if model == "bert" else "images/s",
           "ms_per_step": round(ms, 4), "steps": k, "warmup": warmup, "dtype": "f32",
           "config": {"workload": workload, "model": w.spec.name, "global_batch": B,
                      "seq_len": seq if model == "bert" else None},
           "roofline": w.roofline(kms, ms, value)}
    if cpu_seconds > 0:
        # BASELINE.json configs[0]: the same batch-1 model on RTen's CPU path
        # (the restated algorithm, timed like the headline's cpu_baseline),
        # next to the GPU figure (rten-cli/src/main.rs:296-317 times one
        # Model::run per iteration).
        ent["cpu_baseline"] = cpu_baseline(w.spec, cpu_seconds, B, lambda: w.feed_np)
    del w
    return ent


def host_input_entry(ctx, steps, warmup, headline_ms):
    """ResNet-50 b64 with host-resident inputs and outputs (pinned staging,
    rten_hip/staging.py), timed like the headline, with the PCIe copy rates
    measured in the same run at the staging sizes."""
    from rten_hip.staging import pcie_rates

    w = Workload(ctx, "resnet50", 64, 128, 0, 1, "nccl")
    w.enable_host_input()
    elapsed, _ = w.timed(steps, warmup, None, host=True)
    ms = elapsed / steps * 1e3
    pcie = pcie_rates(w.host_in.size * 4, w.host_out[0].size * 4, w.x.device)
    ent = {"metric": "images/sec ResNet-50 f32 batch=64, host-resident input and logits",
           "value": round(64 * steps / elapsed, 2), "unit": "images/s", "ms_per_step": round(ms, 4),
           "steps": steps, "warmup": warmup, "dtype": "f32",
           "config": {"workload": "resnet50 f32 batch=64, images in pinned host memory (rtenhip_host_alloc) "
                                  "uploaded every step (38.5 MB H2D on the library's copy stream, overlapped with "
                                  "the previous step's forward), logits downloaded every step (256 KB D2H); the "
                                  "drop-in Model::run case (src/model.rs:580-592) through the C ABI "
                                  "(rtenhip_graph_run_host / rtenhip_graph_wait)", "model": w.spec.name,
                      "global_batch": 64},
           "entry": "rtenhip_graph_run_host",
           "pcie": pcie,
           "vs_device_resident": round(headline_ms / ms, 4) if headline_ms else None}
    del w
    return ent


class CpuLogicWorkload:
    """--cpu-logic-test only: the N>1 launch / shard / timing / JSON logic with
    a torch CPU stand-in forward (a small conv net) under gloo.  Not a
    measurement of anything; no GPU and no rten_hip involved."""

    def __init__(self, B, rank, world):
        import torch

        self.B, self.world, self.backend, self.model = B, world, "gloo", "resnet50"
        torch.manual_seed(1234 + rank)
        self.x = torch.rand(B, 3, 32, 32)
        self.wc = torch.rand(8, 3, 3, 3) - 0.5
        self.wf = torch.rand(10, 8) - 0.5
        self.staging = None

        from rten_hip.parallel import BatchShardRunner

        def forward(xb):
            h = torch.relu(torch.nn.functional.conv2d(xb, self.wc, padding=1))
            return h.mean(dim=(2, 3)) @ self.wf.t()

        self.out = forward(self.x)
        self.runner = BatchShardRunner(forward)

    step = Workload.step
    timed = Workload.timed
    gather_us = Workload.gather_us

    def sync(self):
        pass


def device_identity(local):
    """Host name and GPU identity of this rank's device (UUID where torch
    exposes it), for the one-rank-per-GPU check."""
    import socket

    import torch

    ident = None
    try:
        props = torch.cuda.get_device_properties(local)
        ident = str(getattr(props, "uuid", "") or "") or f"{getattr(props, 'name', 'gpu')}#{local}"
    except Exception:  # noqa: BLE001
        ident = f"gpu#{local}"
    return f"{socket.gethostname()}/{ident}"


def main():
    args = parse()
    if args.cpu_logic_test:
        return cpu_logic_main(args)
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    check_world(args, world)
    dist = None
    backend = os.environ.get("RTENHIP_DIST_BACKEND", "nccl")  # "gloo": one-GPU multi-rank rehearsal
    if world > 1:
        import torch.distributed as dist

        # One rank per GPU; with fewer GPUs than ranks (a gloo rehearsal on a
        # one-GPU box) ranks share devices round-robin.
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)

    devices = [device_identity(local)]
    if dist is not None:
        devices = [None] * world
        dist.all_gather_object(devices, device_identity(local))
        if backend == "nccl" and len(set(devices)) != world:
            raise SystemExit(f"bench.py: ranks share a GPU ({devices}); one rank per GPU is required")

    import rten_hip

    ctx = rten_hip.Context(torch.cuda.current_device())
    # One stream for the whole step: the graph executor runs on the stream the
    # steps are issued from (rtenhip_set_exec_stream), so consecutive runs are
    # not separated by cross-stream event round trips.
    step_stream = torch.cuda.Stream()
    torch.cuda.set_stream(step_stream)
    ctx.use_stream(step_stream)
    w = Workload(ctx, args.model, args.batch, args.seq, rank, world, backend)
    if args.host_input:
        w.enable_host_input()
    elapsed, per_rank = w.timed(args.steps, args.warmup, dist, host=args.host_input)
    ms_per_step = elapsed / args.steps * 1e3
    value = world * args.batch * args.steps / elapsed
    gather_us = w.gather_us(max(5, args.steps), dist)
    kms, report = w.kernel_ms(max(1, min(args.steps, 10)))
    roofline = w.roofline(kms, ms_per_step, value)
    metric, workload, _, data = w.describe()
    if args.host_input:
        data = data.replace("resident in HBM", "in pinned host memory, uploaded every step")

    if rank == 0:
        line = {
            "metric": metric,
            "value": round(value, 2),
            "unit": "sequences/s" if args.model == "bert" else "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": data,
            "config": {"workload": workload,
                       "model": w.spec.name, "global_batch": world * args.batch,
                       "seq_len": args.seq if args.model == "bert" else None,
                       "parallelism": f"batch-shard x{world} (replicated weights, "
                                          f"{'RCCL' if backend == 'nccl' else backend} all-gather of logits)"},
            "roofline": roofline,
            "ranks": {"ms_per_step": [round(t / args.steps * 1e3, 4) for t in per_rank],
                      "devices": devices, "allgather_us": gather_us},
            "commit": _git_head(),
        }
        if world == 1 and not args.no_secondary and args.model == "resnet50" and args.batch == 64 \
                and not args.host_input:
            sec = []
            for model, B in (("resnet50", 1), ("mobilenet_v2", 128), ("bert", 32)):
                try:
                    cpu_s = 6.0 if (model, B) == ("resnet50", 1) and not args.no_cpu_baseline else 0.0
                    sec.append(secondary_entry(ctx, model, B, args.seq, args.steps, args.warmup, cpu_s))
                except Exception as e:  # noqa: BLE001 -- reported in the line, never hides the headline
                    sec.append({"model": model, "batch": B, "error": f"{type(e).__name__}: {e}"})
            try:
                sec.append(host_input_entry(ctx, args.steps, args.warmup, ms_per_step))
            except Exception as e:  # noqa: BLE001
                sec.append({"model": "resnet50", "batch": 64, "host_input": True,
                            "error": f"{type(e).__name__}: {e}"})
            line["secondary"] = sec
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(w.spec, args.cpu_seconds, args.batch, lambda: w.feed_np)
        if args.timing_report:
            sys.stderr.write(report + "\n")
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def check_world(args, world):
    """bench.py --gpus N runs as N ranks, one per GPU (the driver launches it
    under torch.distributed.run); anything else is a launch error."""
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch N > 1 as "
                         f"python -m torch.distributed.run --nproc-per-node {args.gpus} --master-addr 127.0.0.1 "
                         f"bench.py --gpus {args.gpus}")


def cpu_logic_main(args):
    """--cpu-logic-test: the same world checks, barriers, max-over-ranks
    timing, per-rank fields and all-gather timing as main(), over gloo with a
    CPU stand-in forward.  Prints one JSON line marked as a logic test."""
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    check_world(args, world)
    d = None
    if world > 1:
        dist.init_process_group("gloo")
        d = dist
    w = CpuLogicWorkload(args.batch, rank, world)
    elapsed, per_rank = w.timed(args.steps, args.warmup, d)
    gather_us = w.gather_us(max(5, args.steps), d)
    gathered = w.runner.run(w.x, world * args.batch)
    if rank == 0:
        print(json.dumps({
            "metric": "logic test (CPU stand-in forward, gloo): not a measurement",
            "value": round(world * args.batch * args.steps / elapsed, 2), "unit": "images/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic, CPU stand-in forward",
            "config": {"workload": "cpu logic test", "global_batch": world * args.batch,
                       "parallelism": f"batch-shard x{world} (gloo all-gather of logits)"},
            "ranks": {"ms_per_step": [round(t / args.steps * 1e3, 4) for t in per_rank],
                      "allgather_us": gather_us},
            "gathered_shape": list(gathered.shape),
        }), flush=True)
    if d is not None:
        d.barrier()
        d.destroy_process_group()


if __name__ == "__main__":
    main()
