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
        return open(os.path.join(ROOT, "BUILD_COMMIT")).read().strip() + " (BUILD_COMMIT)"
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
    gflops_1t = None
    try:
        gflops_1t = round(rten_oracle.gemm_gflops_1t(1024, 1024, 1024, 0.5), 1)
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
        "sample": f"{spec.name} batch {batch} (the benchmark config), {len(times)} runs in ~{seconds:.0f}s, "
                  f"median {med * 1e3:.1f} ms per batch; restated RTen algorithm (C++ BLIS 6x16 "
                  f"AVX2-FMA with x4 unroll + B prefetch, KC=256, im2col offset tables + masked gathers), "
                  f"not the Rust binary; {threads} threads (RTEN_NUM_THREADS = the box's CPU share; RTen's own "
                  f"rule, num_cpus::get_physical(), would start {physical} on this {logical}-CPU lease); "
                  f"1-thread GEMM 1024^3: {gflops_1t} GFLOP/s; host: {cpu_model}",
    }


# Kernel families the roofline's dominant-kernel time covers, per model (the
# ops bench.py sums: Conv / Gemm / MatMul / FusedAttention).
_ROOF_KERNELS = {
    "resnet50": ("gemm_dma_kernel", "gemm_lat", "gemv"),
    "bert": ("gemm_dma_kernel", "pack_a_kernel", "attention_kernel"),
    "mobilenet_v2": ("gemm_dma_kernel", "gemm_lat", "gemv", "conv_pw_valu_kernel", "conv_direct",
                     "depthwise", "expand_dw_kernel"),
}


def traffic_bytes(model, batch):
    """HBM bytes per step of the roofline's kernels, from the newest committed
    rocprofv3 PMC summary of this workload (scripts/gpu_prof.sh ->
    tools/pmc_traffic.py --marker): FETCH_SIZE x2 (gfx950) + WRITE_SIZE,
    eager forwards.  (None, None) when no summary exists for this workload."""
    for rnd in ("r4", "r3"):
        path = os.path.join(ROOT, "profiles", f"{rnd}_pmc_traffic_{model}_b{batch}.json")
        if not os.path.exists(path):
            continue
        try:
            js = json.load(open(path))
            by = js["by_kernel"]
        except (OSError, ValueError, KeyError):
            continue
        fams = _ROOF_KERNELS[model]
        return round(sum(v for k, v in by.items() if any(f in k for f in fams))), \
            f"profiles/{os.path.basename(path)} (commit {js.get('commit', 'unrecorded')})"
    return None, None


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

    def step(self):
        self.runner.run(self.x, self.world * self.B)

    def timed(self, steps, warmup, dist):
        import torch

        for _ in range(warmup):
            self.step()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            self.step()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([elapsed], device=self.x.device if self.backend == "nccl" else "cpu",
                             dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        return elapsed

    def kernel_ms(self, runs):
        """Per-op hipEvent time of the dominant family per step (eager runs of
        the same plan, events on the executor's stream), and the report."""
        import torch

        g = self.g
        g.set_timing(True)
        ms, report = 0.0, ""
        for _ in range(runs):
            g.run({g.input_ids[0]: self.x, **self.extra}, g.output_ids, out=[self.out])
            torch.cuda.synchronize()
            report = g.timing_report()
            for line in report.splitlines()[1:]:
                name = line.split()[0]
                if name.startswith(("Conv", "MatMul", "FusedAttention")) or name == "Gemm":
                    ms += float(line.split()[1])
        g.set_timing(False)
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

    def roofline(self, kernel_ms_eager, ms_per_step, value):
        kms = min(kernel_ms_eager, ms_per_step)
        _, _, kernel_desc, _ = self.describe()
        gemm_flops = self.flops_per_img * self.B
        achieved = gemm_flops / (kms * 1e-3) / 1e12 if kms > 0 else 0.0
        traffic, traffic_src = traffic_bytes(self.model, self.B)
        common = {"traffic": traffic, "traffic_source": traffic_src, "kernel": kernel_desc,
                  "kernel_ms_per_step": round(kms, 4), "kernel_ms_eager_events": round(kernel_ms_eager, 4),
                  "timing": "per-op hipEvents on the executor stream over eager runs, capped at ms_per_step"}
        if self.model == "mobilenet_v2":
            gbs = self.io_bytes / (kms * 1e-3) / 1e9 if kms > 0 else 0.0
            return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(gbs / HBM_PEAK_GBPS, 4), "bytes_per_step": self.io_bytes,
                    "mfma_tflops": round(achieved, 2), **common}
        return {"bound": "mfma", "achieved": round(achieved, 2), "peak": F32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / F32_MFMA_PEAK_TFLOPS, 4), "flops_per_step": gemm_flops,
                "model_frac": round(value / self.world * self.flops_per_img / 1e12 / F32_MFMA_PEAK_TFLOPS, 4),
                **common}


def secondary_entry(ctx, model, B, seq, steps, warmup):
    """One extra single-GPU configuration, timed like the headline: W warmup
    steps, then K steps between synchronisations (K raised so the timed
    region is >= ~0.15 s for short steps)."""
    w = Workload(ctx, model, B, seq, 0, 1, "nccl")
    est = w.timed(3, 1, None) / 3
    k = max(steps, min(2000, int(0.15 / max(est, 1e-5))))
    elapsed = w.timed(k, warmup, None)
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
    del w
    return ent


def main():
    args = parse()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
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

    import rten_hip

    ctx = rten_hip.Context(torch.cuda.current_device())
    w = Workload(ctx, args.model, args.batch, args.seq, rank, world, backend)
    elapsed = w.timed(args.steps, args.warmup, dist)
    ms_per_step = elapsed / args.steps * 1e3
    value = world * args.batch * args.steps / elapsed
    kms, report = w.kernel_ms(max(1, min(args.steps, 10)))
    roofline = w.roofline(kms, ms_per_step, value)
    metric, workload, _, data = w.describe()

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
            "commit": _git_head(),
        }
        if world == 1 and not args.no_secondary and args.model == "resnet50" and args.batch == 64:
            sec = []
            for model, B in (("resnet50", 1), ("mobilenet_v2", 128), ("bert", 32)):
                try:
                    sec.append(secondary_entry(ctx, model, B, args.seq, args.steps, args.warmup))
                except Exception as e:  # noqa: BLE001 -- reported in the line, never hides the headline
                    sec.append({"model": model, "batch": B, "error": f"{type(e).__name__}: {e}"})
            line["secondary"] = sec
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(w.spec, args.cpu_seconds, args.batch, lambda: w.feed_np)
        if args.timing_report:
            sys.stderr.write(report + "\n")
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
