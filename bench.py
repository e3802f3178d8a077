#!/usr/bin/env python3
"""Benchmark: ResNet-50 f32 inference throughput on MI355X (BASELINE.json).

One step = one forward pass of ResNet-50 (f32, batch 64 per GPU, synthetic
input resident in HBM) through the device graph executor
(librten_hip.so: fused conv epilogues, hipGraph replay), plus — for N > 1 —
the RCCL all-gather of every rank's [64, 1000] logits (the one exchange step
of the batch-sharded path).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line.  ``value`` = images/s of the whole job (all
ranks' images / max-over-ranks wall time of the K timed steps).  The
``roofline`` object prices the dominant kernel (the f32 MFMA implicit-GEMM
engine, all Conv + Gemm launches) from per-launch hipEvent times taken on
the executor's stream; ``cpu_baseline`` times the CPU oracle (RTen's
algorithm restated in C++, "port") on a bounded batch-1 sample on the host.
"""
from __future__ import annotations

import argparse
import json
import os
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
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--timing-report", action="store_true")
    return p.parse_args()


def cpu_baseline(spec, seconds: float, batch: int, feed_fn):
    """Time the CPU oracle (RTen's CPU algorithm restated in C++: BLIS 6x16
    AVX2-FMA GEMM, KC = 256, per-image conv parallelism, VirtualIm2Col offset
    tables with masked gathers) on the benchmark's own config and batch.

    RTen sizes its pool to the physical cores (src/threading.rs:41-62); on a
    box whose CPU share is smaller than the machine, that would oversubscribe
    the share, so RTEN_NUM_THREADS is set to the share (OMP_NUM_THREADS when
    the box sets it, else the logical count) -- an RTen-supported setting --
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
        "sample": f"{spec.name} batch {batch} (the benchmark config), {len(times)} runs in ~{seconds:.0f}s, "
                  f"median {med * 1e3:.1f} ms per batch; restated RTen algorithm (C++ BLIS 6x16 "
                  f"AVX2-FMA, KC=256, im2col offset tables + masked gathers), not the Rust binary; "
                  f"{threads} threads (RTEN_NUM_THREADS); host: {cpu_model}, {logical} logical CPUs "
                  f"(num_cpus::get), {physical} physical cores (num_cpus::get_physical)",
    }


# Kernel families the roofline's dominant-kernel time covers, per model (the
# ops bench.py sums: Conv / Gemm / MatMul (incl. its A pack) / FusedAttention).
_ROOF_KERNELS = {
    "resnet50": ("gemm_dma_kernel", "gemm_lat", "gemv"),
    "bert": ("gemm_dma_kernel", "pack_a_kernel", "attention_kernel"),
    "mobilenet_v2": ("gemm_dma_kernel", "gemm_lat", "gemv", "conv_pw_valu_kernel", "conv_direct_valu_kernel",
                     "depthwise", "expand_dw_kernel"),
}


def traffic_bytes(model, batch):
    """HBM bytes per step of the roofline's kernels, from the committed
    rocprofv3 PMC summary of this workload (scripts/gpu_r3_prof.sh ->
    tools/pmc_traffic.py --marker): FETCH_SIZE x2 (gfx950) + WRITE_SIZE,
    eager forwards.  None when no summary exists for this workload."""
    path = os.path.join(ROOT, "profiles", f"r3_pmc_traffic_{model}_b{batch}.json")
    if not os.path.exists(path):
        return None
    try:
        by = json.load(open(path))["by_kernel"]
    except (OSError, ValueError, KeyError):
        return None
    fams = _ROOF_KERNELS[model]
    return round(sum(v for k, v in by.items() if any(f in k for f in fams)))


def main():
    args = parse()
    import numpy as np
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
    from rten_hip import models

    ctx = rten_hip.Context(torch.cuda.current_device())
    B = args.batch
    rng = np.random.default_rng(1234 + rank)
    if args.model == "bert":
        # rten-cli's inputs for a BERT .rten (rten-cli/src/main.rs:250-259):
        # *_ids -> zeros, *_mask -> ones; the embedding Gathers and the mask
        # subgraph run inside the timed step.
        spec = models.bert_encoder(seq=args.seq, embeddings=True)
        flops_per_img = models.bert_flops(seq=args.seq)
        feed_np = {"input_ids": np.zeros((B, args.seq), np.int32),
                   "token_type_ids": np.zeros((B, args.seq), np.int32),
                   "attention_mask": np.ones((B, args.seq), np.int32)}
    else:
        spec = models.resnet50() if args.model == "resnet50" else models.mobilenet_v2()
        flops_per_img = models.conv_flops(spec, 1)
        feed_np = {"input": rng.random((B, 3, 224, 224), dtype=np.float32)}
    g = spec.to_graph(ctx)
    dev = [torch.from_numpy(feed_np[n]).cuda() for n in spec.inputs]
    x = dev[0]
    extra = {g.input_ids[i]: dev[i] for i in range(1, len(dev))}
    (out,) = g.run({g.input_ids[0]: x, **extra}, g.output_ids)  # plans + tunes conv kernels

    from rten_hip.parallel import BatchShardRunner

    def forward(xb):
        g.run({g.input_ids[0]: xb, **extra}, g.output_ids, out=[out])
        return out

    # Rank r holds images [r*B, (r+1)*B) of the world*B job; the only
    # exchange is the all-gather of logits (RCCL) inside runner.run.
    runner = BatchShardRunner(forward)

    def step():
        runner.run(x, world * B)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], device=x.device if backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    value = world * B * args.steps / elapsed

    # Roofline of the dominant kernel: per-launch hipEvent times of every
    # Conv/Gemm launch (the MFMA GEMM engine) on the executor's stream, over
    # the same K steps run eagerly with timing on.
    g.set_timing(True)
    conv_ms = 0.0
    report = ""
    for _ in range(max(1, min(args.steps, 10))):
        g.run({g.input_ids[0]: x, **extra}, g.output_ids, out=[out])
        torch.cuda.synchronize()
        report = g.timing_report()
        for line in report.splitlines()[1:]:
            name = line.split()[0]
            if name.startswith(("Conv", "MatMul", "FusedAttention")) or name == "Gemm":
                conv_ms += float(line.split()[1])
    n_prof = max(1, min(args.steps, 10))
    g.set_timing(False)
    conv_ms /= n_prof
    gemm_flops = flops_per_img * B
    achieved = gemm_flops / (conv_ms * 1e-3) / 1e12 if conv_ms > 0 else 0.0
    hbm_bound = args.model == "mobilenet_v2"
    if hbm_bound:
        io_bytes = models.conv_io_bytes(spec, B)
        achieved_gbs = io_bytes / (conv_ms * 1e-3) / 1e9 if conv_ms > 0 else 0.0

    if args.model == "bert":
        workload = (f"{spec.name} encoder f32 batch={B} per GPU, seq {args.seq}, hidden 768, "
                    f"12 heads, FFN 3072, embeddings + mask subgraph (BASELINE.json configs[3])")
        kernel_desc = "MatMul GEMM launches (gemm_dma_kernel) + FusedAttention"
        data = ("synthetic (rten-cli inputs: input_ids / token_type_ids zeros, attention_mask ones, "
                "resident in HBM; seeded U(+-0.05) weights)")
    else:
        if args.model == "mobilenet_v2":
            cfg = "BASELINE.json configs[2]"
        elif B == 64:
            cfg = "BASELINE.json configs[1]" if world == 1 else "BASELINE.json configs[4]: 64 per GPU"
        elif B == 1:
            cfg = "BASELINE.json metric batch=1 on the GPU path; replicas only for N > 1"
        else:
            cfg = "not a BASELINE.json config"
        workload = f"{spec.name} f32 batch={B} per GPU, 224x224 NCHW, BN folded ({cfg})"
        kernel_desc = ("gemm_dma_kernel (all 53 Conv launches) + FC Gemm" if args.model == "resnet50"
                       else "all Conv launches (DMA GEMM / VALU pointwise / depthwise) + FC Gemm")
        data = "synthetic (U[0,1) images resident in HBM; seeded He-uniform weights)"
    if hbm_bound:
        roofline = {"bound": "hbm", "achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(achieved_gbs / HBM_PEAK_GBPS, 4), "traffic": traffic_bytes(args.model, B),
                    "kernel": kernel_desc, "bytes_per_step": io_bytes,
                    "kernel_ms_per_step": round(conv_ms, 4),
                    "mfma_tflops": round(achieved, 2)}
    else:
        roofline = {"bound": "mfma", "achieved": round(achieved, 2),
                    "peak": F32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(achieved / F32_MFMA_PEAK_TFLOPS, 4),
                    "traffic": traffic_bytes(args.model, B),
                    "kernel": kernel_desc,
                    "flops_per_step": gemm_flops,
                    "kernel_ms_per_step": round(conv_ms, 4),
                    "model_frac": round(value / world * flops_per_img / 1e12 / F32_MFMA_PEAK_TFLOPS, 4)}
    if rank == 0:
        line = {
            "metric": {"resnet50": f"images/sec ResNet-50 f32 batch={B} per GPU",
                       "mobilenet_v2": "images/sec MobileNetV2 f32",
                       "bert": "sequences/sec BERT-base encoder f32"}[args.model],
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
                       "model": spec.name, "global_batch": world * B,
                       "seq_len": args.seq if args.model == "bert" else None,
                       "parallelism": f"batch-shard x{world} (replicated weights, "
                                          f"{'RCCL' if backend == 'nccl' else backend} all-gather of logits)"},
            "roofline": roofline,
        }
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(spec, args.cpu_seconds, B, lambda: feed_np)
        if args.timing_report:
            sys.stderr.write(report + "\n")
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
