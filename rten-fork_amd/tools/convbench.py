#!/usr/bin/env python3
"""Per-layer conv microbenchmark: every distinct ResNet-50 conv at batch B
under each GEMM tile configuration (rtenhip_debug_set_gemm_config).  Prints
TFLOP/s per (layer, config) and checks every config gives bit-identical
outputs (the KC=256 summation order does not depend on tiling)."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np
import torch

import rten_hip
from rten_hip import models


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--cfgs", default="g0,d0,d1,d2,d3,d6",
                    help="g<n>: register-staged kernel config n; d<n>: LDS-DMA kernel config n")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--split", type=int, default=1, help="KC split of remainder tiles (standalone conv path)")
    ap.add_argument("--dmamode", type=int, default=0,
                    help="timing experiment: 1 = no K-loop DMA, 2 = no MFMA (wrong results)")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--shape", action="append", default=[],
                    help="extra conv N,C,H,W,O,k,stride,pad (repeatable); replaces the model's layers")
    args = ap.parse_args()
    lib = rten_hip.lib()
    lib.rtenhip_debug_set_gemm_config.argtypes = [ctypes.c_int]
    lib.rtenhip_debug_set_dma_config.argtypes = [ctypes.c_int]
    lib.rtenhip_debug_set_dma.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.rtenhip_debug_trust_weight_cache.argtypes = [ctypes.c_void_p, ctypes.c_int]
    ctx = rten_hip.default_context().ptr
    lib.rtenhip_debug_trust_weight_cache(ctx, 1)
    lib.rtenhip_debug_set_dma_mode.argtypes = [ctypes.c_int]
    lib.rtenhip_debug_set_dma_mode(args.dmamode)
    lib.rtenhip_debug_set_split.argtypes = [ctypes.c_int]
    lib.rtenhip_debug_set_split(args.split)
    spec = getattr(models, args.model)()
    consts = {n.name: n.data for n in spec.nodes if n.kind == "const"}
    # distinct conv shapes with their input spatial size
    shapes = {spec.inputs[0]: (args.batch, 3, 224, 224)}
    layers = {}
    for n in spec.nodes:
        if n.kind != "op":
            continue
        xs = shapes.get(n.inputs[0])
        if n.op_type == "Conv":
            w = consts[n.inputs[1]]
            p, s, g = n.attrs["pads"], n.attrs["strides"], n.attrs.get("groups", 1)
            oh = (xs[2] + p[0] + p[2] - w.shape[2]) // s[0] + 1
            ow = (xs[3] + p[1] + p[3] - w.shape[3]) // s[1] + 1
            key = (xs, w.shape, tuple(p), tuple(s), g)
            layers.setdefault(key, [0, n.name])[0] += 1
            shapes[n.outputs[0]] = (xs[0], w.shape[0], oh, ow)
        elif n.op_type == "MaxPool":
            shapes[n.outputs[0]] = (xs[0], xs[1], xs[2] // 2, xs[3] // 2)
        elif n.op_type in ("GlobalAveragePool",):
            shapes[n.outputs[0]] = (xs[0], xs[1], 1, 1)
        else:
            shapes[n.outputs[0]] = xs
    if args.shape:
        layers = {}
        for sh in args.shape:
            N, Cc, H, W, O, k, st, pd = [int(v) for v in sh.split(",")]
            layers[((N, Cc, H, W), (O, Cc, k, k), (pd,) * 4, (st, st), 1)] = [1, f"custom{len(layers)}"]
    cfgs = args.cfgs.split(",")
    rng = np.random.default_rng(0)
    total = {c: 0.0 for c in cfgs}
    best_total = 0.0
    print(f"{'layer':28s} {'M':>5s} {'K':>5s} {'N':>7s} cnt " + " ".join(f"{c:>5s}" for c in cfgs))
    for (xs, ws, p, s, g), (cnt, name) in layers.items():
        x = torch.from_numpy(rng.random(xs, dtype=np.float32) - 0.5).cuda()
        w = torch.from_numpy((rng.random(ws, dtype=np.float32) - 0.5) * 0.1).cuda()
        b = torch.from_numpy(rng.random(ws[0], dtype=np.float32)).cuda()
        oh = (xs[2] + p[0] + p[2] - ws[2]) // s[0] + 1
        ow = (xs[3] + p[1] + p[3] - ws[3]) // s[1] + 1
        M, K, N = ws[0] // g, ws[1] * ws[2] * ws[3], xs[0] * oh * ow
        flops = 2.0 * ws[0] * K * N
        ref = None
        row = []
        for c in cfgs:
            if c[0] == "g":
                lib.rtenhip_debug_set_dma(ctx, 0)
                lib.rtenhip_debug_set_gemm_config(int(c[1:]))
            else:
                lib.rtenhip_debug_set_dma(ctx, 1)
                lib.rtenhip_debug_set_dma_config(int(c[1:]))
            y = rten_hip.conv(x, w, b, padding=p, strides=s, groups=g)
            torch.cuda.synchronize()
            if ref is None:
                ref = y.clone()
            elif args.dmamode == 0 and not torch.equal(y.view(torch.int32), ref.view(torch.int32)):
                print(f"  !! cfg {c} output differs on {name}")
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                rten_hip.conv(x, w, b, padding=p, strides=s, groups=g, out=y)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.iters
            total[c] += ms * cnt
            row.append(flops / ms / 1e9)
        bi = max(range(len(row)), key=lambda i: row[i])
        best_total += flops / row[bi] / 1e9 * cnt
        print(f"{name:28s} {M:5d} {K:5d} {N:7d} {cnt:3d} " + " ".join(f"{v:5.1f}" for v in row)
              + f"  best={cfgs[bi]}")
    print("total ms per forward (convs only): " + " ".join(f"{c}={total[c]:.3f}" for c in cfgs))
    print(f"best-per-layer total ms: {best_total:.3f}")


if __name__ == "__main__":
    main()
