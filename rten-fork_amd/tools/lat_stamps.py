#!/usr/bin/env python3
"""Phase timeline of the latency-GEMM launches of one ResNet-50 batch-1
forward (timing experiment; rtenhip_debug_set_lat_stamps).  Per launch:
waves, span, the spread of wave start times, and per-wave phase durations
(operand loads, MFMA chain, store + arrival count, fold, epilogue).
usage: lat_stamps.py [runs]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import rten_hip
from rten_hip import models


W = 10  # u64 per wave (kLatStampWords)


def main():
    torch.cuda.set_device(0)
    spec = models.resnet50()
    g = spec.to_graph()
    x = torch.from_numpy(np.random.default_rng(0).random((1, 3, 224, 224), dtype=np.float32)).cuda()
    (out,) = g.run({g.input_ids[0]: x}, g.output_ids)
    for _ in range(3):
        g.run({g.input_ids[0]: x}, g.output_ids, out=[out])
    torch.cuda.synchronize()
    lib = rten_hip.lib()
    lib.rtenhip_debug_set_lat_stamps.argtypes = [C.c_void_p, C.c_int64]
    lib.rtenhip_debug_lat_stamps_used.restype = C.c_int64
    cap = 1 << 20
    buf = torch.zeros(cap * W, dtype=torch.int64, device="cuda")
    g.set_timing(True)
    g.run({g.input_ids[0]: x}, g.output_ids, out=[out])  # warm eager
    torch.cuda.synchronize()
    lib.rtenhip_debug_set_lat_stamps(C.c_void_p(buf.data_ptr()), cap)
    g.run({g.input_ids[0]: x}, g.output_ids, out=[out])
    torch.cuda.synchronize()
    used = lib.rtenhip_debug_lat_stamps_used()
    lib.rtenhip_debug_set_lat_stamps(None, 0)
    rep = g.timing_report()
    lat_ops = [l for l in rep.splitlines() if l.startswith("op ") and "cfg=lat" in l and "cfg=lat9" not in l]
    a = buf[: used * W].cpu().numpy().view(np.uint64).reshape(-1, W)
    seq = (a[:, 0] >> np.uint64(48)).astype(int)
    xcc = ((a[:, 0] >> np.uint64(40)) & np.uint64(0xFF)).astype(int)
    t = a[:, 1:7].astype(np.int64)
    print(f"{used} waves in {seq.max()} launches")
    print("seq layer                     cfg   waves  span  start_spread | load  chain  arrive  fold  epi  (us, median; p90 in ())")
    for s in range(1, seq.max() + 1):
        m = seq == s
        ts = t[m]
        t0 = ts[:, 0].min()
        us = lambda v: v / 100.0
        span = us(ts[:, 5].max() - t0) if (ts[:, 5] > 0).any() else float("nan")
        spread = us(np.percentile(ts[:, 0] - t0, 90))
        load = us(ts[:, 1] - ts[:, 0])
        chain = us(ts[:, 2] - ts[:, 1])
        arr_m = ts[:, 3] > 0
        arrive = us(ts[arr_m, 3] - ts[arr_m, 2]) if arr_m.any() else np.array([0.0])
        fold_m = ts[:, 4] > 0
        fold = us(ts[fold_m, 4] - ts[fold_m, 3]) if fold_m.any() else np.array([0.0])
        end_m = ts[:, 5] > 0
        prev = np.where(ts[:, 4] > 0, ts[:, 4], ts[:, 2])
        epi = us(ts[end_m, 5] - prev[end_m]) if end_m.any() else np.array([0.0])
        f = lambda v: f"{np.median(v):5.2f}({np.percentile(v, 90):5.2f})"
        name = lat_ops[s - 1].split()[1] if s - 1 < len(lat_ops) else "?"
        cfg = lat_ops[s - 1].split("cfg=")[1].split()[0] if s - 1 < len(lat_ops) else "?"
        extra = ""
        ta, tb = a[m, 8].astype(np.int64), a[m, 9].astype(np.int64)
        if (ta > 0).any():
            extra = f"  A landed {f(us(ta[ta > 0] - ts[ta > 0, 0]))} B landed {f(us(tb[tb > 0] - ts[tb > 0, 0]))}"
        print(f"{s:3d} {name:24s} {cfg:6s} {m.sum():6d} {span:6.2f} {spread:6.2f} | {f(load)} {f(chain)} {f(arrive)} {f(fold)} {f(epi)}"
              + extra)
    print(rep)


if __name__ == "__main__":
    main()
