#!/usr/bin/env python3
"""Depthwise conv microbenchmark (MobileNetV2 b128 shapes): GB/s of the
minimum traffic (input + output + weights)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import rten_hip

shapes = [(128, 32, 112, 1), (128, 96, 112, 2), (128, 144, 56, 1), (128, 144, 56, 2),
          (128, 192, 28, 1), (128, 384, 14, 1), (128, 960, 7, 1)]
rng = np.random.default_rng(0)
for (n, c, hw, s) in shapes:
    x = torch.from_numpy(rng.random((n, c, hw, hw), dtype=np.float32)).cuda()
    w = torch.from_numpy(rng.random((c, 1, 3, 3), dtype=np.float32)).cuda()
    b = torch.from_numpy(rng.random(c, dtype=np.float32)).cuda()
    y = rten_hip.conv(x, w, b, padding=(1, 1, 1, 1), strides=(s, s), groups=c)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        rten_hip.conv(x, w, b, padding=(1, 1, 1, 1), strides=(s, s), groups=c, out=y)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    byts = (x.numel() + y.numel()) * 4
    print(f"dw C={c:4d} {hw}x{hw} s{s}: {ms:.4f} ms  {byts / ms / 1e6:.0f} GB/s")
