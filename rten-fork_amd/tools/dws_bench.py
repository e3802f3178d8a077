#!/usr/bin/env python3
"""Depthwise microbenchmark at MobileNetV2 b128's small-plane shapes (the
streaming kernel, dw_stream.hip, vs depthwise_lds_kernel with
RTENHIP_DW_STREAM=0): per shape 20 launches; run under rocprofv3 for
per-kernel times, or read the event times printed here."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import rten_hip

shapes = [(128, 384, 14, 1), (128, 576, 14, 1), (128, 576, 14, 2), (128, 960, 7, 1)]
rng = np.random.default_rng(0)
for (n, c, hw, s) in shapes:
    x = torch.from_numpy(rng.random((n, c, hw, hw), dtype=np.float32)).cuda()
    w = torch.from_numpy(rng.random((c, 1, 3, 3), dtype=np.float32)).cuda()
    b = torch.from_numpy(rng.random(c, dtype=np.float32)).cuda()
    kw = dict(padding=(1, 1, 1, 1), strides=(s, s), groups=c, act="clip", act_range=(0.0, 6.0))
    y = rten_hip.conv(x, w, b, **kw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        rten_hip.conv(x, w, b, out=y, **kw)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    byts = (x.numel() + y.numel()) * 4
    print(f"dw C={c:4d} {hw}x{hw} s{s}: {ms * 1000:.1f} us  {byts / ms / 1e6:.0f} GB/s", flush=True)
