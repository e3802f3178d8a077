#!/usr/bin/env python3
"""Time the ResNet stem MaxPool (3x3 s2 p1 on [64,64,112,112]) through the op
API against a plain device copy of the same bytes (bandwidth reference)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import rten_hip

x = torch.rand(64, 64, 112, 112, device="cuda")
rten_hip.default_context()


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


t_pool = timeit(lambda: rten_hip.max_pool(x, (3, 3), (2, 2), (1, 1, 1, 1)))
z = torch.empty_like(x)
t_copy = timeit(lambda: z.copy_(x))
mb = (x.numel() + x.numel() // 4) * 4 / 1e6
print(f"maxpool {t_pool * 1e3:.1f} us ({mb / t_pool / 1e3:.2f} TB/s on {mb:.0f} MB); "
      f"copy {t_copy * 1e3:.1f} us ({2 * x.numel() * 4 / 1e9 / t_copy:.2f} TB/s)")
