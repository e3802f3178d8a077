#!/usr/bin/env python3
"""Vendor-library f32 GEMM throughput on this GPU (context for the conv
kernels' roofline fraction; not part of the product)."""
import torch
torch.backends.cuda.matmul.allow_tf32 = False
for (m, n, k) in [(4096, 4096, 4096), (8192, 8192, 8192), (256, 12544, 2304), (512, 3136, 4608), (128, 200704, 256)]:
    a = torch.randn(m, k, device="cuda")
    b = torch.randn(k, n, device="cuda")
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"torch.mm f32 {m}x{n}x{k}: {ms:.3f} ms  {2*m*n*k/ms/1e9:.1f} TFLOP/s")
