#!/usr/bin/env python3
"""Debug aid: one conv with the KC split on and off; prints where they differ
(tile-relative row/col pattern)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import rten_hip
lib = rten_hip.lib()
lib.rtenhip_debug_set_split.argtypes = [ctypes.c_int]
lib.rtenhip_debug_set_dma_config.argtypes = [ctypes.c_int]
cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 7
lib.rtenhip_debug_set_dma_config(cfg)
rng = np.random.default_rng(0)
x = torch.from_numpy(rng.random((2, 64, 14, 14), dtype=np.float32) - 0.5).cuda()
w = torch.from_numpy((rng.random((64, 64, 3, 3), dtype=np.float32) - 0.5) * 0.1).cuda()
b = torch.from_numpy(rng.random(64, dtype=np.float32)).cuda()
outs = []
for sp in (0, 1):
    lib.rtenhip_debug_set_split(sp)
    y = rten_hip.conv(x, w, b, padding=(1, 1, 1, 1))
    torch.cuda.synchronize()
    outs.append(y.cpu().numpy())
a, s = outs
d = a.view(np.uint32) != s.view(np.uint32)
print("cfg", cfg, "differ", int(d.sum()), "of", d.size)
# GEMM view: M = O = 64 rows, N = 2*196 columns
A = a.transpose(1, 0, 2, 3).reshape(64, -1)
S = s.transpose(1, 0, 2, 3).reshape(64, -1)
D = A.view(np.uint32) != S.view(np.uint32)
print("rows differing:", np.nonzero(D.any(axis=1))[0][:40])
print("cols differing (first 40):", np.nonzero(D.any(axis=0))[0][:40])
for r in (0, 1, 2, 4, 8):
    print("row", r, "no-split", A[r, :4], "split", S[r, :4])
