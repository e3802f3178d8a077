#!/usr/bin/env python3
"""Where do the DMA GEMM's workgroups run?  (tuning aid, needs an
RTENHIP_DMA_EXPERIMENT=5 build, see build_exp.sh)

Runs one conv layer with the placement stamps on and prints, per CU, the
blocks it ran and its busy span, against the kernel span: a CU that carries
more tiles than the average sets the kernel time.
usage: RTENHIP_LIB=.../exp5/librten_hip.so placement.py N C H W O k stride pad [cfg [persist_k]]
(timestamps: s_memrealtime, 100 MHz)"""
import ctypes
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import rten_hip

a = [int(v) for v in sys.argv[1:]]
N, C, H, W, O, k, s, p = a[:8]
cfg = a[8] if len(a) > 8 else -1
persist = a[9] if len(a) > 9 else 0
lib = rten_hip.lib()
ctx = rten_hip.default_context().ptr
lib.rtenhip_debug_trust_weight_cache.argtypes = [ctypes.c_void_p, ctypes.c_int]
lib.rtenhip_debug_trust_weight_cache(ctx, 1)
lib.rtenhip_debug_set_dma_config.argtypes = [ctypes.c_int]
lib.rtenhip_debug_set_dma_config(cfg)
lib.rtenhip_debug_set_split.argtypes = [ctypes.c_int]
lib.rtenhip_debug_set_split(1)
lib.rtenhip_debug_set_dma_stamps.argtypes = [ctypes.c_void_p]
lib.rtenhip_debug_set_dma_persist.argtypes = [ctypes.c_int]
lib.rtenhip_debug_set_dma_persist(persist)
rng = np.random.default_rng(0)
x = torch.from_numpy(rng.random((N, C, H, W), dtype=np.float32) - 0.5).cuda()
w = torch.from_numpy((rng.random((O, C, k, k), dtype=np.float32) - 0.5) * 0.1).cuda()
b = torch.from_numpy(rng.random(O, dtype=np.float32)).cuda()
y = rten_hip.conv(x, w, b, padding=(p,) * 4, strides=(s, s))
for _ in range(3):
    rten_hip.conv(x, w, b, padding=(p,) * 4, strides=(s, s), out=y)
stamps = torch.zeros(8 * 200000, dtype=torch.int64, device="cuda")
lib.rtenhip_debug_set_dma_stamps(ctypes.c_void_p(stamps.data_ptr()))
torch.cuda.synchronize()
rten_hip.conv(x, w, b, padding=(p,) * 4, strides=(s, s), out=y)
torch.cuda.synchronize()
lib.rtenhip_debug_set_dma_stamps(None)
st = stamps.cpu().numpy().reshape(-1, 8)
st = st[(st[:, 1] != 0)]
hw = st[:, 0].astype(np.uint64)
hwid = (hw & np.uint64(0xffffffff)).astype(np.int64)
xcc = (hw >> np.uint64(32)).astype(np.int64) & 0xf
cu = (hwid >> 8) & 0xf
sh = (hwid >> 12) & 0x1
se = (hwid >> 13) & 0x7
t0, t1 = st[:, 1], st[:, 2]
span = t1.max() - t0.min()
key = xcc * 1000 + se * 100 + sh * 16 + cu
per = defaultdict(list)
for i in range(len(st)):
    per[key[i]].append((t0[i], t1[i], i))
print(f"blocks {len(st)}  CUs used {len(per)}  kernel span {span / 100:.1f} us")
cnt = np.array([len(v) for v in per.values()])
print(f"blocks per CU: min {cnt.min()} max {cnt.max()} mean {cnt.mean():.2f}  histogram "
      f"{np.bincount(cnt).tolist()}")
# per-CU busy end relative to kernel start
ends = np.array([max(e for _, e, _ in v) - t0.min() for v in per.values()])
print(f"CU finish time / span: min {ends.min()/span:.2f} median {np.median(ends)/span:.2f} max {ends.max()/span:.2f}")
dur = t1 - t0
print(f"block duration us: min {dur.min()/100:.1f} median {np.median(dur)/100:.1f} max {dur.max()/100:.1f}")
nfull = None
# blocks whose id is in the first part (full tiles) vs split units: by duration
big = dur > np.median(dur) * 0.5
fullcnt = defaultdict(int)
for i in range(len(st)):
    if big[i]:
        fullcnt[key[i]] += 1
fc = np.array(list(fullcnt.values()))
print(f"long blocks per CU: min {fc.min()} max {fc.max()} mean {fc.mean():.2f} histogram {np.bincount(fc).tolist()}")
starts = np.sort(t0 - t0.min())
print(f"block start times (us) quantiles: " +
      " ".join(f"{q}:{np.quantile(starts, q)/100:.1f}" for q in (0.1, 0.5, 0.8, 0.9, 0.95, 0.99, 1.0)))
# per-CU busy: sum of block durations (blocks overlap on a CU, so this is
# the CU's wave-time), and per-CU last end
busy = np.array([sum(e - s for s, e, _ in v) for v in per.values()]) / 100
print(f"per-CU summed block time us: min {busy.min():.1f} median {np.median(busy):.1f} max {busy.max():.1f}")
# phases (experiment build 5 stamps the end of the last item's K loop in slot 3)
tk = st[:, 3]
if (tk > 0).all():
    kph = (tk - t0) / 100
    eph = (t1 - tk) / 100
    print(f"start->K-loop end us: median {np.median(kph):.2f} p10 {np.quantile(kph, 0.1):.2f} p90 {np.quantile(kph, 0.9):.2f}")
    print(f"epilogue us:          median {np.median(eph):.2f} p10 {np.quantile(eph, 0.1):.2f} p90 {np.quantile(eph, 0.9):.2f}")
    if (st[:, 4] > 0).all():
        for nm, a_, b_ in (("K end -> drain+barrier", 3, 4), ("-> block 0 in slot", 4, 5), ("-> end", 5, 2)):
            ph = (st[:, b_] - st[:, a_]) / 100
            print(f"  {nm:24s} median {np.median(ph):.2f} p10 {np.quantile(ph, 0.1):.2f} p90 {np.quantile(ph, 0.9):.2f}")
