#!/usr/bin/env python3
"""Run one conv layer N times (for rocprofv3 counter collection).
usage: onelayer.py N C H W O k stride pad [cfg] [iters]"""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import rten_hip
a = [int(v) for v in sys.argv[1:]]
N, C, H, W, O, k, s, p = a[:8]
cfg = a[8] if len(a) > 8 else -1
iters = a[9] if len(a) > 9 else 5
lib = rten_hip.lib(); lib.rtenhip_debug_set_gemm_config.argtypes = [ctypes.c_int]
lib.rtenhip_debug_set_gemm_config(cfg)
# DMA kernel config (RTENHIP_DMA_CFG=-1 default, "off" = register-staged kernel)
dcfg = os.environ.get("RTENHIP_DMA_CFG", "-1")
ctx = rten_hip.default_context().ptr
lib.rtenhip_debug_set_dma.argtypes = [ctypes.c_void_p, ctypes.c_int]
lib.rtenhip_debug_trust_weight_cache.argtypes = [ctypes.c_void_p, ctypes.c_int]
lib.rtenhip_debug_set_dma_config.argtypes = [ctypes.c_int]
lib.rtenhip_debug_trust_weight_cache(ctx, 1)
lib.rtenhip_debug_set_dma_mode.argtypes = [ctypes.c_int]
lib.rtenhip_debug_set_dma_mode(int(os.environ.get("RTENHIP_DMA_MODE", "0")))
# persistent launch override (k blocks per CU; unset: one block per item)
lib.rtenhip_debug_set_dma_persist.argtypes = [ctypes.c_int]
lib.rtenhip_debug_set_dma_persist(int(os.environ.get("RTENHIP_DMA_PERSIST", "-1")))
lib.rtenhip_debug_set_split.argtypes = [ctypes.c_int]
lib.rtenhip_debug_set_split(int(os.environ.get("RTENHIP_DMA_SPLIT", "1")))
if dcfg == "off":
    lib.rtenhip_debug_set_dma(ctx, 0)
else:
    lib.rtenhip_debug_set_dma_config(int(dcfg))
rng = np.random.default_rng(0)
x = torch.from_numpy(rng.random((N, C, H, W), dtype=np.float32) - 0.5).cuda()
w = torch.from_numpy((rng.random((O, C, k, k), dtype=np.float32) - 0.5) * 0.1).cuda()
b = torch.from_numpy(rng.random(O, dtype=np.float32)).cuda()
y = rten_hip.conv(x, w, b, padding=(p,) * 4, strides=(s, s))
for _ in range(iters):
    rten_hip.conv(x, w, b, padding=(p,) * 4, strides=(s, s), out=y)
torch.cuda.synchronize()
print("ok")
