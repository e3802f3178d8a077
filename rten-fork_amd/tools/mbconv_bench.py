#!/usr/bin/env python3
"""Fused expand(1x1)+Clip -> depthwise 3x3+Clip microbenchmark at MobileNetV2
batch 128 shapes (RTENHIP_EXPAND_DW=all: every eligible pair fused): per-pair
time of the device graph (eager runs, so rocprofv3 --pmc can attribute the
kernels) and GB/s of the fused pair's minimum traffic (x in, y out).
usage: mbconv_bench.py [runs]"""
import os
import sys
import time

os.environ.setdefault("RTENHIP_EXPAND_DW", "all")
os.environ.setdefault("RTENHIP_GRAPH", "0")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import rten_hip
from rten_hip.graph import ModelSpec

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 10
# (C_in, H, hidden, stride): features.2, .3, .4, .5, .7
PAIRS = [(16, 112, 96, 2), (24, 56, 144, 1), (24, 56, 144, 2), (32, 28, 192, 1), (32, 28, 192, 2)]
N = 128
rng = np.random.default_rng(0)
torch.cuda.set_device(0)
ctx = rten_hip.Context(0)
for cin, hw, hid, s in PAIRS:
    m = ModelSpec("mb")
    x = m.value("x")
    m.inputs = ["x"]
    lo, hi = m.const("lo", np.array(0.0, np.float32)), m.const("hi", np.array(6.0, np.float32))
    we = m.const("we", rng.uniform(-0.5, 0.5, (hid, cin, 1, 1)).astype(np.float32))
    be = m.const("be", rng.uniform(-0.2, 0.2, (hid,)).astype(np.float32))
    e = m.op("Clip", [m.op("Conv", [x, we, be], {"pads": [0, 0, 0, 0]}), lo, hi])
    wd = m.const("wd", rng.uniform(-0.5, 0.5, (hid, 1, 3, 3)).astype(np.float32))
    bd = m.const("bd", rng.uniform(-0.2, 0.2, (hid,)).astype(np.float32))
    m.outputs = [m.op("Clip", [m.op("Conv", [e, wd, bd], {"pads": [1, 1, 1, 1], "strides": [s, s], "groups": hid}),
                               lo, hi])]
    g = m.to_graph(ctx)
    xd = torch.from_numpy(rng.uniform(-1, 2, (N, cin, hw, hw)).astype(np.float32)).cuda()
    out = g.run({g.input_ids[0]: xd}, g.output_ids)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(runs):
        g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / runs * 1e3
    oh = (hw - 1) // s + 1
    byts = (xd.numel() + N * hid * oh * oh) * 4
    print(f"C_in={cin} {hw}x{hw} hidden={hid} s{s}: {ms:.4f} ms  {byts / ms / 1e6:.0f} GB/s", flush=True)
