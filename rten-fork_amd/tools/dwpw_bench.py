#!/usr/bin/env python3
"""MobileNetV2 features.1 (depthwise 3x3 + Clip -> 1x1 projection to 16) as a
graph at batch B, replayed: ms per replay.  usage: dwpw_bench.py [B] [ITERS]
(RTENHIP_DW_PROJECT=0 runs the two convs apart)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import rten_hip
from rten_hip.graph import ModelSpec

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 50
rng = np.random.default_rng(0)
m = ModelSpec("dwpw")
x = m.value("x")
m.inputs = ["x"]
lo, hi = m.const("lo", np.array(0.0, np.float32)), m.const("hi", np.array(6.0, np.float32))
wd = m.const("wd", rng.uniform(-0.5, 0.5, (32, 1, 3, 3)).astype(np.float32))
bd = m.const("bd", rng.uniform(-0.2, 0.2, (32,)).astype(np.float32))
d = m.op("Clip", [m.op("Conv", [x, wd, bd], {"pads": [1, 1, 1, 1], "strides": [1, 1], "groups": 32}), lo, hi])
wp = m.const("wp", rng.uniform(-0.5, 0.5, (16, 32, 1, 1)).astype(np.float32))
bp = m.const("bp", rng.uniform(-0.2, 0.2, (16,)).astype(np.float32))
y = m.op("Conv", [d, wp, bp], {"pads": [0, 0, 0, 0], "strides": [1, 1]})
m.outputs = [y]
rten_hip.default_context()
g = m.to_graph()
xd = torch.rand((B, 32, 112, 112), device="cuda")
out = g.run({g.input_ids[0]: xd}, g.output_ids)
for _ in range(3):
    out = g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts = []
for _ in range(5):
    e0.record()
    for _ in range(iters):
        g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / iters)
print(f"dwpw b{B} ms/replay min {min(ts):.4f} med {sorted(ts)[2]:.4f}", flush=True)
