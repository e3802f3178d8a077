#!/usr/bin/env python3
"""Time one Conv (+ optional Clip) through the device graph, as the model
benches run it (plan-time tuning, then eager timing runs).  Tuning aid for
the tuner's candidate kernels: set RTENHIP_PW_VALU / RTENHIP_TUNE to force.
usage: conv_graph_time.py N C H W O k stride pad [clip]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import rten_hip
from rten_hip.graph import ModelSpec

a = sys.argv[1:]
N, C, H, W, O, k, s, p = (int(v) for v in a[:8])
clip = len(a) > 8 and a[8] == "clip"
rng = np.random.default_rng(0)
m = ModelSpec("one_conv")
x = m.value("x")
m.inputs = ["x"]
w = m.const("w", rng.uniform(-0.3, 0.3, (O, C, k, k)).astype(np.float32))
b = m.const("b", rng.uniform(-0.1, 0.1, (O,)).astype(np.float32))
y = m.op("Conv", [x, w, b], {"pads": [p] * 4, "strides": [s, s]})
if clip:
    y = m.op("Clip", [y, m.const("lo", np.array(0, np.float32)), m.const("hi", np.array(6, np.float32))])
m.outputs = [y]
g = m.to_graph()
xd = torch.from_numpy(rng.random((N, C, H, W), dtype=np.float32)).cuda()
out = g.run({g.input_ids[0]: xd}, g.output_ids)
torch.cuda.synchronize()
g.set_timing(True)
best = None
for _ in range(10):
    g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
    torch.cuda.synchronize()
    rep = g.timing_report()
    line = [l for l in rep.splitlines() if l.split() and l.split()[0] == "op"][0]
    ms = float(line.split()[4])
    if best is None or ms < best[0]:
        best = (ms, line)
print(f"PW_VALU={os.environ.get('RTENHIP_PW_VALU', '-')} {best[1]}")
