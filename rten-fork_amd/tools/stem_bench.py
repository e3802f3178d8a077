#!/usr/bin/env python3
"""One stem conv (+ Relu / Clip) as a graph, replayed: ms per replay.
usage: stem_bench.py {resnet50|mobilenet_v2} BATCH [ITERS]
RTENHIP_PW_VALU=800 forces the MFMA stem kernel (csrc/conv_stem.hip);
RTENHIP_STEM=0 keeps it out of the tuner."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import rten_hip
from rten_hip.graph import ModelSpec

model = sys.argv[1]
B = int(sys.argv[2])
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 50
k, O, pads = (7, 64, [3, 3, 3, 3]) if model == "resnet50" else (3, 32, [1, 1, 1, 1])
rng = np.random.default_rng(0)
m = ModelSpec("stem")
x = m.value("x")
m.inputs = ["x"]
w = m.const("w", rng.uniform(-0.5, 0.5, (O, 3, k, k)).astype(np.float32))
b = m.const("b", rng.uniform(-0.2, 0.2, (O,)).astype(np.float32))
y = m.op("Relu", [m.op("Conv", [x, w, b], {"pads": pads, "strides": [2, 2]})])
m.outputs = [y]
rten_hip.default_context()
g = m.to_graph()
xd = torch.rand((B, 3, 224, 224), device="cuda")
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
g.set_timing(True)
g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
torch.cuda.synchronize()
cfg = [l for l in g.timing_report().splitlines() if "Conv" in l]
print(f"{model} b{B} ms/replay min {min(ts):.4f} med {sorted(ts)[2]:.4f}  {cfg[0].strip() if cfg else ''}", flush=True)
