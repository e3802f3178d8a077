#!/usr/bin/env python3
"""Batch-1 conv kernels with their operands L2-hot vs L2-cold (timing
experiment, run under rocprofv3 --kernel-trace): one conv graph replayed
back to back (phase A: weights and input still in the XCD L2s from the
previous replay) and then replayed after a 64 MB fill (phase B: L2s
scrubbed, operands from the Infinity Cache).  A marker kernel (a 1-element
fill) separates the phases.  usage: l2_hot_cold.py C H O k [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from rten_hip.graph import ModelSpec

C, H, O, k = (int(v) for v in sys.argv[1:5])
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 50
rng = np.random.default_rng(0)
m = ModelSpec("one_conv")
x = m.value("x")
m.inputs = ["x"]
w = m.const("w", rng.uniform(-0.1, 0.1, (O, C, k, k)).astype(np.float32))
b = m.const("b", rng.uniform(-0.1, 0.1, (O,)).astype(np.float32))
p = k // 2
m.outputs = [m.op("Relu", [m.op("Conv", [x, w, b], {"pads": [p, p, p, p], "strides": [1, 1]})])]
g = m.to_graph()
xd = torch.from_numpy(rng.uniform(-1, 1, (1, C, H, H)).astype(np.float32)).cuda()
out = g.run({g.input_ids[0]: xd}, g.output_ids)
for _ in range(5):
    g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
scrub = torch.empty(16 << 20, dtype=torch.float32, device="cuda")
mark = torch.empty(1, device="cuda")
torch.cuda.synchronize()
for _ in range(reps):
    g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
torch.cuda.synchronize()
mark.fill_(1.0)
torch.cuda.synchronize()
for _ in range(reps):
    scrub.fill_(0.5)
    g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
torch.cuda.synchronize()
print("done", flush=True)
