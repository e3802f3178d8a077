#!/usr/bin/env python3
"""Run ResNet-50 (batch 64) eagerly a few times through the device graph --
the workload for rocprofv3 PMC passes (no hipGraph replay, so every kernel is
a separate dispatch the counters can attribute).  usage: model_once.py [runs]"""
import os
import sys

os.environ.setdefault("RTENHIP_GRAPH", "0")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import rten_hip
from rten_hip import models

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 2
spec = models.resnet50()
g = spec.to_graph(rten_hip.Context(0))
x = torch.from_numpy(np.random.default_rng(1234).random((64, 3, 224, 224), dtype=np.float32)).cuda()
(out,) = g.run({g.input_ids[0]: x}, g.output_ids)  # plan + tuning
torch.cuda.synchronize()
print("MARK tuned", flush=True)
for _ in range(runs):
    g.run({g.input_ids[0]: x}, g.output_ids, out=[out])
torch.cuda.synchronize()
print("done", runs, flush=True)
