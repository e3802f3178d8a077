#!/usr/bin/env python3
"""Run a benchmark model eagerly a few times through the device graph -- the
workload for rocprofv3 PMC passes (no hipGraph replay, so every kernel is a
separate dispatch the counters can attribute).  A torch fill kernel marks the
end of the tuning run: tools/pmc_traffic.py --marker counts only the
librten_hip dispatches after it.

usage: model_once.py [runs] [model] [batch] [--report]   (defaults: 2 resnet50 64;
--report: one more eager run with per-op hipEvent timing, report printed)"""
import os
import sys

os.environ.setdefault("RTENHIP_GRAPH", "0")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import rten_hip
from rten_hip import models

report = "--report" in sys.argv
sys.argv = [a for a in sys.argv if a != "--report"]
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 2
model = sys.argv[2] if len(sys.argv) > 2 else "resnet50"
batch = int(sys.argv[3]) if len(sys.argv) > 3 else 64
torch.cuda.set_device(0)
if model == "bert":
    spec = models.bert_encoder(seq=128, embeddings=True)
    feed = {"input_ids": np.zeros((batch, 128), np.int32), "token_type_ids": np.zeros((batch, 128), np.int32),
            "attention_mask": np.ones((batch, 128), np.int32)}
else:
    spec = models.resnet50() if model == "resnet50" else models.mobilenet_v2()
    feed = {"input": np.random.default_rng(1234).random((batch, 3, 224, 224), dtype=np.float32)}
g = spec.to_graph(rten_hip.Context(0))
dev = {g.input_ids[i]: torch.from_numpy(feed[n]).cuda() for i, n in enumerate(spec.inputs)}
(out,) = g.run(dev, g.output_ids)  # plan + tuning
torch.cuda.synchronize()
marker = torch.zeros(1, device="cuda")
marker.fill_(1.0)  # the marker dispatch
torch.cuda.synchronize()
print("MARK tuned", flush=True)
for _ in range(runs):
    g.run(dev, g.output_ids, out=[out])
torch.cuda.synchronize()
print("done", runs, flush=True)
if report:
    g.set_timing(True)
    g.run(dev, g.output_ids, out=[out])
    torch.cuda.synchronize()
    print(g.timing_report(), flush=True)
