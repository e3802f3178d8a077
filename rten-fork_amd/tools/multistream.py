#!/usr/bin/env python3
"""Prototype (tuning aid): ResNet-50 at batch B split into S sub-batches, each
run by its own device graph (own context, own executor streams) so the
sub-batches' layers overlap on the GPU.  Prints images/s per S.
usage: multistream.py [B] [S ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import rten_hip
from rten_hip import models

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
splits = [int(v) for v in sys.argv[2:]] or [1, 2, 4]
spec = models.resnet50()
x = torch.from_numpy(np.random.default_rng(0).random((B, 3, 224, 224), dtype=np.float32)).cuda()
ref = None
for S in splits:
    b = B // S
    ctxs = [rten_hip.Context(0) for _ in range(S)]
    graphs = [spec.to_graph(c) for c in ctxs]
    streams = [torch.cuda.Stream() for _ in range(S)]
    xs = [x[i * b:(i + 1) * b].contiguous() for i in range(S)]
    outs = [None] * S

    def step():
        for i in range(S):
            with torch.cuda.stream(streams[i]):
                outs[i] = graphs[i].run({graphs[i].input_ids[0]: xs[i]}, graphs[i].output_ids, out=outs[i])
        for s in streams:
            torch.cuda.current_stream().wait_stream(s)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    y = torch.cat([o[0] for o in outs]).cpu().numpy()
    if ref is None:
        ref = y
    same = np.array_equal(y.view(np.uint32), ref.view(np.uint32))
    n = 20
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    print(f"S={S} sub-batch {b}: {dt * 1e3:.3f} ms/step  {B / dt:.0f} img/s  bit-identical to S={splits[0]}: {same}",
          flush=True)
