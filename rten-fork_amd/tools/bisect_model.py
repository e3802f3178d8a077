#!/usr/bin/env python3
"""Locate a whole-model parity failure: run ResNet-50 (batch 2) through the
device graph under several executor settings and report, per setting and per
run (run 0 eager, later runs hipGraph replay), whether the logits are
bit-exact with the CPU oracle; then run once with every op output requested
(so each intermediate is materialised) and name the first op that differs.

usage: bisect_model.py [resnet50|mobilenet_v2] [batch]   (debug tool, GPU)
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(ROOT, "oracle")]

import numpy as np
import torch

import graph_runner
import rten_hip
from rten_hip import models


def bits_equal(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    spec = getattr(models, name)()
    x = np.random.default_rng(1234).random((batch, 3, 224, 224), dtype=np.float32)
    op_outs = [n.outputs[0] for n in spec.nodes if n.kind == "op"]
    exp_all = graph_runner.run(spec, {"input": x}, outputs=op_outs)
    exp = exp_all[spec.outputs[0]]
    xd = torch.from_numpy(x).cuda()
    rten_hip.default_context()
    settings = [
        dict(),
        dict(RTENHIP_GRAPH="0"),
        dict(RTENHIP_TUNE="0"),
        dict(RTENHIP_GRAPH="0", RTENHIP_TUNE="0"),
    ]
    reps = int(os.environ.get("BISECT_REPS", "3"))
    for optimize in (False, True):
        for env in settings * reps:
            for k in ("RTENHIP_GRAPH", "RTENHIP_TUNE"):
                os.environ.pop(k, None)
            os.environ.update(env)
            g = spec.to_graph(optimize=optimize)
            res = []
            out = None
            for _ in range(3):
                out = g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
                torch.cuda.synchronize()
                res.append(bits_equal(out[0].cpu().numpy(), exp))
            print(f"optimize={optimize} env={env} runs bit-exact={res}", flush=True)
            g.close()
    for k in ("RTENHIP_GRAPH", "RTENHIP_TUNE"):
        os.environ.pop(k, None)
    # Every op output requested: per-op comparison.
    g = spec.to_graph(optimize=False)
    ids = [g.node_id(o) for o in op_outs]
    outs = g.run({g.input_ids[0]: xd}, ids)
    torch.cuda.synchronize()
    bad = 0
    for n, o, t in zip([n for n in spec.nodes if n.kind == "op"], op_outs, outs):
        got = t.cpu().numpy()
        if not bits_equal(got, exp_all[o]):
            d = np.abs(got.astype(np.float64) - exp_all[o])
            print(f"DIFF {n.name} {n.op_type} {n.attrs} shape={got.shape} max_abs={d.max():.3g} "
                  f"n={(d > 0).sum()}", flush=True)
            bad += 1
            if bad >= 5:
                break
    print("per-op bad:", bad, flush=True)


if __name__ == "__main__":
    main()
