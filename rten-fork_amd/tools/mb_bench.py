"""Fused inverted residual block launch timing at MobileNetV2 b128 shapes:
one block per run (argv: features index 1..13, default 3), 50 replays, run
under ``rocprofv3 --kernel-trace --stats``.  RTENHIP_LIB selects a timing
experiment build (csrc/mbconv_block.hip RTENHIP_MB_EXPERIMENT); RTENHIP_MBCONV=0
runs the block's convs apart for comparison.  Results are not checked."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from rten_hip.graph import ModelSpec  # noqa: E402

# features index -> (C_in, H, hidden, C_out, stride)
BLOCKS = {1: (32, 112, 0, 16, 1), 2: (16, 112, 96, 24, 2), 3: (24, 56, 144, 24, 1), 4: (24, 56, 144, 32, 2),
          5: (32, 28, 192, 32, 1), 7: (32, 28, 192, 64, 2), 8: (64, 14, 384, 64, 1), 11: (64, 14, 384, 96, 1),
          12: (96, 14, 576, 96, 1)}
idx = int(sys.argv[1]) if len(sys.argv) > 1 else 3
C, H, M, O, s = BLOCKS[idx]
rng = np.random.default_rng(idx)
m = ModelSpec(f"features{idx}")
x = m.value("x")
m.inputs = ["x"]
lo, hi = m.const("lo", np.array(0.0, np.float32)), m.const("hi", np.array(6.0, np.float32))
e = x
if M:
    e = m.op("Clip", [m.op("Conv", [x, m.const("we", rng.uniform(-0.3, 0.3, (M, C, 1, 1)).astype(np.float32)),
                                    m.const("be", rng.uniform(-0.1, 0.1, M).astype(np.float32))],
                           {"pads": [0, 0, 0, 0], "strides": [1, 1]}), lo, hi])
hid = M or C
d = m.op("Clip", [m.op("Conv", [e, m.const("wd", rng.uniform(-0.3, 0.3, (hid, 1, 3, 3)).astype(np.float32)),
                                m.const("bd", rng.uniform(-0.1, 0.1, hid).astype(np.float32))],
                       {"pads": [1, 1, 1, 1], "strides": [s, s], "groups": hid}), lo, hi])
y = m.op("Conv", [d, m.const("wp", rng.uniform(-0.1, 0.1, (O, hid, 1, 1)).astype(np.float32)),
                  m.const("bp", rng.uniform(-0.1, 0.1, O).astype(np.float32))], {"pads": [0, 0, 0, 0], "strides": [1, 1]})
if s == 1 and C == O:
    y = m.op("Add", [y, x])
m.outputs = [y]
g = m.to_graph()
xd = torch.from_numpy(rng.uniform(-1, 2, (128, C, H, H)).astype(np.float32)).cuda()
out = None
for _ in range(50):
    out = g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
torch.cuda.synchronize()
print("mb_bench done", idx, os.environ.get("RTENHIP_LIB", "product"), os.environ.get("RTENHIP_MBCONV", ""))
