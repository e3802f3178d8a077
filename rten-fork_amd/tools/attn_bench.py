"""FusedAttention launch timing at BERT-base b32 (B=32, H=12, S=128, D=64),
with q / k / v laid out as BERT's projections leave them ([B, S, 768] rows,
heads by Reshape + Transpose, k transposed to [B, H, D, S]) and a [B, 1, 1, S]
additive mask.  200 replays; run under ``rocprofv3 --kernel-trace --stats``.
RTENHIP_LIB=.../exp_att/librten_hip_attN.so selects an experiment build
(csrc/attention.hip RTENHIP_ATT_EXPERIMENT; timing only, results not checked).
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from rten_hip.graph import ModelSpec  # noqa: E402

B, H, S, D = 32, 12, 128, 64
m = ModelSpec("attn_bert")
m.inputs = ["q", "k", "v", "mask"]
for n in m.inputs:
    m.value(n)
heads = m.const("heads", np.array([0, 0, H, D], np.float32))
q = m.op("Transpose", [m.op("Reshape", ["q", heads])], {"perm": [0, 2, 1, 3]})
k = m.op("Transpose", [m.op("Reshape", ["k", heads])], {"perm": [0, 2, 3, 1]})
v = m.op("Transpose", [m.op("Reshape", ["v", heads])], {"perm": [0, 2, 1, 3]})
s = m.op("Div", [m.op("MatMul", [q, k]), m.const("scale", np.array([8.0], np.float32))])
s = m.op("Softmax", [m.op("Add", [s, "mask"])], {"axis": -1})
o = m.op("Transpose", [m.op("MatMul", [s, v])], {"perm": [0, 2, 1, 3]})
m.outputs = [o]
g = m.to_graph()
rng = np.random.default_rng(3)
ins = [torch.from_numpy(rng.uniform(-1, 1, (B, S, H * D)).astype(np.float32)).cuda() for _ in range(3)]
ins.append(torch.zeros(B, 1, 1, S).cuda())
dev = {g.input_ids[i]: t for i, t in enumerate(ins)}
out = None
for _ in range(200):
    out = g.run(dev, g.output_ids, out=out)
torch.cuda.synchronize()
print("attn_bench done", os.environ.get("RTENHIP_LIB", "product"), float(out[0].float().abs().sum()))
