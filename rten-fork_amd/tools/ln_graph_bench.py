"""LayerNorm launch timing as BERT-base b32 runs it: [32, 128, 768] rows
through LayerNormalization into a MatMul, so the executor plans the LayerNorm
to also store the MatMul's packed A (csrc/norm.hip layer_norm_rows_kernel's
packed phase), and into a residual Add.  200 replays; run under
``rocprofv3 --kernel-trace --stats``.  RTENHIP_LIB=.../exp_ln/librten_hip_lnN.so
selects a timing-experiment build (RTENHIP_LN_EXPERIMENT; results unchecked).
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from rten_hip.graph import ModelSpec  # noqa: E402

rng = np.random.default_rng(4)
m = ModelSpec("ln_bert")
m.inputs = ["x"]
m.value("x")
g_ = m.const("gamma", (1 + rng.uniform(-0.1, 0.1, 768)).astype(np.float32))
b_ = m.const("beta", rng.uniform(-0.1, 0.1, 768).astype(np.float32))
h = m.op("LayerNormalization", ["x", g_, b_], {"axis": -1, "epsilon": 1e-12})
w = m.const("w", rng.uniform(-0.05, 0.05, (768, 768)).astype(np.float32))
bb = m.const("b", rng.uniform(-0.01, 0.01, 768).astype(np.float32))
y = m.op("Add", [m.op("Add", [m.op("MatMul", [h, w]), bb]), h])
m.outputs = [y]
g = m.to_graph()
x = torch.from_numpy(rng.uniform(-2, 2, (32, 128, 768)).astype(np.float32)).cuda()
out = None
for _ in range(200):
    out = g.run({g.input_ids[0]: x}, g.output_ids, out=out)
torch.cuda.synchronize()
print("ln_graph_bench done", os.environ.get("RTENHIP_LIB", "product"), float(out[0].abs().sum()))
