"""LayerNorm launch timing probe: BERT-base shape (4096 x 768), 200 launches.

Run under ``rocprofv3 --kernel-trace --stats`` for per-launch durations;
RTENHIP_LN_ROWS selects the rows per workgroup (experiments only).
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import rten_hip as rh  # noqa: E402

rows, length = int(os.environ.get("LN_ROWS_TOTAL", 4096)), 768
g = torch.Generator(device="cpu").manual_seed(5)
x = (torch.rand(rows, length, generator=g) * 4 - 2).cuda()
sc = (torch.rand(length, generator=g) + 1).cuda()
bi = torch.rand(length, generator=g).cuda()
for _ in range(200):
    y = rh.layer_normalization(x, sc, bi, -1, 1e-12)
if os.environ.get("LN_COPY"):  # HBM floor of the same bytes: one device copy
    z = torch.empty_like(x)
    for _ in range(200):
        z.copy_(x)
torch.cuda.synchronize()
print("ln_bench done", float(y.sum()))
