#!/bin/bash
# Per-layer times with the DMA GEMM launch mode forced (RTENHIP_PERSIST=0,2,3,4).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for m in 0 2 3 4; do
  RTENHIP_PERSIST=$m timeout -k 10 300 python bench.py --no-cpu-baseline --timing-report --steps 10 > gpurun_out/pc_$m.log 2> gpurun_out/pc_$m.err || { echo bench $m failed; tail gpurun_out/pc_$m.err; exit 1; }
done
python3 - <<'PY'
import re
rows={}
for m in "0234":
    for line in open(f"gpurun_out/pc_{m}.err"):
        if line.startswith("op "):
            f=line.split(); rows.setdefault(f[1],{})[m]=float(f[4])
tot={m:0 for m in "0234"}
for k,v in rows.items():
    print(f"{k:22s} "+" ".join(f"{v.get(m,0):8.4f}" for m in "0234"))
    for m in "0234": tot[m]+=v.get(m,0)
print("total", tot)
for m in "0234": print(m, open(f"gpurun_out/pc_{m}.log").read()[:120])
PY
