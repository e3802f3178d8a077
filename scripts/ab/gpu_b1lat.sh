#!/bin/bash
# ResNet-50 b1 with each latency-GEMM variant forced on every conv vs the
# per-layer tuned mix (the tuner times each conv alone, with its weights hot).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/b1lat_${1:-now}; mkdir -p $O
for v in -1 72 74 71 91 92 41 21 11 -1; do
  RTENHIP_LAT=$v timeout -k 10 300 python -u bench.py --batch 1 --steps 300 --warmup 30 --no-secondary --no-cpu-baseline \
    > $O/b1_$v.json 2> $O/b1_$v.err || { echo "bench $v failed"; tail -3 $O/b1_$v.err; continue; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('lat', sys.argv[2], d['value'], d['ms_per_step'])" $O/b1_$v.json $v
done
