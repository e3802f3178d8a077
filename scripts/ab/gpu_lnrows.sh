#!/bin/bash
# BERT-base b32: LayerNorm rows per workgroup (RTENHIP_LN_ROWS tuning knob) A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/lnrows_${1:-now}; mkdir -p $O
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --model bert --batch 32 --steps 40 --warmup 5 --no-secondary --no-cpu-baseline \
    > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -3 $O/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$tag.json $tag
}
for i in 1 2; do for r in 8 4 2 16; do run r${r}_$i RTENHIP_LN_ROWS=$r; done; done
