#!/bin/bash
# BERT b32: packed-A producer stores on / off (RTENHIP_NO_PK_OUT, RTENHIP_ATTN_PK), interleaved bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/bertpk; mkdir -p $O
for v in base nopk noattnpk base nopk noattnpk; do
  case $v in base) E="";; nopk) E="RTENHIP_NO_PK_OUT=1";; noattnpk) E="RTENHIP_ATTN_PK=0";; esac
  env $E timeout -k 10 300 python -u bench.py --model bert --batch 32 --no-cpu-baseline --no-secondary --steps 30 --warmup 5 > $O/$v.json 2> $O/$v.err || { echo "bench failed $v"; tail -5 $O/$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$v.json $v
done
