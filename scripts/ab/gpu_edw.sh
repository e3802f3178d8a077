#!/bin/bash
# MobileNetV2 b128: fused expand+depthwise on every eligible pair
# (RTENHIP_EXPAND_DW=all) vs the default (features.2 only); interleaved bench
# lines and the per-op reports.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/edw; mkdir -p $O
run() {
  local tag=$1 v=$2
  RTENHIP_EXPAND_DW=$v timeout -k 10 240 python3 bench.py --model mobilenet_v2 --batch 128 --no-cpu-baseline --no-secondary --steps 20 --warmup 3 > $O/$tag.json 2> $O/$tag.err \
    || { echo "bench $tag failed"; tail $O/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$tag.json $tag
}
for r in 1 2; do run def$r default && run all$r all || exit 1; done
for v in default all; do
  RTENHIP_EXPAND_DW=$v timeout -k 10 200 python3 rten-fork_amd/tools/model_once.py 2 mobilenet_v2 128 --report > $O/rep_$v.txt 2>&1 || { tail $O/rep_$v.txt; exit 1; }
  grep -E "^op features\.[1-6]\." $O/rep_$v.txt | head -24
done
