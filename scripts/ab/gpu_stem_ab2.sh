#!/bin/bash
# ResNet-50 b64 with / without the stem candidate: longer interleaved runs and
# the per-op report of conv1 in each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/stemab2_${1:-now}; mkdir -p $O
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --batch 64 --steps 100 --warmup 10 --no-secondary --no-cpu-baseline \
    > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -3 $O/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$tag.json $tag
}
for i in 1 2 3; do run off$i RTENHIP_STEM=0; run on$i RTENHIP_STEM=1; done
for v in 0 1; do
  RTENHIP_STEM=$v timeout -k 10 300 python -u rten-fork_amd/tools/model_once.py 1 resnet50 64 --report > $O/report_$v.txt 2>&1 || { echo "report failed"; tail -5 $O/report_$v.txt; exit 1; }
  grep "op conv1 \|op maxpool\|op layer1.0.conv1 " $O/report_$v.txt
done
