#!/bin/bash
# ResNet-50 b64: the dual conv3 + downsample GEMM as tuned vs never
# (RTENHIP_NO_DUAL=1), interleaved, plus the tuner's dual decisions.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/dualab_${1:-now}; mkdir -p $O
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-secondary --no-cpu-baseline \
    > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -3 $O/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$tag.json $tag
}
for i in 1 2; do run dual$i RTENHIP_DUAL_DEBUG=1; run nodual$i RTENHIP_NO_DUAL=1; done
grep -h "dual" $O/dual1.err | head -12
