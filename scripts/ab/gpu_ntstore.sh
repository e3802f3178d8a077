#!/bin/bash
# Non-temporal epilogue stores in the DMA conv GEMM (RTENHIP_NT_STORE=1) vs
# plain stores: ResNet-50 b64 and MobileNetV2 b128, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/nt_${1:-now}; mkdir -p $O
run() {  # tag model batch steps env...
  local tag=$1 model=$2 batch=$3 steps=$4; shift 4
  env "$@" timeout -k 10 300 python -u bench.py --model $model --batch $batch --steps $steps --warmup 10 --no-secondary --no-cpu-baseline \
    > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -3 $O/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$tag.json $tag
}
for i in 1 2; do run r_off$i resnet50 64 60 RTENHIP_NT_STORE=0; run r_on$i resnet50 64 60 RTENHIP_NT_STORE=1; done
for i in 1 2; do run m_off$i mobilenet_v2 128 60 RTENHIP_NT_STORE=0; run m_on$i mobilenet_v2 128 60 RTENHIP_NT_STORE=1; done
