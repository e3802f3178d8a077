#!/bin/bash
# Dual DMA GEMM (conv3 + downsample) as one continuous K loop
# (DmaDesc::dual_one) vs two passes: parity both ways, the ResNet-50 b64
# per-op report both ways, and an interleaved bench A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/dual${TAG:-}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_model_gpu.py -k "dual or resnet" > $O/t1.log 2>&1 || { tail -30 $O/t1.log; exit 1; }
tail -1 $O/t1.log
RTENHIP_DMA_DUAL1=0 timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_model_gpu.py -k "dual" > $O/t0.log 2>&1 || { tail -30 $O/t0.log; exit 1; }
tail -1 $O/t0.log
for v in 1 0; do
  RTENHIP_DMA_DUAL1=$v timeout -k 10 200 python3 rten-fork_amd/tools/model_once.py 2 resnet50 64 --report > $O/rep$v.txt 2>&1 || { tail $O/rep$v.txt; exit 1; }
  grep -E "dual" $O/rep$v.txt | head -8
done
run() {
  local tag=$1 v=$2
  RTENHIP_DMA_DUAL1=$v timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-secondary --steps 20 --warmup 3 > $O/$tag.json 2> $O/$tag.err \
    || { echo "bench $tag failed"; tail $O/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$tag.json $tag
}
for r in 1 2; do run one$r 1 && run two$r 0 || exit 1; done
