#!/bin/bash
# Expand on MFMA inside the fused expand -> depthwise kernel
# (expand_dw_mfma_kernel): parity, then MobileNetV2 b128 with it or the
# VALU-expand banded kernel (RTENHIP_EDW_MFMA=0), interleaved, and the report.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/edwm_${1:-now}; mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_conv_pointwise_gpu.py -k "expand or mobilenet or dw_project" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
run() {  # tag model batch steps env...
  local tag=$1 model=$2 batch=$3 steps=$4; shift 4
  env "$@" timeout -k 10 300 python -u bench.py --model $model --batch $batch --steps $steps --warmup 10 --no-secondary --no-cpu-baseline \
    > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -3 $O/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$tag.json $tag
}
for i in 1 2; do run m_off$i mobilenet_v2 128 60 RTENHIP_EDW_MFMA=0; run m_on$i mobilenet_v2 128 60 RTENHIP_EDW_MFMA=1; done
for v in 0 1; do
  RTENHIP_EDW_MFMA=$v timeout -k 10 300 python -u rten-fork_amd/tools/model_once.py 1 mobilenet_v2 128 --report > $O/report_$v.txt 2>&1 || { echo "report failed"; tail -5 $O/report_$v.txt; exit 1; }
  grep "expand+dw\|features.[234].conv.1 \|features.[234].*dw" $O/report_$v.txt | head -6
done
