#!/bin/bash
# Stem -> depthwise -> projection fusion (dw_project.hip stem_dw_project_kernel):
# parity (new kernel, the dw_project pair, full-size MobileNetV2 b128), then
# MobileNetV2 b128 with the stem apart or fused (RTENHIP_STEM_DWPW=0),
# interleaved, and the per-op report.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/stemdwpw_${1:-now}; mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_conv_pointwise_gpu.py -k "stem_dw_project or dw_project" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 $PYT tests/test_full_size_gpu.py -k mobilenet > $O/full.log 2>&1 || { echo "full-size failed"; tail -40 $O/full.log; exit 1; }
tail -1 $O/full.log
run() {  # tag model batch steps env...
  local tag=$1 model=$2 batch=$3 steps=$4; shift 4
  env "$@" timeout -k 10 300 python -u bench.py --model $model --batch $batch --steps $steps --warmup 10 --no-secondary --no-cpu-baseline \
    > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -3 $O/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$tag.json $tag
}
for i in 1 2; do run m_off$i mobilenet_v2 128 60 RTENHIP_STEM_DWPW=0; run m_on$i mobilenet_v2 128 60 RTENHIP_STEM_DWPW=1; done
timeout -k 10 300 python -u rten-fork_amd/tools/model_once.py 1 mobilenet_v2 128 --report > $O/report_m128.txt 2>&1 || { echo "report failed"; tail -5 $O/report_m128.txt; exit 1; }
grep "features.0\|features.1\.\|dw+project\|expand+dw" $O/report_m128.txt | head -12
