#!/bin/bash
# Tests of the changed kernels, fused expand+depthwise timing + SQ counters,
# BERT / MobileNetV2 bench lines, ResNet-50 b1 side-stream A/B and trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/combo; mkdir -p $O
export RTEN_NUM_THREADS=8
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_conv_pointwise_gpu.py tests/test_model_gpu.py \
  -k "expand or attention or bert or mobilenet or matmul or layernorm" > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/gpu_r3_mbpmc.sh || exit 1
for m in "mnv2 --model mobilenet_v2 --batch 128" "bert --model bert --batch 32"; do
  set -- $m; n=$1; shift
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --timing-report "$@" > $O/$n.json 2> $O/$n.txt || { tail $O/$n.txt; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n', d['value'], d['ms_per_step'])"
done
bash scripts/gpu_r3_b1prof.sh || exit 1
