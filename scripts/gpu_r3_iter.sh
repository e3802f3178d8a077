#!/bin/bash
# Iteration check: the tests of the kernels changed (latency GEMM, fused
# expand+depthwise, attention), then bench lines + timing reports for
# ResNet-50 b1, MobileNetV2 b128 and BERT b32.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/iter; mkdir -p $O
export RTEN_NUM_THREADS=8
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_conv_lat_gpu.py tests/test_conv_pointwise_gpu.py tests/test_model_gpu.py \
  -k "lat or chain or expand or attention or bert or mobilenet or matmul or side or layernorm" > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bench() {  # name, args
  local n=$1; shift
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --timing-report "$@" > $O/$n.json 2> $O/$n.txt || { tail $O/$n.txt; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n', d['value'], d['ms_per_step'])"
}
bench b1 --batch 1 --steps 200 --warmup 20
RTENHIP_SIDE_STREAM=0 bench b1_noside --batch 1 --steps 200 --warmup 20
bench mnv2 --model mobilenet_v2 --batch 128
bench bert --model bert --batch 32
if [ -n "$FULL" ]; then
  timeout -k 10 600 $PYT tests/test_full_size_gpu.py > $O/full.log 2>&1 || { echo "full-size failed"; tail -30 $O/full.log; exit 1; }
  tail -2 $O/full.log
fi
