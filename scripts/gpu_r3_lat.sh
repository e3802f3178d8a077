#!/bin/bash
# Latency GEMM (ResNet-50 batch 1) bring-up: bit-exact tests, then the b1 and
# MobileNetV2 bench lines with timing reports.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export RTEN_NUM_THREADS=8
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_conv_lat_gpu.py -k "not resnet50" > gpurun_out/lat_tests.log 2>&1 \
  || { echo "lat tests failed"; tail -40 gpurun_out/lat_tests.log; exit 1; }
tail -3 gpurun_out/lat_tests.log
timeout -k 10 300 $PYT tests/test_conv_lat_gpu.py -k "resnet50" tests/test_conv_pointwise_gpu.py -k "resnet50 or expand or mobilenet" > gpurun_out/lat_tests2.log 2>&1 \
  || { echo "lat tests 2 failed"; tail -40 gpurun_out/lat_tests2.log; exit 1; }
tail -3 gpurun_out/lat_tests2.log
timeout -k 10 300 python -u bench.py --batch 1 --steps 50 --no-cpu-baseline --timing-report > gpurun_out/lat_bench_b1.json 2> gpurun_out/lat_bench_b1.err || exit 1
cat gpurun_out/lat_bench_b1.json
timeout -k 10 300 python -u bench.py --model mobilenet_v2 --batch 128 --no-cpu-baseline --timing-report > gpurun_out/lat_bench_mnv2.json 2> gpurun_out/lat_bench_mnv2.err || exit 1
head -c 400 gpurun_out/lat_bench_mnv2.json
