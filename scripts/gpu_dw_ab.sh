#!/bin/bash
# Depthwise change: its GPU parity tests, dwbench under both builds, then a
# MobileNetV2 A/B (ab_base vs ab_dw).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
RTENHIP_LIB=$PWD/rten-fork_amd/ab_dw/librten_hip.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "depthwise or mobilenet or dw" > gpurun_out/dw_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/dw_tests.log; exit 1; }
tail -2 gpurun_out/dw_tests.log
for v in ab_base ab_dw; do
  echo "== $v"; RTENHIP_LIB=$PWD/rten-fork_amd/$v/librten_hip.so timeout -k 10 120 python3 rten-fork_amd/tools/dwbench.py > gpurun_out/dwbench_$v.log 2>&1 || { echo dwbench failed; tail gpurun_out/dwbench_$v.log; exit 1; }
  cat gpurun_out/dwbench_$v.log
done
VARS="ab_base ab_dw" BENCH_ARGS="--model mobilenet_v2 --batch 128" bash scripts/gpu_abn.sh
