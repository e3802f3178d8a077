#!/bin/bash
# Round 3: full-size parity tests for the BASELINE configs, then bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export RTEN_NUM_THREADS=8
timeout -k 10 300 python -u -m pytest tests/test_threads.py tests/test_conv_pointwise_gpu.py -k "thread or misaligned" -x -v \
  --timeout 120 --timeout-method thread > gpurun_out/r3_quick.log 2>&1 || { echo "quick tests failed"; tail -30 gpurun_out/r3_quick.log; exit 1; }
tail -3 gpurun_out/r3_quick.log
timeout -k 10 900 python -u -m pytest tests/test_full_size_gpu.py -x -v --timeout 600 --timeout-method thread \
  > gpurun_out/r3_full.log 2>&1 || { echo "full-size tests failed"; tail -30 gpurun_out/r3_full.log; exit 1; }
tail -5 gpurun_out/r3_full.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err || exit 1
cat gpurun_out/r3_bench.json
timeout -k 10 300 python -u bench.py --batch 1 --steps 50 --no-cpu-baseline > gpurun_out/r3_bench_b1.json 2>> gpurun_out/r3_bench.err || exit 1
cat gpurun_out/r3_bench_b1.json
