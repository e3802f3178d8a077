#!/bin/bash
# Targeted GPU check: the tests named by $1 (pytest -k expression), then an
# optional bench line for model $2.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$1" > gpurun_out/quick_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/quick_tests.log; exit 1; }
tail -3 gpurun_out/quick_tests.log
if [ -n "$2" ]; then
  timeout -k 10 300 python bench.py --model $2 $3 --no-cpu-baseline --timing-report > gpurun_out/quick_bench.log 2> gpurun_out/quick_bench.err || { echo bench failed; tail -20 gpurun_out/quick_bench.err; exit 1; }
  cat gpurun_out/quick_bench.log
fi
