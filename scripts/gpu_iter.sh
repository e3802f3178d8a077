#!/bin/bash
# Iteration check: selected GPU parity tests (PYTEST_K) + ResNet-50 per-layer timing bench.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$PYTEST_K" > gpurun_out/pytest_iter.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_iter.log; exit 1; }
  tail -2 gpurun_out/pytest_iter.log
fi
timeout -k 10 400 python bench.py --no-cpu-baseline --timing-report --steps 20 ${BENCH_ARGS} > gpurun_out/layers.log 2> gpurun_out/layers.err || { echo bench failed; tail gpurun_out/layers.err; exit 1; }
cat gpurun_out/layers.log
grep "^op " gpurun_out/layers.err | awk '{printf "%-22s %8s %s %s %s %s %s %s %s\n", $2, $5, $7,$8,$9,$10,$11,$12,$13}'
