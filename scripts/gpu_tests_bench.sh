#!/bin/bash
# GPU parity suite, smoke and the default bench line; each GPU step has its
# own time limit and the script stops at the first failure.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { echo bench failed; exit 1; }
cat gpurun_out/bench.log
