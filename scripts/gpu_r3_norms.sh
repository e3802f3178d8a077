#!/bin/bash
# LogSoftmax / InstanceNormalization parity, then the round-3 full check.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
export RTEN_NUM_THREADS=8
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py \
  -k "log_softmax or instance_norm" > gpurun_out/r3_norms.log 2>&1 || { tail -30 gpurun_out/r3_norms.log; exit 1; }
tail -1 gpurun_out/r3_norms.log
bash scripts/gpu_r3_full.sh
