#!/bin/bash
# gemv (M == 1) parity tests, then the batch-1 ResNet-50 bench + profile.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/b1
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q -k "gemv or gemm" --timeout 120 --timeout-method thread > gpurun_out/b1/pytest.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/b1/pytest.log; exit 1; }
tail -2 gpurun_out/b1/pytest.log
bash scripts/gpu_batch1.sh
