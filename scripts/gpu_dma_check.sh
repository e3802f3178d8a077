#!/bin/bash
# DMA GEMM change check: conv/matmul GPU parity tests, then the per-layer
# config sweep.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/dma_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/dma_tests.log; exit 1; }
tail -2 gpurun_out/dma_tests.log
CFGS=${CFGS:-d0,d1,d2,d3,d4,d5,d6,d7,d8,d9,d10,d11,d12,d13,d14,d15,d16,d17,d18}
timeout -k 10 300 python rten-fork_amd/tools/convbench.py --cfgs $CFGS > gpurun_out/convbench.log 2>&1 || { echo convbench failed; tail gpurun_out/convbench.log; exit 1; }
cat gpurun_out/convbench.log
