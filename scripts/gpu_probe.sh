#!/bin/bash
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rten-fork_amd/tools/mfma_shape_probe > gpurun_out/mfma_shape_probe.log 2>&1 || { echo probe failed; cat gpurun_out/mfma_shape_probe.log; exit 1; }
cat gpurun_out/mfma_shape_probe.log
