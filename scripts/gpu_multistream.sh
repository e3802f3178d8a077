#!/bin/bash
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 500 python rten-fork_amd/tools/multistream.py 64 1 2 4 > gpurun_out/multistream.log 2>&1 || { echo failed; tail -20 gpurun_out/multistream.log; exit 1; }
grep -v amdgpu.ids gpurun_out/multistream.log
