#!/bin/bash
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for sh in "64 256 14 14 256 3 1 1 1 0" "64 256 14 14 256 3 1 1 1 3" "64 256 14 14 256 3 1 1 1 4" "64 64 56 56 64 3 1 1 1 0" "64 64 56 56 64 3 1 1 1 3"; do
  echo "== $sh"
  RTENHIP_LIB=$PWD/rten-fork_amd/exp5/librten_hip.so timeout -k 10 100 python3 rten-fork_amd/tools/placement.py $sh 2>&1 | grep -v amdgpu.ids || exit 1
done
