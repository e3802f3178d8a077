#!/bin/bash
# Placement / phase stamps of the DMA conv GEMM (experiment build 5, see
# rten-fork_amd/build_exp.sh) on given layers.  usage: SHAPES="N C H W O k s p cfg persist;..." bash scripts/gpu_place.sh
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
IFS=';' read -ra LIST <<< "${SHAPES:-64 256 14 14 256 3 1 1 1 0}"
for sh in "${LIST[@]}"; do
  echo "== $sh"
  RTENHIP_LIB=$PWD/rten-fork_amd/exp5/librten_hip.so timeout -k 10 100 python3 rten-fork_amd/tools/placement.py $sh 2>&1 | grep -v amdgpu.ids || exit 1
done
