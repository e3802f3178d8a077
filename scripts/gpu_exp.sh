#!/bin/bash
# DMA-GEMM timing experiments: convbench under the exp0 (normal), exp1 (no
# K-loop DMA) and exp2 (no MFMA) builds of rten-fork_amd/build_exp.sh.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for m in ${MODES:-0 1 2}; do
  RTENHIP_LIB=$PWD/rten-fork_amd/exp$m/librten_hip.so timeout -k 10 200 python rten-fork_amd/tools/convbench.py --cfgs ${CFGS:-d0,d1,d2,d3} > gpurun_out/exp$m.log 2>&1 || { echo exp$m failed; tail gpurun_out/exp$m.log; exit 1; }
  echo "== mode $m"; grep -v amdgpu.ids gpurun_out/exp$m.log
done
