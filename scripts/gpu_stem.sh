#!/bin/bash
# Stem conv bound probe: stride-2 7x7 vs a stride-1 7x7 of the same GEMM shape,
# with the K-loop DMA or the MFMAs switched off (timing experiment modes).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for m in 0 1 2; do
  echo "== dmamode $m"
  timeout -k 10 200 python3 rten-fork_amd/tools/convbench.py --iters 10 --cfgs ${CFGS:-d20,d22,d24} --dmamode $m \
    --shape 64,3,224,224,64,7,2,3 --shape 64,3,112,112,64,7,1,3 > gpurun_out/stem_$m.log 2>&1 || { echo failed; tail gpurun_out/stem_$m.log; exit 1; }
  cat gpurun_out/stem_$m.log
done
