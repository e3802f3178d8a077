#!/bin/bash
# Per-layer conv microbenchmark under every DMA tile config, plus the
# no-DMA (mode 1) and no-MFMA (mode 2) timing experiments.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
CFGS=${CFGS:-d0,d1,d2,d3,d4,d5,d6,d7,d8,d9,d10,d11,d12,d13,d14,d15,d16,d17,d18}
timeout -k 10 300 python rten-fork_amd/tools/convbench.py --cfgs $CFGS > gpurun_out/convbench_m0.log 2>&1 || { echo m0 failed; tail gpurun_out/convbench_m0.log; exit 1; }
timeout -k 10 300 python rten-fork_amd/tools/convbench.py --cfgs $CFGS --dmamode 1 > gpurun_out/convbench_m1.log 2>&1 || { echo m1 failed; exit 1; }
timeout -k 10 300 python rten-fork_amd/tools/convbench.py --cfgs $CFGS --dmamode 2 > gpurun_out/convbench_m2.log 2>&1 || { echo m2 failed; exit 1; }
echo done
