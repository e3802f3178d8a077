#!/bin/bash
# ResNet-50 b64 stem: 7x7 stride-2 conv vs a stride-1 conv of the same GEMM
# shape (M=64, K=147, N=802816), per DMA config -- how much the stride-2
# gather of B costs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/stem3; mkdir -p $O
timeout -k 10 300 python3 rten-fork_amd/tools/convbench.py --cfgs d19,d13,d20,d21,d22 --iters 20 \
  --shape 64,3,224,224,64,7,2,3 --shape 64,3,112,112,64,7,1,3 > $O/cb.txt 2>&1 || { tail $O/cb.txt; exit 1; }
cat $O/cb.txt
