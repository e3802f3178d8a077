#!/bin/bash
# PMC passes (SQ timing / instruction mix) for a few conv layers x DMA configs.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
run() { PMC_TAG=$1 RTENHIP_DMA_CFG=$2 bash scripts/gpu_pmc2.sh $3 || exit 1; }
run l20c1_d1 1 "64 256 56 56 128 1 1 0"
run l20c1_d7 7 "64 256 56 56 128 1 1 0"
run l20c1_d0 0 "64 256 56 56 128 1 1 0"
for t in l20c1_d1 l20c1_d7 l20c1_d0; do python3 rten-fork_amd/tools/pmc_layer.py gpurun_out/pmc2 $t; done
timeout -k 10 100 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS --output-format csv -d gpurun_out/pmc3 -o d1 -- python3 rten-fork_amd/tools/onelayer.py 64 256 56 56 128 1 1 0 -1 5 > gpurun_out/pmc3.log 2>&1 || { echo pmc3 failed; tail -5 gpurun_out/pmc3.log; }
