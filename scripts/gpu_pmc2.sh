#!/bin/bash
# Two PMC passes (SQ timing/instruction mix) for one conv layer:
#   PMC_TAG=name RTENHIP_DMA_CFG=n bash scripts/gpu_pmc2.sh N C H W O k stride pad
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
ARGS="$@ -1 5"
TAG=${PMC_TAG:-l}
P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc2 -o ${TAG}_$i -- python3 rten-fork_amd/tools/onelayer.py $ARGS > gpurun_out/pmc2_${TAG}_$i.log 2>&1 || exit $?
done
