#!/bin/bash
# PMC (SQ timing + instruction mix) of one conv layer, cfg 14 (64x64, 4 stages),
# one block per item vs persistent with 3 and 4 blocks per CU.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/pmc2
SHAPE=${SHAPE:-"64 256 14 14 256 3 1 1"}
P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS"
run() {  # tag persist pass counters
  RTENHIP_DMA_CFG=14 RTENHIP_DMA_PERSIST=$2 timeout -s KILL 100 rocprofv3 --pmc $4 --output-format csv -d gpurun_out/pmc2 -o $1_$3 -- python3 rten-fork_amd/tools/onelayer.py $SHAPE -1 5 > gpurun_out/pmc2_$1_$3.log 2>&1
}
for v in "p0 -1" "p3 3" "p4 4"; do
  set -- $v
  run $1 $2 1 "$P1" && run $1 $2 2 "$P2" || { echo "$1 failed"; tail -5 gpurun_out/pmc2_$1_*.log; exit 1; }
  python3 rten-fork_amd/tools/pmc_layer.py gpurun_out/pmc2 $1
done
