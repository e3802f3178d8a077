#!/bin/bash
# PMC pass 1 (SQ timing) for one conv layer under the normal build and the
# exp4 (MFMA-only) build.  usage: bash scripts/gpu_pmc_exp.sh
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/pmc2
SHAPE=${SHAPE:-"64 256 14 14 256 3 1 1"}
P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS"
run() {  # tag lib cfg pass counters
  RTENHIP_LIB=$PWD/rten-fork_amd/$2/librten_hip.so RTENHIP_DMA_CFG=$3 timeout -s KILL 100 rocprofv3 --pmc $5 --output-format csv -d gpurun_out/pmc2 -o $1_$4 -- python3 rten-fork_amd/tools/onelayer.py $SHAPE -1 5 > gpurun_out/pmc2_$1_$4.log 2>&1
}
for v in "n14 . 14" "e4 exp4 1" "e0 exp0 1"; do
  set -- $v
  run $1 $2 $3 1 "$P1" && run $1 $2 $3 2 "$P2" || { echo "$1 failed"; tail -5 gpurun_out/pmc2_$1_*.log; exit 1; }
  python3 rten-fork_amd/tools/pmc_layer.py gpurun_out/pmc2 $1
done
