#!/bin/bash
# SQ counters of one conv layer's kernels (tools/conv_graph_time.py), one
# counter pass per run.  usage: SHAPE="..." MODE=332 bash scripts/gpu_pmc_conv.sh
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/pmc_conv
export RTENHIP_PW_VALU=$MODE
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc_conv -o p1 -- python3 rten-fork_amd/tools/conv_graph_time.py $SHAPE > gpurun_out/pmc_conv/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_BUSY_CYCLES \
  --output-format csv -d gpurun_out/pmc_conv -o p2 -- python3 rten-fork_amd/tools/conv_graph_time.py $SHAPE > gpurun_out/pmc_conv/p2.log 2>&1 || exit 1
echo pmc-ok
