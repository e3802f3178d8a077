#!/bin/bash
# Fused expand+depthwise kernels at MobileNetV2 b128 shapes: timing, then SQ
# counter passes (one pass per counter group).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/mbpmc; mkdir -p $O
timeout -k 10 200 python3 rten-fork_amd/tools/mbconv_bench.py 10 > $O/bench.txt 2>&1 || { tail $O/bench.txt; exit 1; }
cat $O/bench.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
  --output-format csv -d $O/p1 -o p1 -- python3 rten-fork_amd/tools/mbconv_bench.py 2 > $O/p1.log 2>&1 || { tail $O/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE \
  --output-format csv -d $O/p2 -o p2 -- python3 rten-fork_amd/tools/mbconv_bench.py 2 > $O/p2.log 2>&1 || { tail $O/p2.log; exit 1; }
python3 rten-fork_amd/tools/pmc_kernels.py $O expand > $O/pmc.txt && cat $O/pmc.txt
rm -rf $O/p1 $O/p2
