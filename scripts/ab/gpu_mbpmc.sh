#!/bin/bash
# PMC counters of the fused inverted residual block (tools/mb_bench.py,
# features index $1, default 5): one rocprofv3 pass per counter group.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/mbpmc; mkdir -p $O
B=${1:-5}
export RTENHIP_GRAPH=0  # eager dispatches: counters attribute per kernel
export RTENHIP_MBCONV=all
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run \
    -- python3 rten-fork_amd/tools/mb_bench.py $B > $O/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail $O/p$i.log; exit 1; }
  python3 rten-fork_amd/tools/pmc_kernels.py $O/p$i mbconv > $O/sum_$i.txt 2>&1 || { cat $O/sum_$i.txt; exit 1; }
  rm -rf $O/p$i
  cat $O/sum_$i.txt
done
