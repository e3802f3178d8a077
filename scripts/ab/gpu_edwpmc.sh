#!/bin/bash
# SQ counters of MobileNetV2 b128's kernel families (eager forwards, RTENHIP_GRAPH=0;
# the first forward's tuning launches are included for the tuned GEMM families):
# where the fused expand+depthwise kernels' time goes (next round's MFMA-expand plan).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/edwpmc; mkdir -p $O
export RTENHIP_GRAPH=0
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run \
    -- python3 rten-fork_amd/tools/model_once.py 2 mobilenet_v2 128 > $O/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail $O/p$i.log; exit 1; }
  python3 rten-fork_amd/tools/pmc_kernels.py $O/p$i rtenhip > $O/sum_$i.txt 2>&1 || { cat $O/sum_$i.txt; exit 1; }
  rm -rf $O/p$i
  cat $O/sum_$i.txt
done
