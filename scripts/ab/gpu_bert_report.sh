#!/bin/bash
# BERT-base b32: eager per-op report (configs, TF/s) and one PMC pass per
# dispatch (MFMA busy, wave states) over the last eager forward.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
R=$PWD
O=$PWD/gpurun_out/bertrep_${1:-now}; mkdir -p $O
timeout -k 10 300 python -u rten-fork_amd/tools/model_once.py 1 bert 32 --report > $O/report.txt 2>&1 || { echo "report failed"; tail -5 $O/report.txt; exit 1; }
grep "^op " $O/report.txt | head -20
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $O/pmc -o run -- python3 $R/rten-fork_amd/tools/model_once.py 2 bert 32 > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
cd $R
python3 rten-fork_amd/tools/pmc_dispatch.py $O/pmc 2 > $O/dispatch.txt
rm -rf $O/pmc
head -30 $O/dispatch.txt
