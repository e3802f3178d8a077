set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=$PWD/gpurun_out/r6k; mkdir -p $O
R=$PWD
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $O/pmc_bert -o run -- python3 $R/rten-fork_amd/tools/model_once.py 2 bert 32 > $O/pmc_bert.log 2>&1 || { tail -5 $O/pmc_bert.log; exit 1; }
cd $R
python3 rten-fork_amd/tools/pmc_dispatch.py $O/pmc_bert 2 > $O/dispatch_bert.txt; rm -rf $O/pmc_bert
head -40 $O/dispatch_bert.txt
