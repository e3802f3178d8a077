set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=$PWD/gpurun_out/r6f; mkdir -p $O
R=$PWD
for cfg in "mobilenet_v2 128" "bert 32"; do
  set -- $cfg
  cd /tmp
  timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $O/pmc_$1 -o run -- python3 $R/rten-fork_amd/tools/model_once.py 2 $1 $2 > $O/pmc_$1.log 2>&1 || { tail -5 $O/pmc_$1.log; exit 1; }
  cd $R
  python3 rten-fork_amd/tools/pmc_dispatch.py $O/pmc_$1 2 > $O/dispatch_$1.txt; rm -rf $O/pmc_$1
  timeout -k 10 300 python -u rten-fork_amd/tools/model_once.py 1 $1 $2 --report > $O/report_$1.txt 2>&1 || exit 1
done
echo ok
