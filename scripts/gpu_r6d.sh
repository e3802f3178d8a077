set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash scripts/gpu_prof.sh r6a resnet50_b1 resnet50_b64 || exit 1
O=$PWD/gpurun_out/r6d; mkdir -p $O
R=$PWD
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $O/pmc -o run -- python3 $R/rten-fork_amd/tools/model_once.py 2 resnet50 64 > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
cd $R
python3 rten-fork_amd/tools/pmc_dispatch.py $O/pmc 2 > $O/dispatch_b64.txt; rm -rf $O/pmc
cat $O/dispatch_b64.txt
