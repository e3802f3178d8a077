#!/bin/bash
# stem_dw_project_kernel: kernel trace + two PMC passes over MobileNetV2 b128
# eager forwards (tools/model_once.py); per-kernel counter means.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
R=$PWD
O=$PWD/gpurun_out/sdpmc_${1:-now}; mkdir -p $O
M="python3 $R/rten-fork_amd/tools/model_once.py 2 mobilenet_v2 128"
cd /tmp
[ -n "$SKIP_KT" ] || timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $M > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- $M > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o run -- $M > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
cd $R
python3 - "$O" <<'PY'
import csv, glob, sys
O = sys.argv[1]
for f in glob.glob(O + "/kt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "dw_project" in r.get("Name", "") or "expand_dw" in r.get("Name", ""):
            print("stats", r.get("Name", "")[:70], r.get("Calls"), r.get("AverageNs"))
PY
python3 rten-fork_amd/tools/pmc_kernels.py $O/p1 dw_project
python3 rten-fork_amd/tools/pmc_kernels.py $O/p2 dw_project
rm -rf $O/p1 $O/p2
