#!/bin/bash
# One PMC pass + kernel trace over a standalone tool run; prints the per-kernel
# averages of the kernels whose name contains $2.
# usage: gpu_kern_pmc.sh TAG NAME_SUBSTR TOOL ARGS...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=$PWD/gpurun_out/kpmc_$1; mkdir -p $O
SUB=$2; shift 2
R=$PWD
cd /tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/"$@" > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o run -- python3 $R/"$@" > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc2 -o run -- python3 $R/"$@" > $O/pmc2.log 2>&1 || { tail -5 $O/pmc2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc3 -o run -- python3 $R/"$@" > $O/pmc3.log 2>&1 || { tail -5 $O/pmc3.log; exit 1; }
cd $R
python3 - "$O" "$SUB" <<'PY'
import csv, glob, sys, collections
O, sub = sys.argv[1], sys.argv[2]
for f in glob.glob(O + "/kt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if sub in r.get("Name", ""):
            print("stats", r["Name"][:70], r.get("Calls"), r.get("AverageNs"))
acc = collections.defaultdict(list)
for f in glob.glob(O + "/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if sub in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print("pmc", k, len(v), sum(v) / len(v))
PY
