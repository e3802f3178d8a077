#!/bin/bash
# Stem kernel PMC pass (forced stem, standalone), ResNet-50 b64.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=$PWD/gpurun_out/stempmc_${1:-now}; mkdir -p $O
R=$PWD
cd /tmp
RTENHIP_PW_VALU=800 timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/rten-fork_amd/tools/stem_bench.py ${2:-resnet50} ${3:-64} 5 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
RTENHIP_PW_VALU=800 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o run -- python3 $R/rten-fork_amd/tools/stem_bench.py ${2:-resnet50} ${3:-64} 5 > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
cd $R
python3 - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
ks = glob.glob(O + "/kt/**/*kernel_stats.csv", recursive=True)
for f in ks:
    for r in list(csv.DictReader(open(f)))[:6]:
        print("stats", r.get("Name", "")[:60], r.get("Calls"), r.get("AverageNs"))
pm = glob.glob(O + "/pmc/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(list)
for f in pm:
    for r in csv.DictReader(open(f)):
        if "stem" not in r.get("Kernel_Name", ""):
            continue
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print("pmc", k, len(v), sum(v) / len(v))
PY
