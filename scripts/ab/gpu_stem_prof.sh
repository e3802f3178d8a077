#!/bin/bash
# Stem kernel standalone: forced MFMA stem vs the tuner without it, and the
# rocprof kernel statistics of each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=$PWD/gpurun_out/stemprof_${1:-now}; mkdir -p $O
T=rten-fork_amd/tools/stem_bench.py
for mdl in "resnet50 64" "mobilenet_v2 128" "resnet50 1"; do
  RTENHIP_PW_VALU=800 timeout -k 10 120 python -u $T $mdl 50 >> $O/times.txt 2>&1 || { tail -5 $O/times.txt; exit 1; }
  RTENHIP_STEM=0 timeout -k 10 120 python -u $T $mdl 50 >> $O/times.txt 2>&1 || { tail -5 $O/times.txt; exit 1; }
done
cat $O/times.txt
R=$PWD
cd /tmp
RTENHIP_PW_VALU=800 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_r -o run -- python3 $R/$T resnet50 64 20 > $O/prof_r.log 2>&1 || { tail -5 $O/prof_r.log; exit 1; }
RTENHIP_PW_VALU=800 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_m -o run -- python3 $R/$T mobilenet_v2 128 20 > $O/prof_m.log 2>&1 || { tail -5 $O/prof_m.log; exit 1; }
find $O -name "*kernel_stats.csv" | while read f; do echo "== $f"; head -6 "$f" | cut -c1-200; done
