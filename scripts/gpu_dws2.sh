#!/bin/bash
# Streaming depthwise standalone: event times and rocprof kernel stats, both kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/dws2_${1:-now}; mkdir -p $O
for v in 0 1; do
  echo "== RTENHIP_DW_STREAM=$v"
  RTENHIP_DW_STREAM=$v timeout -k 10 120 python -u rten-fork_amd/tools/dws_bench.py || exit 1
done
RTENHIP_DW_STREAM=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof1 -o run -- python3 rten-fork_amd/tools/dws_bench.py > $O/prof1.log 2>&1 || { echo "rocprof failed"; tail $O/prof1.log; exit 1; }
f=$(find $O/prof1 -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -8
