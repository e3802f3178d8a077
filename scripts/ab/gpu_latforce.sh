#!/bin/bash
# One batch-1 conv per latency-GEMM variant (RTENHIP_LAT forced): kernel time
# (rocprofv3, tools/l2_hot_cold.py's cold phase) per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/latforce_${1:-now}; mkdir -p $O
for shp in "256 14 256 3" "512 7 512 3" "128 28 128 3"; do
  set -- $shp
  for v in 72 74 71 86 61 62 63 66 11 41; do
    tag=c$1h$2o$3k$4_v$v
    RTENHIP_LAT=$v timeout -k 10 120 rocprofv3 --kernel-trace -d $O/$tag -o run --output-format csv -- python3 rten-fork_amd/tools/l2_hot_cold.py $shp 30 > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
    f=$(find $O/$tag -name 'run_kernel_trace.csv' | head -n 1)
    echo -n "$tag  "; python3 rten-fork_amd/tools/l2_hot_cold_summary.py "$f" || exit 1
    rm -rf $O/$tag
  done
done
