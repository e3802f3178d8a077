#!/bin/bash
# Batch-1 conv kernels with L2-hot vs L2-cold operands (tools/l2_hot_cold.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/l2hot_${1:-now}; mkdir -p $O
for shp in "256 14 256 3" "512 7 512 3" "256 14 1024 1" "1024 14 256 1" "128 28 128 3" "64 56 64 3"; do
  set -- $shp
  tag=c$1h$2o$3k$4
  timeout -k 10 120 rocprofv3 --kernel-trace -d $O/$tag -o run --output-format csv -- python3 rten-fork_amd/tools/l2_hot_cold.py $shp > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  f=$(find $O/$tag -name 'run_kernel_trace.csv' | head -n 1)
  echo -n "$tag  "; python3 rten-fork_amd/tools/l2_hot_cold_summary.py "$f" || exit 1
  rm -rf $O/$tag
done
