#!/bin/bash
# stem_dw_project_kernel part timings (RTENHIP_SD_DBG: 1 = no stem steps, 2 = no
# depthwise steps, 3 = neither) from MobileNetV2 b128 per-op reports.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/sddbg_${1:-now}; mkdir -p $O
for v in ${DBGS:-0 1 2 3 0}; do
  RTENHIP_SD_DBG=$v timeout -k 10 300 python -u rten-fork_amd/tools/model_once.py 1 mobilenet_v2 128 --report > $O/r$v.txt 2>&1 || { echo "report $v failed"; tail -5 $O/r$v.txt; exit 1; }
  echo "dbg=$v $(grep 'op features.1.project' $O/r$v.txt)"
done
