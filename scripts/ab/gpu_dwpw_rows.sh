#!/bin/bash
# dw_project.hip: 4 vs 8 output rows per workgroup (RTENHIP_DP_ROWS), and the
# unfused pair, standalone at MobileNetV2 b128.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/dwpwrows_${1:-now}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_pointwise_gpu.py -k "dw_project" > $O/tests4.log 2>&1 || { echo "tests failed"; tail -30 $O/tests4.log; exit 1; }
RTENHIP_DP_ROWS=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_pointwise_gpu.py -k "dw_project" > $O/tests8.log 2>&1 || { echo "tests8 failed"; tail -30 $O/tests8.log; exit 1; }
tail -1 $O/tests4.log $O/tests8.log
T=rten-fork_amd/tools/dwpw_bench.py
for i in 1 2; do
  for v in 4 8; do echo -n "rows$v " >> $O/t.txt; RTENHIP_DP_ROWS=$v timeout -k 10 120 python -u $T 128 50 2>/dev/null >> $O/t.txt || exit 1; done
  echo -n "unfused " >> $O/t.txt; RTENHIP_DW_PROJECT=0 timeout -k 10 120 python -u $T 128 50 2>/dev/null >> $O/t.txt || exit 1
done
cat $O/t.txt
