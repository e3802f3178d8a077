#!/bin/bash
# dw_project.hip: one or two MFMA k-steps per staged step / barrier
# (RTENHIP_DP_KPB), parity and standalone features.1 timing at b128.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/dwpwkpb_${1:-now}; mkdir -p $O
for v in 1 2; do
  RTENHIP_DP_KPB=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_pointwise_gpu.py -k "dw_project" > $O/tests$v.log 2>&1 || { echo "tests $v failed"; tail -30 $O/tests$v.log; exit 1; }
  tail -n 1 $O/tests$v.log
done
T=rten-fork_amd/tools/dwpw_bench.py
for i in 1 2; do
  for v in 1 2; do echo -n "kpb$v " >> $O/t.txt; RTENHIP_DP_KPB=$v timeout -k 10 120 python -u $T 128 50 2>/dev/null >> $O/t.txt || exit 1; done
done
cat $O/t.txt
