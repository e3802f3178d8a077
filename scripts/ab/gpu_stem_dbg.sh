#!/bin/bash
# Stem kernel timing experiments (RTENHIP_STEM_DBG bits: 1 no stores, 2 no
# band loads, 4 no MFMA; wrong results) vs the tuner without the stem.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=$PWD/gpurun_out/stemdbg_${1:-now}; mkdir -p $O
T=rten-fork_amd/tools/stem_bench.py
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_pointwise_gpu.py -k "stem_mfma_bitexact" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for mdl in "resnet50 64" "mobilenet_v2 128"; do
  for dbg in ${DBGS:-0 1 2 3 4 5 6}; do
    echo -n "dbg$dbg " >> $O/times.txt
    RTENHIP_STEM_DBG=$dbg RTENHIP_PW_VALU=800 timeout -k 10 120 python -u $T $mdl 50 2>/dev/null >> $O/times.txt || { tail -5 $O/times.txt; exit 1; }
  done
  echo -n "tuned-no-stem " >> $O/times.txt
  RTENHIP_STEM=0 timeout -k 10 120 python -u $T $mdl 50 2>/dev/null >> $O/times.txt || { tail -5 $O/times.txt; exit 1; }
done
cat $O/times.txt
