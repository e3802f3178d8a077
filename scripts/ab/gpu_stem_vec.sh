#!/bin/bash
# Stem kernel with the MFMA operands swapped (pixels as rows: 16-byte stores):
# parity tests, then per-replay stem time (compare profiles/r5_stem_mfma.txt).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/stemvec_${1:-now}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_pointwise_gpu.py -k stem > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
T=rten-fork_amd/tools/stem_bench.py
for i in 1 2; do
  for b in 64 1; do
    echo -n "forced " >> $O/t.txt; RTENHIP_PW_VALU=800 timeout -k 10 120 python -u $T resnet50 $b 30 2>/dev/null >> $O/t.txt || exit 1
  done
  echo -n "forced " >> $O/t.txt; RTENHIP_PW_VALU=800 timeout -k 10 120 python -u $T mobilenet_v2 128 30 2>/dev/null >> $O/t.txt || exit 1
done
cat $O/t.txt
