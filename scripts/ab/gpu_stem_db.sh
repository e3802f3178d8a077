#!/bin/bash
# Stem kernel: the 8-wave, DMA double-buffered variant vs the 4-wave one
# (RTENHIP_STEM_DB=0): parity tests, then per-replay stem time.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/stemdb_${1:-now}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_pointwise_gpu.py -k stem > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
T=rten-fork_amd/tools/stem_bench.py
for i in 1 2; do
  for db in 1 0; do
    echo -n "db$db " >> $O/t.txt; RTENHIP_STEM_DB=$db RTENHIP_PW_VALU=800 timeout -k 10 120 python -u $T resnet50 64 30 2>/dev/null >> $O/t.txt || exit 1
    echo -n "db$db " >> $O/t.txt; RTENHIP_STEM_DB=$db RTENHIP_PW_VALU=800 timeout -k 10 120 python -u $T mobilenet_v2 128 30 2>/dev/null >> $O/t.txt || exit 1
  done
done
echo -n "tuned " >> $O/t.txt; timeout -k 10 120 python -u $T mobilenet_v2 128 30 2>/dev/null >> $O/t.txt || exit 1
cat $O/t.txt
