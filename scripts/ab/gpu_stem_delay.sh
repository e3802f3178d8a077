#!/bin/bash
# Stem kernel: de-phase the CU's two workgroups by delaying the second half of
# the persistent grid (RTENHIP_STEM_DELAY rounds of s_sleep 127, ~8K cycles each).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/stemdelay_${1:-now}; mkdir -p $O
T=rten-fork_amd/tools/stem_bench.py
for i in 1 2; do
  for dl in 0 3 6 12; do echo -n "delay$dl " >> $O/t.txt; RTENHIP_STEM_DELAY=$dl RTENHIP_PW_VALU=800 timeout -k 10 120 python -u $T resnet50 64 30 2>/dev/null >> $O/t.txt || exit 1; done
done
cat $O/t.txt
