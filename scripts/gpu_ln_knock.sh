#!/bin/bash
# LayerNorm phase knockout: per-launch time without the serial folds
# (ab_nochain, wrong values, timing only) vs the in-tree build, plus a
# device copy of the same bytes.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/lnk; mkdir -p $O
for v in nochain new; do
  lib=""; [ $v = nochain ] && lib=$PWD/rten-fork_amd/ab_nochain/librten_hip.so
  RTENHIP_LIB=$lib LN_COPY=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 rten-fork_amd/tools/ln_bench.py > $O/$v.log 2>&1 || { echo rocprof $v failed; tail $O/$v.log; exit 1; }
  echo "== $v"; find $O/$v -name "*kernel_stats.csv" -exec cat {} + | cut -c1-60,150-
done
