#!/bin/bash
# Chain timing experiments: sc1 hand-off loads / stores vs plain (timing only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out/p6
O=gpurun_out/p6
export RTEN_NUM_THREADS=8
for dbg in 0; do
  RTENHIP_CHAIN_DBG=$dbg RTENHIP_CHAIN=1 timeout -k 10 200 python -u bench.py --batch 1 --steps 20 --no-cpu-baseline --timing-report > $O/b1_$dbg.json 2> $O/b1_$dbg.err || { tail $O/b1_$dbg.err; exit 1; }
  echo "dbg $dbg"; grep "conv chain" $O/b1_$dbg.err
done
