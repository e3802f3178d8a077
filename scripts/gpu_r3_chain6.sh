#!/bin/bash
# Chain timing experiment: hand-off loads / stores sc1 (0) vs plain (3, timing only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out/p9
O=gpurun_out/p9
export RTEN_NUM_THREADS=8
for dbg in 0 3 1; do
  RTENHIP_CHAIN_DBG=$dbg RTENHIP_CHAIN=1 RTENHIP_CHAIN_STAMPS=$O/st$dbg timeout -k 10 200 python -u bench.py --batch 1 --steps 3 --warmup 2 --no-cpu-baseline --timing-report > $O/b$dbg.json 2> $O/b$dbg.err || { tail $O/b$dbg.err; exit 1; }
  echo "dbg $dbg"; grep "conv chain" $O/b$dbg.err; python3 rten-fork_amd/tools/chain_stamps.py $O/st$dbg.0 > $O/tl$dbg.txt; head -1 $O/tl$dbg.txt
done
