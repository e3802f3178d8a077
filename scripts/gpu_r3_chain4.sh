#!/bin/bash
# Chain timeline: per-unit timestamps of the forced chain at batch 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out/p7
O=gpurun_out/p7
export RTEN_NUM_THREADS=8
RTENHIP_CHAIN=1 RTENHIP_CHAIN_STAMPS=$O/st timeout -k 10 200 python -u bench.py --batch 1 --steps 3 --warmup 2 --no-cpu-baseline --timing-report > $O/b1.json 2> $O/b1.err || { tail $O/b1.err; exit 1; }
grep "conv chain" $O/b1.err
for c in 0 1 2 3; do python3 rten-fork_amd/tools/chain_stamps.py $O/st.$c; done
