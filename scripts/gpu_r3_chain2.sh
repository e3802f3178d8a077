#!/bin/bash
# Chain timing: b1 bench with the chain forced and in auto mode (timing
# reports name the chain's build-time comparison).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out/p5
O=gpurun_out/p5
export RTEN_NUM_THREADS=8
timeout -k 10 300 python -u bench.py --batch 1 --steps 50 --no-cpu-baseline --timing-report > $O/bench_b1.json 2> $O/bench_b1.err || { tail $O/bench_b1.err; exit 1; }
cat $O/bench_b1.json; grep "conv chain" $O/bench_b1.err
RTENHIP_CHAIN=1 timeout -k 10 300 python -u bench.py --batch 1 --steps 50 --no-cpu-baseline --timing-report > $O/bench_b1_forced.json 2> $O/bench_b1_forced.err || { tail $O/bench_b1_forced.err; exit 1; }
cat $O/bench_b1_forced.json; grep "conv chain\|ConvChain" $O/bench_b1_forced.err
