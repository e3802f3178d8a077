#!/bin/bash
# BERT b32 dispatch sequence of one forward (which launch follows each pack_a).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/bertseq; mkdir -p $O
export RTEN_NUM_THREADS=8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --model bert --batch 32 --steps 10 --warmup 3 --no-cpu-baseline --timing-report > $O/prof.log 2>&1 || { echo "rocprof failed"; tail $O/prof.log; exit 1; }
f=$(find $O/prof -name 'run_kernel_trace.csv' | head -n 1)
python3 rten-fork_amd/tools/rocprof_per_forward.py "$f" 10 4 --seq > $O/seq.txt || exit 1
rm -rf $O/prof
grep -c "pack_a" $O/seq.txt || echo "no pack_a in the step"
