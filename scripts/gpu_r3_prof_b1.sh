#!/bin/bash
# ResNet-50 batch-1 kernel trace: per-forward dispatch sequence (durations and
# gaps) of the steady state.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out/p3
O=gpurun_out/p3
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_b1 -o run --output-format csv \
  -- python3 bench.py --batch 1 --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_b1.log 2>&1 \
  || { echo "rocprof failed"; tail $O/prof_b1.log; exit 1; }
f=$(find $O/prof_b1 -name 'run_kernel_trace.csv' | head -n 1)
python3 rten-fork_amd/tools/rocprof_per_forward.py "$f" 10 4 --seq > $O/b1_seq.txt && cat $O/b1_seq.txt
