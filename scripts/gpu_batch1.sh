#!/bin/bash
# ResNet-50 batch 1 (BASELINE.json "batch=1/64"; replicas-only config): bench
# line with per-op timing, rocprofv3 kernel trace + stats and a per-forward
# summary.  Each GPU step has its own time limit; stops at the first failure.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/b1; mkdir -p $O
timeout -k 10 400 python3 bench.py --batch 1 --steps 200 --warmup 20 --no-cpu-baseline --timing-report > $O/bench_b1.json 2> $O/timing_b1.txt || { echo bench failed; tail $O/timing_b1.txt; exit 1; }
cat $O/bench_b1.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --batch 1 --steps 50 --warmup 10 --no-cpu-baseline > $O/prof.log 2>&1 || { echo rocprof failed; tail $O/prof.log; exit 1; }
python3 rten-fork_amd/tools/rocprof_per_forward.py $(find $O/prof -name run_kernel_trace.csv) 10 > $O/per_forward_b1.txt && cat $O/per_forward_b1.txt
