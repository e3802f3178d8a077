#!/bin/bash
# End-of-session check of the committed tree: GPU parity suite, smoke, the
# default bench line and the BERT bench line with kernel stats.  Each GPU step
# has its own time limit; stops at the first failure.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo pytest failed; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 python3 bench.py --model bert --batch 32 --no-cpu-baseline --timing-report > $O/bench_bert.json 2> $O/timing_bert.txt || { echo bert failed; tail $O/timing_bert.txt; exit 1; }
cat $O/bench_bert.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_bert -o run --output-format csv -- python3 bench.py --model bert --batch 32 --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_bert.log 2>&1 || { echo rocprof failed; tail $O/prof_bert.log; exit 1; }
python3 rten-fork_amd/tools/rocprof_per_forward.py $(find $O/prof_bert -name run_kernel_trace.csv) 10 156 > $O/per_forward_bert.txt && cat $O/per_forward_bert.txt
