#!/bin/bash
# Conv chain bring-up: lat + chain tests, then the b1 bench with its timing
# report and a kernel trace of the steady state.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out/p4
O=gpurun_out/p4
export RTEN_NUM_THREADS=8
PYT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_conv_lat_gpu.py -k "chain" > $O/chain_tests.log 2>&1 \
  || { echo "chain tests failed"; tail -40 $O/chain_tests.log; exit 1; }
tail -3 $O/chain_tests.log
timeout -k 10 300 python -u bench.py --batch 1 --steps 50 --no-cpu-baseline --timing-report > $O/bench_b1.json 2> $O/bench_b1.err || { tail $O/bench_b1.err; exit 1; }
cat $O/bench_b1.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b1 -o run --output-format csv \
  -- python3 bench.py --batch 1 --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_b1.log 2>&1 \
  || { echo "rocprof failed"; tail $O/prof_b1.log; exit 1; }
f=$(find $O/prof_b1 -name 'run_kernel_trace.csv' | head -n 1)
python3 rten-fork_amd/tools/rocprof_per_forward.py "$f" 10 4 --seq > $O/b1_seq.txt && cat $O/b1_seq.txt
