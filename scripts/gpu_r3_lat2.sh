#!/bin/bash
# Latency GEMM variants (incl. workgroup fold) bit-exact, then b1 bench + trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out/p10
O=gpurun_out/p10
export RTEN_NUM_THREADS=8
PYT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_conv_lat_gpu.py tests/test_model_gpu.py -k "lat or chain or fc or resnet50" > $O/lat_tests.log 2>&1 \
  || { echo "lat tests failed"; tail -40 $O/lat_tests.log; exit 1; }
tail -3 $O/lat_tests.log
timeout -k 10 200 python -u bench.py --batch 1 --steps 50 --no-cpu-baseline --timing-report > $O/b1.json 2> $O/b1.err || { tail $O/b1.err; exit 1; }
cat $O/b1.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b1 -o run --output-format csv \
  -- python3 bench.py --batch 1 --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_b1.log 2>&1 \
  || { echo "rocprof failed"; tail $O/prof_b1.log; exit 1; }
f=$(find $O/prof_b1 -name 'run_kernel_trace.csv' | head -n 1)
python3 rten-fork_amd/tools/rocprof_per_forward.py "$f" 10 4 --seq > $O/b1_seq.txt && head -12 $O/b1_seq.txt
