#!/bin/bash
# Per-op timing report + rocprofv3 kernel-trace stats of the benchmark.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --timing-report --no-cpu-baseline > gpurun_out/bench_t.log 2> gpurun_out/bench_t.err
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench_t.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc" >> gpurun_out/prof.log
exit $rc
