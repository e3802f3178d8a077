#!/bin/bash
# One GPU session: smoke, default bench line, rocprofv3 kernel stats of the
# bench, PMC HBM traffic.  Every GPU step has its own time limit; the script
# stops at the first failure.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { echo bench failed; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo rocprof failed; exit 1; }
bash scripts/gpu_traffic.sh || { echo traffic failed; exit 1; }
echo round-ok
