#!/bin/bash
# Batch-1 iteration: latency-GEMM parity tests, the stamp timeline of the
# batch-1 forward, and the b1 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/b1_${1:-now}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_lat_gpu.py ${PYTEST_K:+-k "$PYTEST_K"} > $O/lat_tests.log 2>&1 || { echo "lat tests failed"; tail -30 $O/lat_tests.log; exit 1; }
tail -1 $O/lat_tests.log
timeout -k 10 200 python -u rten-fork_amd/tools/lat_stamps.py > $O/stamps.txt 2>&1 || { echo "stamps failed"; tail -20 $O/stamps.txt; exit 1; }
head -20 $O/stamps.txt
timeout -k 10 300 python -u bench.py --batch 1 --steps 200 --warmup 20 --no-cpu-baseline --timing-report > $O/b1.json 2> $O/b1.err || { echo "bench failed"; tail -20 $O/b1.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b1.json'));print('b1', d['value'], d['ms_per_step'])"
