#!/bin/bash
# Batch-1 latency path: latency-GEMM and whole-model tests, then the b1 bench
# (A/B against an env-selected variant when given) and its timing report.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/b1; mkdir -p $O
export RTEN_NUM_THREADS=8
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 500 $PYT tests/test_conv_lat_gpu.py tests/test_full_size_gpu.py -k "lat or chain or batch1" > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
timeout -k 10 200 python -u bench.py --batch 1 --steps 200 --warmup 20 --no-cpu-baseline > $O/b1_$i.json 2> $O/b1.err || { tail $O/b1.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b1_$i.json'));print('b1', d['value'], d['ms_per_step'])"
done
timeout -k 10 200 python -u bench.py --batch 1 --steps 50 --no-cpu-baseline --timing-report > /dev/null 2> $O/b1_report.txt || exit 1
head -70 $O/b1_report.txt
