#!/bin/bash
# Host-resident input staging: its GPU tests, then the full bench line twice
# (the host-input secondary runs after the other configs, in one process) and
# the --host-input headline alone.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/hostin_${1:-now}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_staging_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench_$r.json 2> $O/bench_$r.err || { echo "bench failed"; tail $O/bench_$r.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('head', d['value'], d['ms_per_step'])
for s in d['secondary']:
    if 'host' in s.get('metric', ''): print('  host', s['value'], s['ms_per_step'], s['vs_device_resident'], s.get('error', ''))" $O/bench_$r.json
done
timeout -k 10 300 python -u bench.py --host-input --no-secondary --no-cpu-baseline > $O/alone.json 2> $O/alone.err || { echo "alone failed"; tail $O/alone.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('alone', d['value'], d['ms_per_step'])" $O/alone.json
