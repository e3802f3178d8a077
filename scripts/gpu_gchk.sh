#!/bin/bash
# Gather check ring: gather / BERT / host-run tests, BERT b32 bench lines, BERT per-forward summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/gchk_${1:-now}; mkdir -p $O
timeout -k 10 500 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_model_gpu.py tests/test_host_run_gpu.py tests/test_full_size_gpu.py -k "gather or Gather or bert or host" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; grep -E "^FAILED" $O/tests.log | head; [ $rc -eq 0 ] || { echo "tests failed"; exit 1; }
for r in 1 2; do
timeout -k 10 300 python -u bench.py --model bert --batch 32 --no-cpu-baseline --no-secondary --steps 30 --warmup 5 > $O/bert_$r.json 2> $O/bert_$r.err || { echo "bench failed"; tail -5 $O/bert_$r.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bert', d['value'], d['ms_per_step'])" $O/bert_$r.json
done
bash scripts/gpu_prof.sh gchk_${1:-now} bert_b32
