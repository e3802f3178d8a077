#!/bin/bash
# LayerNorm rows kernel: parity tests, rocprof of tools/ln_bench.py, BERT b32
# bench lines and the BERT per-forward kernel summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/ln_${1:-now}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_ops_gpu.py tests/test_model_gpu.py tests/test_full_size_gpu.py -k "layer_norm or LayerNorm or bert" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; grep -E "^FAILED" $O/tests.log | head; [ $rc -eq 0 ] || { echo "tests failed"; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 rten-fork_amd/tools/ln_bench.py > $O/p.log 2>&1 || { echo "rocprof fail"; tail -5 $O/p.log; exit 1; }
f=$(find $O/p -name "run_kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "layer_norm" in r["Name"]:
        print(r["Name"][:40], "calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1000, 2))
PY
for r in 1 2; do
timeout -k 10 300 python -u bench.py --model bert --batch 32 --no-cpu-baseline --no-secondary --steps 30 --warmup 5 > $O/bert_$r.json 2> $O/bert_$r.err || { echo "bench failed"; tail -5 $O/bert_$r.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bert', d['value'], d['ms_per_step'])" $O/bert_$r.json
done
bash scripts/gpu_prof.sh ln_${1:-now} bert_b32
