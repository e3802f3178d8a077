#!/bin/bash
# Attention storing the output projection's packed A: parity (attention / BERT
# tests, BERT b32 full size), then BERT b32 bench + per-forward kernel counts.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/attnpk; mkdir -p $O
export RTEN_NUM_THREADS=8
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py tests/test_ops_gpu.py \
  -k "attention or bert or grouped or matmul" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_full_size_gpu.py -k bert > $O/full.log 2>&1 || { tail -30 $O/full.log; exit 1; }
tail -1 $O/full.log
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --model bert --batch 32 --no-cpu-baseline --timing-report > $O/bert_$i.json 2> $O/bert_$i.txt || { tail $O/bert_$i.txt; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bert_$i.json'));print('bert', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --model bert --batch 32 --steps 10 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "rocprof failed"; tail $O/prof.log; exit 1; }
f=$(find $O/prof -name 'run_kernel_stats.csv' | head -n 1)
cp "$f" $O/bert_kernel_stats.csv
rm -rf $O/prof
head -12 $O/bert_kernel_stats.csv
