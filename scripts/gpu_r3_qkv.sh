#!/bin/bash
# Grouped Q/K/V GEMM: parity (new test, BERT model tests, BERT b32 full size),
# then BERT b32 with grouping on / off (interleaved).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/qkv; mkdir -p $O
export RTEN_NUM_THREADS=8
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py \
  -k "grouped or bert or matmul" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_full_size_gpu.py -k bert > $O/full.log 2>&1 || { tail -30 $O/full.log; exit 1; }
tail -1 $O/full.log
for i in 1 2; do
  for v in on off; do
    if [ $v = off ]; then export RTENHIP_MM_GROUP=0; else unset RTENHIP_MM_GROUP; fi
    timeout -k 10 240 python -u bench.py --model bert --batch 32 --no-cpu-baseline --timing-report > $O/bert_${v}_$i.json 2> $O/bert_${v}_$i.txt || { tail $O/bert_${v}_$i.txt; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bert_${v}_$i.json'));print('bert $v', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
unset RTENHIP_MM_GROUP
grep -E "op layer0\.(q|k|v)\.matmul" $O/bert_on_1.txt $O/bert_off_1.txt
