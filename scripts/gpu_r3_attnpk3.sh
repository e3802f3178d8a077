#!/bin/bash
# Attention packed-A only (no row-major copy): parity, then an interleaved
# BERT b32 A/B against RTENHIP_ATTN_PK=0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/attnpk3; mkdir -p $O
export RTEN_NUM_THREADS=8
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py tests/test_ops_gpu.py tests/test_rten_file.py tests/test_optimizer_gpu.py \
  -k "attention or bert or grouped or matmul" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_full_size_gpu.py -k bert > $O/full.log 2>&1 || { tail -30 $O/full.log; exit 1; }
tail -1 $O/full.log
for i in 1 2; do
  for v in on off; do
    if [ $v = off ]; then export RTENHIP_ATTN_PK=0; else unset RTENHIP_ATTN_PK; fi
    timeout -k 10 240 python -u bench.py --model bert --batch 32 --no-cpu-baseline > $O/bert_${v}_$i.json 2> $O/bert_${v}_$i.err || { tail $O/bert_${v}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bert_${v}_$i.json'));print('bert $v', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
