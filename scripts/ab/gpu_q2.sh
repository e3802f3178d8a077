#!/bin/bash
# Quick measurements after the pointwise revert and the LayerNorm row padding:
# the LayerNorm / pointwise parity tests, the LayerNorm launch timing, and the
# MobileNetV2 / BERT bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/q2_${1:-now}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k "layer_norm" tests/test_conv_pointwise_gpu.py tests/test_model_gpu.py -k "layer_norm or bert or pointwise or mobilenet" > $O/t.log 2>&1; rc=$?
tail -2 $O/t.log; grep -E "^FAILED" $O/t.log | head; [ $rc -le 1 ] || exit 1
LN_EXPS=" " LN_ROWS_SWEEP="${LN_ROWS_SWEEP:-4 2}" bash scripts/ab/gpu_ln.sh || exit 1
for m in "mobilenet_v2 128" "bert 32"; do
  set -- $m
  timeout -k 10 300 python -u bench.py --model $1 --batch $2 --no-secondary --no-cpu-baseline > $O/$1.json 2> $O/$1.err || { echo "bench $1 failed"; tail $O/$1.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$1.json $1
done
