#!/bin/bash
# Quick check: attention / BERT parity tests and the attention timing
# experiments, then MobileNetV2 b128's per-op report with the convs apart.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/quick_${1:-now}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_model_gpu.py -k "attention or bert" tests/test_vecmath_gpu.py > $O/att.log 2>&1; rc=$?
tail -2 $O/att.log; grep -E "^FAILED" $O/att.log | head; [ $rc -le 1 ] || { echo "aborted rc=$rc"; exit 1; }
ATT_EXPS="1 2 4" bash scripts/ab/gpu_attn.sh || exit 1
timeout -k 10 300 python -u rten-fork_amd/tools/model_once.py 1 mobilenet_v2 128 --report > $O/mnv2_apart.txt 2>&1 || echo "report failed"
grep -E "^op features\.(1|2|3|4|5|8|12)\." $O/mnv2_apart.txt
