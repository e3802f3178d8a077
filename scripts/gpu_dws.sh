#!/bin/bash
# Streaming depthwise (dw_stream.hip): parity tests, then MobileNetV2 b128
# interleaved A/B against the whole-plane LDS kernel (RTENHIP_DW_STREAM=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/dws_${1:-now}; mkdir -p $O
PYT="python -u -m pytest -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $PYT -x tests/test_ops_gpu.py -k "depthwise or conv_bitexact" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; grep -E "^FAILED|Error" $O/tests.log | head -20
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; exit 1; }
B="python -u bench.py --model mobilenet_v2 --batch 128 --no-cpu-baseline --no-secondary --steps 30 --warmup 5"
for r in 1 2; do
  for v in 0 1; do
    env "RTENHIP_DW_STREAM${DWS_VAR:-}=$v" timeout -k 10 300 $B > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { echo "bench failed"; tail -20 $O/b_${v}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/b_${v}_$r.json "${DWS_VAR:-stream}=$v run$r"
  done
done
