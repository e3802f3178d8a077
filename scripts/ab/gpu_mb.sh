#!/bin/bash
# Fused inverted residual block check: its parity tests, MobileNetV2 b128 A/B
# (RTENHIP_MBCONV=0 runs the convs apart) with the per-op timing report, the
# batch-1 forced-variant tests and the world-2 ResNet-50 test.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/mb_${1:-now}; mkdir -p $O
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $PYT -x tests/test_mbconv_block_gpu.py > $O/mb.log 2>&1; rc=$?
tail -2 $O/mb.log; [ $rc -le 1 ] || { echo "aborted rc=$rc"; exit 1; }
for v in 1 0; do
  RTENHIP_MBCONV=$v timeout -k 10 300 python -u bench.py --model mobilenet_v2 --batch 128 --no-secondary --no-cpu-baseline > $O/mnv2_$v.json 2> $O/mnv2_$v.err \
    || { echo "bench failed"; tail $O/mnv2_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('mnv2 MBCONV=' + sys.argv[2], d['value'], d['ms_per_step'])" $O/mnv2_$v.json $v
done
RTENHIP_MBCONV=1 timeout -k 10 300 python -u rten-fork_amd/tools/model_once.py 2 mobilenet_v2 128 --report > $O/report.txt 2>&1 || echo "report failed"
head -40 $O/report.txt
timeout -k 10 600 $PYT tests/test_conv_lat_gpu.py -k forced_variant tests/test_parallel_gpu.py > $O/lat.log 2>&1; tail -3 $O/lat.log; grep -E "^FAILED|differ in" $O/lat.log | head
