#!/bin/bash
# Direct conv with LDS-staged input rows (MobileNetV2 stem): parity, then
# MobileNetV2 b128 bench + timing report (the tuner picks per layer).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/stem; mkdir -p $O
export RTEN_NUM_THREADS=8
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_conv_pointwise_gpu.py -k "direct or misaligned" > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --model mobilenet_v2 --batch 128 --no-cpu-baseline --timing-report > $O/mnv2_$i.json 2> $O/mnv2_$i.txt || { tail $O/mnv2_$i.txt; exit 1; }
  python3 -c "import json;d=json.load(open('$O/mnv2_$i.json'));print('mnv2', d['value'], d['ms_per_step'])"
  RTENHIP_PW_VALU=332 timeout -k 10 240 python -u bench.py --model mobilenet_v2 --batch 128 --no-cpu-baseline > $O/mnv2_332_$i.json 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('$O/mnv2_332_$i.json'));print('mnv2 forced332', d['value'], d['ms_per_step'])"
done
grep -E "features.0 " $O/mnv2_*.txt
