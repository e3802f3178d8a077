#!/bin/bash
# Fused depthwise -> project: parity, then MobileNetV2 b128 with the fusion on
# and off (interleaved), timing reports kept.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/dwpw; mkdir -p $O
export RTEN_NUM_THREADS=8
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_pointwise_gpu.py \
  -k "depthwise_pointwise" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in on off; do
    if [ $v = on ]; then export RTENHIP_DWPW=1; else unset RTENHIP_DWPW; fi
    timeout -k 10 240 python -u bench.py --model mobilenet_v2 --batch 128 --no-cpu-baseline --timing-report > $O/mnv2_${v}_$i.json 2> $O/mnv2_${v}_$i.txt || { tail $O/mnv2_${v}_$i.txt; exit 1; }
    python3 -c "import json;d=json.load(open('$O/mnv2_${v}_$i.json'));print('mnv2 $v', d['value'], d['ms_per_step'])"
  done
done
unset RTENHIP_DWPW
grep -E "Conv\(dw\+pw\)|features.(1|3|5|6)\.(dw|project) " $O/mnv2_on_1.txt $O/mnv2_off_1.txt
