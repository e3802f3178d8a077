#!/bin/bash
# Cross-item prefetch of persistent DMA GEMM launches: parity (forced
# persistent modes included), then interleaved A/B of ResNet-50 b64 and
# MobileNetV2 b128 with RTENHIP_DMA_PF=0 / 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/pf_${1:-now}; mkdir -p $O
PYT="python -u -m pytest -q -x --timeout 300 --timeout-method thread"
if [ -z "$NO_TESTS" ]; then
timeout -k 10 600 $PYT tests/test_model_gpu.py -k "resnet50 or mobilenet or bottleneck or prefetch" tests/test_full_size_gpu.py -k "mobilenet or resnet or persistent or bottleneck" tests/test_ops_gpu.py > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; grep -E "^FAILED|Error" $O/tests.log | head -20
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; exit 1; }
fi
for r in 1 2; do
  for v in 0 1; do
    for m in "resnet50 --batch 64" "mobilenet_v2 --batch 128"; do
      t=$(echo $m | cut -d' ' -f1)
      RTENHIP_DMA_PF=$v timeout -k 10 300 python -u bench.py --model $m --no-cpu-baseline --no-secondary --steps 30 --warmup 5 > $O/${t}_${v}_$r.json 2> $O/${t}_${v}_$r.err || { echo "bench failed"; tail -20 $O/${t}_${v}_$r.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/${t}_${v}_$r.json "$t pf=$v run$r"
    done
  done
done
