#!/bin/bash
# B-stationary pointwise GEMM (gemm_pwb.hip, latency variants 6x): parity
# tests, then the per-op reports of ResNet-50 b64 / MobileNetV2 b128 (which
# convs the tuner gives it) and the two bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/pwb_${1:-now}; mkdir -p $O
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_pwb_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for cfg in "resnet50 64" "mobilenet_v2 128"; do
  set -- $cfg
  timeout -k 10 300 python -u rten-fork_amd/tools/model_once.py 1 $1 $2 --report > $O/report_$1_b$2.txt 2>&1 || { echo "report $1 $2 failed"; tail -5 $O/report_$1_b$2.txt; exit 1; }
  echo "$1 b$2: $(grep -c 'cfg=lat6' $O/report_$1_b$2.txt) convs on lat6x"
  grep "cfg=lat6" $O/report_$1_b$2.txt | head -40
done
timeout -k 10 300 python -u bench.py --no-secondary --no-cpu-baseline > $O/b64.json 2> $O/b64.err || { echo "bench failed"; tail -5 $O/b64.err; exit 1; }
timeout -k 10 300 python -u bench.py --model mobilenet_v2 --batch 128 --no-secondary --no-cpu-baseline > $O/mnv2.json 2> $O/mnv2.err || { echo "bench mnv2 failed"; tail -5 $O/mnv2.err; exit 1; }
for f in b64 mnv2; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['frac'])" $O/$f.json $f
done
