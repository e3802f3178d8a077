#!/bin/bash
# Stem MFMA kernel (csrc/conv_stem.hip): parity, standalone stem timings,
# then ResNet-50 b64 / b1 and MobileNetV2 b128 with the stem candidate offered
# to the tuner or not (RTENHIP_STEM=0), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/stem_${1:-now}; mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_conv_pointwise_gpu.py -k "stem" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
T=rten-fork_amd/tools/stem_bench.py
for mdl in "resnet50 64" "mobilenet_v2 128" "resnet50 1"; do
  echo -n "forced-stem " >> $O/stem.txt
  RTENHIP_PW_VALU=800 timeout -k 10 120 python -u $T $mdl 50 2>/dev/null >> $O/stem.txt || { tail -5 $O/stem.txt; exit 1; }
  echo -n "tuned-no-stem " >> $O/stem.txt
  RTENHIP_STEM=0 timeout -k 10 120 python -u $T $mdl 50 2>/dev/null >> $O/stem.txt || { tail -5 $O/stem.txt; exit 1; }
  echo -n "tuned " >> $O/stem.txt
  timeout -k 10 120 python -u $T $mdl 50 2>/dev/null >> $O/stem.txt || { tail -5 $O/stem.txt; exit 1; }
done
cat $O/stem.txt
run() {  # tag model batch steps env...
  local tag=$1 model=$2 batch=$3 steps=$4; shift 4
  env "$@" timeout -k 10 300 python -u bench.py --model $model --batch $batch --steps $steps --warmup 10 --no-secondary --no-cpu-baseline \
    > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -3 $O/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$tag.json $tag
}
run r_off1 resnet50 64 40 RTENHIP_STEM=0
run r_on1 resnet50 64 40 RTENHIP_STEM=1
run r_off2 resnet50 64 40 RTENHIP_STEM=0
run r_on2 resnet50 64 40 RTENHIP_STEM=1
run m_off1 mobilenet_v2 128 60 RTENHIP_STEM=0
run m_on1 mobilenet_v2 128 60 RTENHIP_STEM=1
run b1_off resnet50 1 300 RTENHIP_STEM=0
run b1_on resnet50 1 300 RTENHIP_STEM=1
