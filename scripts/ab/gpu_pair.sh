#!/bin/bash
# conv3 -> conv1 pairs (csrc/conv_pair.hip): parity (unit cases + ResNet-50
# b64 full size), then ResNet-50 b64 with and without (RTENHIP_CONV_PAIR=0),
# interleaved, and the per-op report.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/pair_${1:-now}; mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_conv_pair_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 600 $PYT tests/test_model_gpu.py -k "batch64" > $O/tests64.log 2>&1 || { echo "b64 tests failed"; tail -40 $O/tests64.log; exit 1; }
tail -n 1 $O/tests64.log
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --batch 64 --steps 60 --warmup 10 --no-secondary --no-cpu-baseline \
    > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -3 $O/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$tag.json $tag
}
for i in 1 2 3; do run off$i RTENHIP_CONV_PAIR=0; run on$i RTENHIP_CONV_PAIR=1; done
for v in 0 1; do
  RTENHIP_CONV_PAIR=$v timeout -k 10 300 python -u rten-fork_amd/tools/model_once.py 1 resnet50 64 --report > $O/report_$v.txt 2>&1 || { echo "report failed"; tail -5 $O/report_$v.txt; exit 1; }
  grep "conv3+conv1\|layer1.[12].conv[13] \|layer2.0.conv1 " $O/report_$v.txt | head -8
done
