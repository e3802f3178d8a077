#!/bin/bash
# Stem kernel's small-batch variant (one output row per band, 2 items per
# wave): parity, standalone b1 stem, and ResNet-50 b1 with / without the stem
# candidate (RTENHIP_STEM=0), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/stemb1_${1:-now}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_pointwise_gpu.py -k "stem" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
T=rten-fork_amd/tools/stem_bench.py
for v in 800 0; do
  if [ $v = 800 ]; then E="RTENHIP_PW_VALU=800"; else E="RTENHIP_STEM=0"; fi
  echo -n "$E " >> $O/t.txt; env $E timeout -k 10 120 python -u $T resnet50 1 200 2>/dev/null >> $O/t.txt || exit 1
done
cat $O/t.txt
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --batch 1 --steps 300 --warmup 30 --no-secondary --no-cpu-baseline \
    > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -3 $O/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$tag.json $tag
}
for i in 1 2; do run off$i RTENHIP_STEM=0; run on$i RTENHIP_STEM=1; done
