#!/bin/bash
# Batch-1 conv1 + downsample pair launches (gemm_lat2_pair_kernel): parity,
# the tuner's pair decisions, b1 bench interleaved with RTENHIP_LAT_PAIR=0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/latpair_${1:-now}; mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_full_size_gpu.py tests/test_model_gpu.py -k "batch1 or b1 or forced" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
RTENHIP_LAT_PAIR_DEBUG=1 timeout -k 10 300 python -u rten-fork_amd/tools/model_once.py 1 resnet50 1 --report > $O/report.txt 2>&1 || { echo "report failed"; tail -5 $O/report.txt; exit 1; }
grep "lat pair\|^Graph run\|Conv(" $O/report.txt | head -20
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --batch 1 --steps 200 --warmup 20 --no-secondary --no-cpu-baseline \
    > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -3 $O/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$tag.json $tag
}
for i in 1 2; do run off$i RTENHIP_LAT_PAIR=0; run on$i RTENHIP_LAT_PAIR=1; done
