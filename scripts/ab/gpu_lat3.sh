#!/bin/bash
# Pipelined LDS-staged latency GEMM (gemm_lat3_kernel, variants 8x): parity
# (every latency variant on the conv cases and on ResNet-50 b1), then the b1
# bench with the 8x variants offered to the tuner or not (RTENHIP_LAT3=0),
# interleaved, each 8x variant forced, and the stamp anatomy.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/lat3_${1:-now}; mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_conv_lat_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
b1() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --batch 1 --steps 300 --warmup 30 --no-secondary --no-cpu-baseline \
    > $O/b1_$tag.json 2> $O/b1_$tag.err || { echo "bench $tag failed"; tail -3 $O/b1_$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/b1_$tag.json $tag
}
b1 off1 RTENHIP_LAT3=0
b1 on1 RTENHIP_LAT3=1
b1 off2 RTENHIP_LAT3=0
b1 on2 RTENHIP_LAT3=1
for v in 81 82 84 85 86 88; do b1 f$v RTENHIP_LAT=$v; done
timeout -k 10 300 python3 rten-fork_amd/tools/lat_stamps.py > $O/stamps.txt 2>&1 || { echo "stamps failed"; tail $O/stamps.txt; exit 1; }
grep -E "^ +[0-9]+ |^op " $O/stamps.txt | head -120
