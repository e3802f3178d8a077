#!/bin/bash
# Slab latency GEMM (gemm_lat4_kernel, variants 6x): parity on every latency
# variant, then ResNet-50 b1 with the 6x variants offered to the tuner or not
# (RTENHIP_LAT_SLAB=0), interleaved, and the per-op report.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/slab_${1:-now}; mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_conv_lat_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
b1() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --batch 1 --steps 300 --warmup 30 --no-secondary --no-cpu-baseline \
    > $O/b1_$tag.json 2> $O/b1_$tag.err || { echo "bench $tag failed"; tail -3 $O/b1_$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/b1_$tag.json $tag
}
b1 off1 RTENHIP_LAT_SLAB=0
b1 on1 RTENHIP_LAT_SLAB=1
b1 off2 RTENHIP_LAT_SLAB=0
b1 on2 RTENHIP_LAT_SLAB=1
timeout -k 10 300 python -u rten-fork_amd/tools/model_once.py 1 resnet50 1 --report > $O/report_b1.txt 2>&1 || { echo "report failed"; tail -5 $O/report_b1.txt; exit 1; }
grep "^op " $O/report_b1.txt | grep "layer3\|layer4"
