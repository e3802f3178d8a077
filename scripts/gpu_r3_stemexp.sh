#!/bin/bash
# MobileNetV2 stem (features.0) A/B: the conv's time under each forced kernel
# (eager timing report of a MobileNetV2 b128 run), and the LDS-row kernel with
# its stores skipped (experiment build; results invalid, timing only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/stemexp; mkdir -p $O
export RTEN_NUM_THREADS=8
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --model mobilenet_v2 --batch 128 --steps 5 --warmup 2 --no-cpu-baseline --timing-report > $O/$n.json 2> $O/$n.txt || { tail $O/$n.txt; exit 1; }
  echo "$n $(grep -E 'op features.0 ' $O/$n.txt)"
}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_pointwise_gpu.py -k "direct or misaligned" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run dma RTENHIP_PW_VALU=0
run v332 RTENHIP_PW_VALU=332
run v416 RTENHIP_PW_VALU=416
run v432 RTENHIP_PW_VALU=432
run v416_nostore RTENHIP_PW_VALU=416 RTENHIP_LIB=rten-fork_amd/stemexp/librten_hip.so
run v432_nostore RTENHIP_PW_VALU=432 RTENHIP_LIB=rten-fork_amd/stemexp/librten_hip.so
