#!/bin/bash
# expand -> depthwise with the expand on v_mfma_f32_4x4x1 (RTENHIP_EDW_MX=0: VALU
# expand): parity, MobileNetV2 b128 bench interleaved, replayed per-kernel sums.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/edwmx_${1:-now}; mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_conv_pointwise_gpu.py -k "expand" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
RTENHIP_EXPAND_DW=all timeout -k 10 600 $PYT tests/test_conv_pointwise_gpu.py -k "expand" > $O/tests_all.log 2>&1 || { echo "tests (all) failed"; tail -40 $O/tests_all.log; exit 1; }
tail -1 $O/tests_all.log
timeout -k 10 600 $PYT tests/test_full_size_gpu.py -k mobilenet > $O/full.log 2>&1 || { echo "full-size failed"; tail -40 $O/full.log; exit 1; }
tail -1 $O/full.log
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --model mobilenet_v2 --batch 128 --steps 60 --warmup 10 --no-secondary --no-cpu-baseline \
    > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -3 $O/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$tag.json $tag
}
for i in 1 2; do run off$i RTENHIP_EDW_MX=0; run on$i RTENHIP_EDW_MX=1; done
for v in 1 0; do
  RTENHIP_EDW_MX=$v timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-secondary --model mobilenet_v2 --batch 128 --steps 20 --warmup 3 > $O/p.log 2>&1 || { echo "rocprof failed"; tail $O/p.log; exit 1; }
  f=$(find $O/p -name 'run_kernel_trace.csv' | head -n 1)
  python3 rten-fork_amd/tools/rocprof_per_forward.py "$f" 10 4 --seq > $O/pf$v.txt || exit 1
  rm -rf $O/p
  echo "== EDW_MX=$v"; sed -n 2,6p $O/pf$v.txt; grep expand_dw $O/pf$v.txt | tail -4
done
