#!/bin/bash
# gemm_lat2 16-byte B copies: latency-GEMM parity tests, the batch-1 model
# tests, then ResNet-50 b1 interleaved A/B (RTENHIP_LAT_NO_BVEC=1 = gathers).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/b1v_${1:-now}; mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_conv_lat_gpu.py tests/test_full_size_gpu.py -k "lat or batch1" tests/test_model_gpu.py -k "unfolded or lat or batch1" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; grep -E "^FAILED|Error" $O/tests.log | head -10
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; exit 1; }
for r in 1 2; do
  for m in on off; do
    if [ $m = off ]; then export RTENHIP_LAT_NO_BVEC=1; else unset RTENHIP_LAT_NO_BVEC; fi
    timeout -k 10 300 python -u bench.py --batch 1 --steps 300 --warmup 30 --no-secondary --no-cpu-baseline \
      > $O/b1_${m}_$r.json 2> $O/b1_${m}_$r.err || { echo "bench $m failed"; tail $O/b1_${m}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bvec', sys.argv[2], d['value'], d['ms_per_step'])" $O/b1_${m}_$r.json $m
  done
done
unset RTENHIP_LAT_NO_BVEC
timeout -k 10 300 python -u rten-fork_amd/tools/model_once.py 1 resnet50 1 --report > $O/report.txt 2>&1 && grep -E "^op layer[1-4]\.[0-9]\.conv[13]|^op layer[1-4].0.downsample" $O/report.txt | head -40
