#!/bin/bash
# A/B/... of library builds in one box session: bench.py with per-op timing,
# each variant twice, interleaved.  usage: VARS="ab_base ab_x" [BENCH_ARGS=...] bash scripts/gpu_abn.sh
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/ab
for r in 1 2; do
  for v in $VARS; do
    RTENHIP_LIB=$PWD/rten-fork_amd/$v/librten_hip.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --timing-report --steps 20 $BENCH_ARGS \
      > gpurun_out/ab/${v}_$r.json 2> gpurun_out/ab/${v}_$r.err || { echo "$v failed"; tail gpurun_out/ab/${v}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/${v}_$r.json')); print('$v', $r, d['value'], d['roofline']['kernel_ms_per_step'])"
  done
done
