#!/bin/bash
# attention change: full GPU parity suite, then BERT b32 A/B (ab_base =
# previous attention kernel) with rocprof per-forward summaries and bench lines.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/att; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo pytest failed; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
BASE=$PWD/rten-fork_amd/ab_base/librten_hip.so
for v in base new; do
  lib=""; [ $v = base ] && lib=$BASE
  RTENHIP_LIB=$lib timeout -k 10 400 rocprofv3 --kernel-trace -d $O/prof_$v -o run --output-format csv -- python3 bench.py --model bert --batch 32 --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_$v.log 2>&1 || { echo rocprof $v failed; tail $O/prof_$v.log; exit 1; }
  echo "== $v"; python3 rten-fork_amd/tools/rocprof_per_forward.py $(find $O/prof_$v -name run_kernel_trace.csv) 10 156
done
for r in 1 2; do
  for v in base new; do
    lib=""; [ $v = base ] && lib=$BASE
    RTENHIP_LIB=$lib timeout -k 10 300 python3 bench.py --model bert --batch 32 --no-cpu-baseline > $O/bert_${v}_$r.json 2> $O/bert_${v}_$r.err || { echo bench failed; tail $O/bert_${v}_$r.err; exit 1; }
    python3 -c "import json; b=json.load(open('$O/bert_${v}_$r.json')); print('$v', $r, 'bert', b['value'])"
  done
done
