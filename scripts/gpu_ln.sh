#!/bin/bash
# LayerNorm: bit-exact parity tests, then per-launch kernel stats of the
# baseline build (ab_base) and the in-tree build at several rows-per-workgroup
# settings, then the BERT bench A/B.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/ln; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q -k "layer_norm" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo pytest failed; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
BASE=$PWD/rten-fork_amd/ab_base/librten_hip.so
for v in base new; do
  for R in ${RS:-0 4 8}; do
    lib=""; [ $v = base ] && lib=$BASE
    RTENHIP_LIB=$lib RTENHIP_LN_ROWS=$R timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/${v}_r$R -o run --output-format csv -- python3 rten-fork_amd/tools/ln_bench.py > $O/${v}_r$R.log 2>&1 || { echo rocprof $v R=$R failed; tail $O/${v}_r$R.log; exit 1; }
    echo "$v R=$R"; find $O/${v}_r$R -name "*kernel_stats.csv" -exec grep -h layer_norm {} +
  done
done
for r in 1 2; do
  for v in base new; do
    lib=""; [ $v = base ] && lib=$BASE
    RTENHIP_LIB=$lib timeout -k 10 300 python bench.py --model bert --batch 32 --no-cpu-baseline > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || { echo bench failed; tail $O/bench_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${v}_$r.json')); print('$v', $r, d['value'])"
  done
done
