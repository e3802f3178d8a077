#!/bin/bash
# LayerNorm grouped-loop pipeline: LN parity tests (default grid and a 64-block
# grid that loops), then per-launch stats and the BERT bench per RTENHIP_LN_GRID.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/lngrid; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q -k "layer_norm" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo pytest failed; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
RTENHIP_LN_GRID=64 timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_model_gpu.py -m gpu -x -q -k "layer_norm or bert" --timeout 120 --timeout-method thread > $O/pytest64.log 2>&1 || { echo pytest64 failed; tail -30 $O/pytest64.log; exit 1; }
tail -1 $O/pytest64.log
for G in 0 128 256 384; do
  RTENHIP_LN_GRID=$G timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/g$G -o run --output-format csv -- python3 rten-fork_amd/tools/ln_bench.py > $O/g$G.log 2>&1 || { echo rocprof $G failed; tail $O/g$G.log; exit 1; }
  echo "G=$G $(find $O/g$G -name '*kernel_stats.csv' -exec grep -h layer_norm {} + | awk -F'",' '{print $2}')"
done
for r in 1 2; do
  for G in 0 256; do
    RTENHIP_LN_GRID=$G timeout -k 10 300 python3 bench.py --model bert --batch 32 --no-cpu-baseline > $O/bert_${G}_$r.json 2> $O/bert_${G}_$r.err || { echo bench failed; tail $O/bert_${G}_$r.err; exit 1; }
    python3 -c "import json; b=json.load(open('$O/bert_${G}_$r.json')); print('G=$G', $r, 'bert', b['value'])"
  done
done
