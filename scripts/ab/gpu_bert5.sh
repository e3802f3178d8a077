#!/bin/bash
# BERT side kernels: attention query halves (V over K) and the LayerNorm's
# packed-A stores from registers -- parity tests, interleaved BERT-base b32
# A/B (RTENHIP_ATT_QW=4 = one workgroup per (batch, head)), and the
# per-forward rocprof summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/bert5_${1:-now}; mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_model_gpu.py -k "attention or bert or layernorm or matmul" tests/test_ops_gpu.py -k "layer_norm or attention" tests/test_full_size_gpu.py -k bert > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; grep -E "^FAILED|Error" $O/tests.log | head -10
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; exit 1; }
for r in 1 2; do
  for m in 2 4; do
    RTENHIP_ATT_QW=$m timeout -k 10 300 python -u bench.py --model bert --batch 32 --steps 40 --warmup 5 --no-cpu-baseline \
      > $O/bert_${m}_$r.json 2> $O/bert_${m}_$r.err || { echo "bench $m failed"; tail $O/bert_${m}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('qw', sys.argv[2], d['value'], d['ms_per_step'])" $O/bert_${m}_$r.json $m
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv \
  -- python3 bench.py --model bert --batch 32 --steps 20 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "rocprof failed"; tail $O/prof.log; exit 1; }
f=$(find $O/prof -name 'run_kernel_trace.csv' | head -n 1)
python3 rten-fork_amd/tools/rocprof_per_forward.py "$f" 10 85 > $O/per_forward.txt && head -12 $O/per_forward.txt
rm -rf $O/prof
