#!/bin/bash
# Attention / LayerNorm parity tests, then per-launch times under rocprof:
# attention QW=2 vs QW=4 (tools/attn_bench.py) and the LayerNorm rows kernel
# as BERT runs it (tools/ln_graph_bench.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/bert5b_${1:-now}; mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_model_gpu.py tests/test_ops_gpu.py -k "attention or layernorm or layer_norm or packed" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; grep -E "^FAILED|Error" $O/tests.log | head -10
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; exit 1; }
stat() { python3 -c "import csv,sys; [print(sys.argv[2], r['Name'][:48], r['Calls'], '%.2f us' % (float(r['AverageNs']) / 1e3)) for r in csv.DictReader(open(sys.argv[1])) if any(k in r['Name'] for k in ('attention', 'layer_norm'))]" "$1" "$2"; }
for qw in 2 4 2 4; do
  RTENHIP_ATT_QW=$qw timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/a$qw -o run --output-format csv \
    -- python3 rten-fork_amd/tools/attn_bench.py > $O/a$qw.log 2>&1 || { echo "attn $qw failed"; tail $O/a$qw.log; exit 1; }
  stat "$(find $O/a$qw -name 'run_kernel_stats.csv' | head -n 1)" "qw$qw"; rm -rf $O/a$qw
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/ln -o run --output-format csv \
  -- python3 rten-fork_amd/tools/ln_graph_bench.py > $O/ln.log 2>&1 || { echo "ln failed"; tail $O/ln.log; exit 1; }
stat "$(find $O/ln -name 'run_kernel_stats.csv' | head -n 1)" ln; rm -rf $O/ln
