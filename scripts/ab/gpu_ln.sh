#!/bin/bash
# LayerNorm timing experiments (tools/ln_graph_bench.py, BERT-base b32 shape
# with the packed-A output): the product kernel and the RTENHIP_LN_EXPERIMENT
# builds (make lnexp); average layer_norm_rows_kernel duration per launch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/ln; mkdir -p $O
for v in product ${LN_EXPS:-1 2 3}; do
  lib=""; [ $v != product ] && lib=rten-fork_amd/exp_ln/librten_hip_ln$v.so
  RTENHIP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv \
    -- python3 rten-fork_amd/tools/ln_graph_bench.py > $O/$v.log 2>&1 || { echo "ln $v failed"; tail $O/$v.log; exit 1; }
  f=$(find $O/$v -name 'run_kernel_stats.csv' | head -n 1)
  python3 -c "import csv,sys; [print(sys.argv[2], r['Name'][:50], r['Calls'], '%.2f us' % (float(r['AverageNs']) / 1e3)) for r in csv.DictReader(open(sys.argv[1])) if 'layer_norm' in r['Name'] or 'gemm' in r['Name']]" "$f" $v
  rm -rf $O/$v
done
for r in ${LN_ROWS_SWEEP:-}; do  # rows per workgroup (product default 6144 / len = 8)
  RTENHIP_LN_ROWS=$r timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/r$r -o run --output-format csv \
    -- python3 rten-fork_amd/tools/ln_graph_bench.py > $O/r$r.log 2>&1 || { echo "ln rows $r failed"; tail $O/r$r.log; exit 1; }
  f=$(find $O/r$r -name 'run_kernel_stats.csv' | head -n 1)
  python3 -c "import csv,sys; [print(sys.argv[2], r['Name'][:50], r['Calls'], '%.2f us' % (float(r['AverageNs']) / 1e3)) for r in csv.DictReader(open(sys.argv[1])) if 'layer_norm' in r['Name']]" "$f" rows$r
  rm -rf $O/r$r
done
