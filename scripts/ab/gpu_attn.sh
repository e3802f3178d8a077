#!/bin/bash
# FusedAttention timing experiments (tools/attn_bench.py at BERT-base b32):
# the product kernel and the RTENHIP_ATT_EXPERIMENT builds (make attexp),
# average attention_kernel duration from rocprofv3 --kernel-trace --stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/attn; mkdir -p $O
for v in product ${ATT_EXPS:-1 2 3 4 5}; do
  lib=""; [ $v != product ] && lib=rten-fork_amd/exp_att/librten_hip_att$v.so
  RTENHIP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv \
    -- python3 rten-fork_amd/tools/attn_bench.py > $O/$v.log 2>&1 || { echo "attn $v failed"; tail $O/$v.log; exit 1; }
  f=$(find $O/$v -name 'run_kernel_stats.csv' | head -n 1)
  python3 -c "import csv,sys; [print(sys.argv[2], r['Name'][:40], r['Calls'], '%.2f us' % (float(r['AverageNs']) / 1e3)) for r in csv.DictReader(open(sys.argv[1])) if 'attention' in r['Name']]" "$f" $v
  rm -rf $O/$v
done
