#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/lnrows; mkdir -p $O
for r in 8 4 6 12 16; do
  RTENHIP_LN_ROWS=$r timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$r -o run -- python3 rten-fork_amd/tools/ln_bench.py > $O/p$r.log 2>&1 || { echo "rocprof fail $r"; tail -5 $O/p$r.log; exit 1; }
  f=$(find $O/p$r -name "run_kernel_stats.csv" | head -1)
  python3 -c "import csv,sys; [print(sys.argv[2], r['Name'][:40], round(float(r['AverageNs'])/1000,2)) for r in csv.DictReader(open(sys.argv[1])) if 'layer_norm' in r['Name']]" "$f" $r
  rm -rf $O/p$r
done
for r in 8 6 8 6; do
RTENHIP_LN_ROWS=$r timeout -k 10 300 python -u bench.py --model bert --batch 32 --no-cpu-baseline --no-secondary --steps 30 --warmup 5 > $O/bert_$r.json 2> $O/bert_$r.err || { echo "bench failed"; tail -5 $O/bert_$r.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bert rows', sys.argv[2], d['value'], d['ms_per_step'])" $O/bert_$r.json $r
done
