#!/bin/bash
# Attention packed-A store: interleaved BERT b32 A/B (RTENHIP_ATTN_PK=0 off),
# and a per-forward rocprof kernel summary of the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/attnpk2; mkdir -p $O
export RTEN_NUM_THREADS=8
for i in 1 2; do
  for v in on off; do
    if [ $v = off ]; then export RTENHIP_ATTN_PK=0; else unset RTENHIP_ATTN_PK; fi
    timeout -k 10 240 python -u bench.py --model bert --batch 32 --no-cpu-baseline > $O/bert_${v}_$i.json 2> $O/bert_${v}_$i.err || { tail $O/bert_${v}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bert_${v}_$i.json'));print('bert $v', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
unset RTENHIP_ATTN_PK
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --model bert --batch 32 --steps 10 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "rocprof failed"; tail $O/prof.log; exit 1; }
f=$(find $O/prof -name 'run_kernel_trace.csv' | head -n 1)
python3 rten-fork_amd/tools/rocprof_per_forward.py "$f" 10 > $O/per_forward.txt || exit 1
rm -rf $O/prof
head -12 $O/per_forward.txt
