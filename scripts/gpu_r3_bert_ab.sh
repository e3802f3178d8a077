#!/bin/bash
# BERT-base b32: producer-packed A on / off (interleaved bench runs), then the
# per-op timing report with it on.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/bertab; mkdir -p $O
export RTEN_NUM_THREADS=8
for i in 1 2 3; do
  for v in "pk:RTENHIP_X=1" "nopk:RTENHIP_NO_PK_OUT=1"; do
    name=${v%%:*}
    env ${v#*:} timeout -k 10 200 python -u bench.py --model bert --batch 32 --steps 30 --no-cpu-baseline > $O/${name}_$i.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${name}_$i.json'));print('$name', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv \
  -- python3 bench.py --model bert --batch 32 --steps 20 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "rocprof failed"; tail $O/prof.log; exit 1; }
f=$(find $O/prof -name 'run_kernel_trace.csv' | head -n 1)
python3 rten-fork_amd/tools/rocprof_per_forward.py "$f" 10 156 > $O/per_forward.txt || exit 1
rm -rf $O/prof
cat $O/per_forward.txt
