#!/bin/bash
# ResNet-50 batch 1: bench A/B (side stream on / off, interleaved) and a
# rocprofv3 kernel trace cut into forwards (dispatch sequence with durations).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/b1p; mkdir -p $O
export RTEN_NUM_THREADS=8
# variants: side stream on/off; latency GEMM K table / late epilogue loads (the round-2 forms)
for i in 1 2; do
  for v in "s0:RTENHIP_SIDE_STREAM=0" "s1:RTENHIP_SIDE_STREAM=1" "ktab:RTENHIP_SIDE_STREAM=0 RTENHIP_LAT_KTAB=1" \
           "late:RTENHIP_SIDE_STREAM=0 RTENHIP_LAT_DBG=4" "old:RTENHIP_SIDE_STREAM=0 RTENHIP_LAT_KTAB=1 RTENHIP_LAT_DBG=4"; do
    name=${v%%:*}
    env ${v#*:} timeout -k 10 200 python -u bench.py --batch 1 --steps 300 --warmup 30 --no-cpu-baseline > $O/b1_${name}_$i.json 2> $O/b1.err || { tail $O/b1.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b1_${name}_$i.json'));print('$name', d['value'], d['ms_per_step'])"
  done
done
RTENHIP_SIDE_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv \
  -- python3 bench.py --batch 1 --steps 20 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "rocprof failed"; tail $O/prof.log; exit 1; }
f=$(find $O/prof -name 'run_kernel_trace.csv' | head -n 1)
python3 rten-fork_amd/tools/rocprof_per_forward.py "$f" 10 4 --seq > $O/seq.txt || exit 1
rm -rf $O/prof
head -70 $O/seq.txt
