#!/bin/bash
# Batch-1 latency anatomy: per-launch stamp timeline of the latency GEMMs
# (tools/lat_stamps.py, eager forward) next to the rocprof kernel durations of
# the same launches, then the replayed bench's per-forward rocprof summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/b1anat_${1:-now}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t -o run --output-format csv \
  -- python3 rten-fork_amd/tools/lat_stamps.py > $O/stamps.txt 2>&1 || { echo "stamps failed"; tail $O/stamps.txt; exit 1; }
f=$(find $O/t -name 'run_kernel_trace.csv' | head -n 1)
python3 rten-fork_amd/tools/last_forward.py "$f" 60 > $O/dur.txt || exit 1
rm -rf $O/t
grep -E "^ +[0-9]+ " $O/stamps.txt | head -60 > $O/st.txt; paste $O/st.txt $O/dur.txt | cut -c1-250
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run --output-format csv \
  -- python3 bench.py --no-cpu-baseline --no-secondary --batch 1 --steps 50 --warmup 5 > $O/bench.log 2>&1 || { echo "rocprof b1 failed"; tail $O/bench.log; exit 1; }
f=$(find $O/p -name 'run_kernel_trace.csv' | head -n 1)
python3 rten-fork_amd/tools/rocprof_per_forward.py "$f" 10 4 --seq > $O/b1_per_forward.txt || exit 1
rm -rf $O/p
head -14 $O/b1_per_forward.txt
