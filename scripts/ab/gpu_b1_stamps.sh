#!/bin/bash
# Stamp timeline of the batch-1 forward under rocprofv3 (kernel durations of
# the same eager launches); env settings as arguments ("-" = default).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/b1st; mkdir -p $O
i=0
for cfg in "$@"; do
  i=$((i+1))
  envs=(); [ "$cfg" != "-" ] && IFS=',' read -ra envs <<< "$cfg"
  for e in "${envs[@]}"; do export "$e"; done
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t$i -o run --output-format csv \
    -- python3 rten-fork_amd/tools/lat_stamps.py > $O/stamps_$i.txt 2>&1 || { echo "stamps $cfg failed"; tail $O/stamps_$i.txt; exit 1; }
  for e in "${envs[@]}"; do unset "${e%%=*}"; done
  f=$(find $O/t$i -name 'run_kernel_trace.csv' | head -n 1)
  python3 rten-fork_amd/tools/last_forward.py "$f" 60 > $O/dur_$i.txt || exit 1
  rm -rf $O/t$i
  echo "== $cfg"; grep -E "^ +[0-9]+ " $O/stamps_$i.txt | head -60 > $O/st_$i.txt; paste $O/st_$i.txt $O/dur_$i.txt | cut -c1-250
done
