#!/bin/bash
# rocprofv3 kernel trace of the batch-1 bench (hipGraph replay) under env
# settings given as arguments ("-" = default); per-forward dispatch sequence.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/b1prof; mkdir -p $O
i=0
for cfg in "$@"; do
  i=$((i+1))
  envs=(); [ "$cfg" != "-" ] && IFS=',' read -ra envs <<< "$cfg"
  for e in "${envs[@]}"; do export "$e"; done
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t$i -o run --output-format csv \
    -- python3 bench.py --batch 1 --steps 50 --warmup 5 --no-cpu-baseline > $O/t$i.log 2>&1 || { echo "rocprof $cfg failed"; tail $O/t$i.log; exit 1; }
  for e in "${envs[@]}"; do unset "${e%%=*}"; done
  f=$(find $O/t$i -name 'run_kernel_trace.csv' | head -n 1)
  python3 rten-fork_amd/tools/rocprof_per_forward.py "$f" 10 4 --seq > $O/seq_$i.txt || exit 1
  rm -rf $O/t$i
  echo "== $cfg"; head -12 $O/seq_$i.txt
done
