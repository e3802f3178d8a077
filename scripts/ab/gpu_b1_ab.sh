#!/bin/bash
# Batch-1 A/B: the b1 bench line (hipGraph replay) under env settings given
# as arguments ("NAME=VAL[,NAME=VAL]" or "-" for the default), two rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/b1ab; mkdir -p $O
for round in 1 2; do
  for cfg in "$@"; do
    envs=(); [ "$cfg" != "-" ] && IFS=',' read -ra envs <<< "$cfg"
    env "${envs[@]}" timeout -k 10 200 python -u bench.py --batch 1 --steps 300 --warmup 30 --no-cpu-baseline > $O/r.json 2> $O/r.err || { echo "bench failed: $cfg"; tail $O/r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/r.json'));print('$round', '$cfg', d['value'], d['ms_per_step'])"
  done
done
