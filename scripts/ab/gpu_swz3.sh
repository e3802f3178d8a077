#!/bin/bash
# BERT-base b32: dense MatMul strip width, fixed (8) vs sized per GEMM from B's
# bytes (RTENHIP_DMA_SWZ_MM=-KiB), interleaved, two rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/swz3; mkdir -p $O
for r in 1 2; do
  for v in 8 -1024 -2048 -3072 4; do
    RTENHIP_DMA_SWZ_MM=$v timeout -k 10 300 python -u bench.py --model bert --batch 32 --steps 20 --warmup 3 --no-secondary --no-cpu-baseline > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { echo "bench $v failed"; tail $O/b_${v}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); print('swz $v round $r', d['value'], d['ms_per_step'])"
  done
done
