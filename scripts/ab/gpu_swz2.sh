#!/bin/bash
# Tile-order sweep, second pass: BERT-base b32 dense MatMuls in strips of 8 (default) / 16 / 32
# tile columns, ResNet-50 b64 conv GEMMs m-fastest (default) / strips of 2 / 4; interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/swz2; mkdir -p $O
run() {  # tag, env..., -- bench args
  local tag=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-secondary "$@" > $O/$tag.json 2> $O/$tag.err \
    || { echo "bench $tag failed"; tail $O/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$tag.json $tag
}
for r in 1 2; do
  run bert_s8_$r X=0 -- --model bert --batch 32 --steps 20 --warmup 3 || exit 1
  run bert_s16_$r RTENHIP_DMA_SWZ_MM=16 -- --model bert --batch 32 --steps 20 --warmup 3 || exit 1
  run bert_s32_$r RTENHIP_DMA_SWZ_MM=32 -- --model bert --batch 32 --steps 20 --warmup 3 || exit 1
  run rn_def$r X=0 -- --steps 20 --warmup 3 || exit 1
  run rn_s2_$r RTENHIP_DMA_SWZ=2 -- --steps 20 --warmup 3 || exit 1
  run rn_s4_$r RTENHIP_DMA_SWZ=4 -- --steps 20 --warmup 3 || exit 1
done
