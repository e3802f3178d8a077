#!/bin/bash
# A/B of the DMA GEMM tile order (DmaDesc::swz): BERT-base b32 with the dense
# MatMuls in strips of g tile columns vs the default order, and ResNet-50 b64
# with every DMA GEMM swizzled; interleaved, two rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/swz; mkdir -p $O
run() {  # tag, env..., -- bench args
  local tag=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-secondary "$@" > $O/$tag.json 2> $O/$tag.err \
    || { echo "bench $tag failed"; tail $O/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$tag.json $tag
}
for r in 1 2; do
  run bert_def$r X=0 -- --model bert --batch 32 --steps 20 --warmup 3
  run bert_s8_$r RTENHIP_DMA_SWZ_MM=8 -- --model bert --batch 32 --steps 20 --warmup 3
  run bert_s4_$r RTENHIP_DMA_SWZ_MM=4 -- --model bert --batch 32 --steps 20 --warmup 3
  run rn_def$r X=0 -- --steps 20 --warmup 3
  run rn_s8_$r RTENHIP_DMA_SWZ=8 -- --steps 20 --warmup 3
done
