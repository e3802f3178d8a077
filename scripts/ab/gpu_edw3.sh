#!/bin/bash
# A/B: expand+depthwise with packed depthwise pairs (product) vs the unpacked
# kernel (exp_edw/librten_hip_edwold.so, same fusion policy), MobileNetV2 b128
# interleaved; then the LayerNorm with 16 rows per workgroup (exp_ln/librten_hip_lnr16.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/edw3; mkdir -p $O
run() {
  local tag=$1 lib=$2
  RTENHIP_LIB=$lib timeout -k 10 240 python3 bench.py --model mobilenet_v2 --batch 128 --no-cpu-baseline --no-secondary --steps 30 --warmup 3 > $O/$tag.json 2> $O/$tag.err \
    || { echo "bench $tag failed"; tail $O/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$tag.json $tag
}
for r in 1 2 3; do run packed$r "" && run old$r rten-fork_amd/exp_edw/librten_hip_edwold.so || exit 1; done
LN_EXPS=r16 bash scripts/ab/gpu_ln.sh
