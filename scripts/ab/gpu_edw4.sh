#!/bin/bash
# A/B on one box: expand+depthwise also fused for C_in = 32 at stride 2 (features.7, product)
# vs C_in 16 / 24 only (exp_edw/librten_hip_pol.so); MobileNetV2 b128 interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/edw4; mkdir -p $O
for r in 1 2 3; do
  for v in new old; do
    lib=""; [ $v = old ] && lib=rten-fork_amd/exp_edw/librten_hip_pol.so
    RTENHIP_LIB=$lib timeout -k 10 240 python3 bench.py --model mobilenet_v2 --batch 128 --no-cpu-baseline --no-secondary --steps 30 --warmup 3 > $O/$v$r.json 2> $O/$v$r.err || { tail $O/$v$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$v$r.json $v
  done
done
