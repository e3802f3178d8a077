#!/bin/bash
# A/B of the pointwise VALU conv kernel: the current build vs the one before
# the round-4 load batching (exp_pwold), MobileNetV2 b128 bench interleaved,
# and the per-op reports of the VALU-picked layers.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/pwab; mkdir -p $O
for r in 1 2; do
  for v in new old; do
    lib=""; [ $v = old ] && lib=rten-fork_amd/exp_pwold/librten_hip_pwold.so
    RTENHIP_LIB=$lib timeout -k 10 300 python -u bench.py --model mobilenet_v2 --batch 128 --no-secondary --no-cpu-baseline > $O/$v$r.json 2> $O/$v$r.err || { echo "bench $v failed"; tail $O/$v$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$v$r.json $v$r
  done
done
for v in new old; do
  lib=""; [ $v = old ] && lib=rten-fork_amd/exp_pwold/librten_hip_pwold.so
  RTENHIP_LIB=$lib timeout -k 10 300 python -u rten-fork_amd/tools/model_once.py 1 mobilenet_v2 128 --report > $O/rep_$v.txt 2>&1 || exit 1
  echo "== $v"; grep -E "valu" $O/rep_$v.txt
done
