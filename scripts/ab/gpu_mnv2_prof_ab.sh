#!/bin/bash
# MobileNetV2 b128 replayed forwards under rocprofv3, the stem fused into the
# depthwise -> projection kernel or not (RTENHIP_STEM_DWPW=0): per-kernel
# per-forward summaries side by side.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/mnv2ab_${1:-now}; mkdir -p $O
for v in 1 0; do
  RTENHIP_STEM_DWPW=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p$v -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-secondary --model mobilenet_v2 --batch 128 --steps 20 --warmup 3 > $O/p$v.log 2>&1 || { echo "rocprof $v failed"; tail $O/p$v.log; exit 1; }
  f=$(find $O/p$v -name 'run_kernel_trace.csv' | head -n 1)
  python3 rten-fork_amd/tools/rocprof_per_forward.py "$f" 10 4 --seq > $O/pf$v.txt || exit 1
  rm -rf $O/p$v
  echo "== STEM_DWPW=$v"; sed -n 2,8p $O/pf$v.txt; sed -n '/one forward/,+4p' $O/pf$v.txt
done
