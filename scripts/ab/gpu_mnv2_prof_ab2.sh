#!/bin/bash
# MobileNetV2 b128: rocprofv3 replayed forwards, stem fusion on / off
# interleaved twice; per-forward kernel sums (first kernels vs the rest).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/mnv2ab2_${1:-now}; mkdir -p $O
for it in 1 2; do for v in 1 0; do
  RTENHIP_STEM_DWPW=$v timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p$v -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-secondary --model mobilenet_v2 --batch 128 --steps 20 --warmup 3 > $O/p$v.log 2>&1 || { echo "rocprof $v failed"; tail $O/p$v.log; exit 1; }
  f=$(find $O/p$v -name 'run_kernel_trace.csv' | head -n 1)
  python3 rten-fork_amd/tools/rocprof_per_forward.py "$f" 10 4 --seq > $O/pf${v}_$it.txt || exit 1
  rm -rf $O/p$v
  python3 - $O/pf${v}_$it.txt $v <<'PY'
import re, sys
rows = []
on = False
for l in open(sys.argv[1]):
    if l.startswith('--- one forward'): on = True; continue
    m = re.match(r'\s*(\d+)\s+([\d.]+)\s+gap', l) if on else None
    if m: rows.append(float(m.group(2)))
k = 1 if sys.argv[2] == '1' else 2
print(f"STEM_DWPW={sys.argv[2]} first {sum(rows[:k]):.1f} rest {sum(rows[k:]):.1f} total {sum(rows):.1f} us")
PY
done; done
