#!/bin/bash
# MobileNetV2 b128 rocprof sums: fused / unfused stem under arena offset shifts
# (RTENHIP_ARENA_PAD_MB) and its compute switched off (RTENHIP_SD_DBG), to
# separate layout and clock effects from the kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/mnv2pad_${1:-now}; mkdir -p $O
for cfg in ${CFGS:-1:0 0:0 1:205 1:2 0:2}; do  # fused:pad_mb[:dbg]
  set -- ${cfg//:/ }
  RTENHIP_SD_DBG=${3:-0} RTENHIP_STEM_DWPW=$1 RTENHIP_ARENA_PAD_MB=$2 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-secondary --model mobilenet_v2 --batch 128 --steps 20 --warmup 3 > $O/p.log 2>&1 || { echo "rocprof $cfg failed"; tail $O/p.log; exit 1; }
  f=$(find $O/p -name 'run_kernel_trace.csv' | head -n 1)
  python3 rten-fork_amd/tools/rocprof_per_forward.py "$f" 10 4 --seq > $O/pf_$1_$2.txt || exit 1
  rm -rf $O/p
  python3 - $O/pf_$1_$2.txt $1 $2 ${3:-0} <<'PY'
import re, sys
rows = []
on = False
for l in open(sys.argv[1]):
    if l.startswith('--- one forward'): on = True; continue
    m = re.match(r'\s*(\d+)\s+([\d.]+)\s+gap', l) if on else None
    if m: rows.append(float(m.group(2)))
k = 1 if sys.argv[2] == '1' else 2
print(f"STEM_DWPW={sys.argv[2]} pad={sys.argv[3]}MB dbg={sys.argv[4]} first {sum(rows[:k]):.1f} rest {sum(rows[k:]):.1f} total {sum(rows):.1f} us")
PY
done
