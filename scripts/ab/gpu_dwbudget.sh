#!/bin/bash
# Depthwise LDS budget (RTENHIP_DW_LDS_FLOATS, default 4096) per MobileNetV2 layer:
# per-op reports and bench lines at 4096 / 8192 / 16384 floats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/dwb; mkdir -p $O
for b in 4096 8192 16384; do
  RTENHIP_DW_LDS_FLOATS=$b timeout -k 10 200 python3 rten-fork_amd/tools/model_once.py 2 mobilenet_v2 128 --report > $O/rep_$b.txt 2>&1 || { tail $O/rep_$b.txt; exit 1; }
  echo "== budget $b"; grep -E "\.dw |Graph run" $O/rep_$b.txt
done
for r in 1 2; do
  for b in 4096 8192; do
    RTENHIP_DW_LDS_FLOATS=$b timeout -k 10 240 python3 bench.py --model mobilenet_v2 --batch 128 --no-cpu-baseline --no-secondary --steps 30 --warmup 3 > $O/b${b}_$r.json 2> $O/b${b}_$r.err || { tail $O/b${b}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/b${b}_$r.json b$b
  done
done
