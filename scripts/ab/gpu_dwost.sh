#!/bin/bash
# Depthwise whole-plane blocks with LDS-staged 16-byte output stores (product)
# vs direct per-row stores (exp_dw/librten_hip_dwold.so): parity, per-op reports,
# interleaved MobileNetV2 b128 bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/dwost; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py tests/test_full_size_gpu.py tests/test_model_gpu.py -k "depthwise or dw or mobilenet or pool" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for v in new old; do
  lib=""; [ $v = old ] && lib=rten-fork_amd/exp_dw/librten_hip_dwold.so
  RTENHIP_LIB=$lib timeout -k 10 200 python3 rten-fork_amd/tools/model_once.py 2 mobilenet_v2 128 --report > $O/rep_$v.txt 2>&1 || { tail $O/rep_$v.txt; exit 1; }
  echo "== $v"; grep -E "features\.(7|8|12|14|15)\.dw |Graph run" $O/rep_$v.txt
done
for r in 1 2 3; do
  for v in new old; do
    lib=""; [ $v = old ] && lib=rten-fork_amd/exp_dw/librten_hip_dwold.so
    RTENHIP_LIB=$lib timeout -k 10 240 python3 bench.py --model mobilenet_v2 --batch 128 --no-cpu-baseline --no-secondary --steps 30 --warmup 3 > $O/$v$r.json 2> $O/$v$r.err || { tail $O/$v$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$v$r.json $v
  done
done
