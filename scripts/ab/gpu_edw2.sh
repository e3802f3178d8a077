#!/bin/bash
# Fused expand+depthwise with packed depthwise pairs, default on for C_in 16 / 24:
# parity (pair tests, MobileNetV2 graph tests, full size b128), bench lines, per-op report.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/edw2${TAG:-}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_conv_pointwise_gpu.py tests/test_full_size_gpu.py -k "expand or mobilenet" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2; do
  timeout -k 10 240 python3 bench.py --model mobilenet_v2 --batch 128 --no-cpu-baseline --no-secondary --steps 20 --warmup 3 > $O/b$r.json 2> $O/b$r.err || { tail $O/b$r.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('mnv2', d['value'], d['ms_per_step'])" $O/b$r.json
done
timeout -k 10 200 python3 rten-fork_amd/tools/model_once.py 2 mobilenet_v2 128 --report > $O/rep.txt 2>&1 || { tail $O/rep.txt; exit 1; }
grep -E "^op features\.[1-7]\.|Conv\(expand" $O/rep.txt | head -24
