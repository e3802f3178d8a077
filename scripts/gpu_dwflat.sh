#!/bin/bash
# Whole-plane depthwise staging: conv parity tests, dwbench with it off/on,
# then MobileNetV2 bench lines off/on (interleaved).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/dwf
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or depthwise or mobilenet" > gpurun_out/dwf/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/dwf/tests.log; exit 1; }
tail -2 gpurun_out/dwf/tests.log
for on in 0 1; do
  echo "== RTENHIP_DW_FLAT=$on"; RTENHIP_DW_FLAT=$on timeout -k 10 120 python3 rten-fork_amd/tools/dwbench.py > gpurun_out/dwf/dwbench_$on.log 2>&1 || { echo dwbench failed; tail gpurun_out/dwf/dwbench_$on.log; exit 1; }
  grep dw gpurun_out/dwf/dwbench_$on.log
done
for r in 1 2; do for on in 0 1; do
  RTENHIP_DW_FLAT=$on timeout -k 10 300 python3 bench.py --model mobilenet_v2 --batch 128 --no-cpu-baseline --timing-report --steps 20 > gpurun_out/dwf/mb_${on}_$r.json 2> gpurun_out/dwf/mb_${on}_$r.err || { echo bench failed; tail gpurun_out/dwf/mb_${on}_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/dwf/mb_${on}_$r.json')); print('flat=$on', $r, d['value'])"
done; done
