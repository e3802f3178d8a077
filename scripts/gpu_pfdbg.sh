#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/pfdbg; mkdir -p $O
for v in 0 1; do
RTENHIP_DMA_PF=$v timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_model_gpu.py -k "persistent_modes or unfolded_bn or batch64_full or bottleneck" > $O/t_$v.log 2>&1
echo "PF=$v rc=$?"; tail -2 $O/t_$v.log; grep -E "^FAILED" $O/t_$v.log | head
done
