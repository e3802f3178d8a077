#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export RTEN_NUM_THREADS=8 RTENHIP_DUAL_DEBUG=1
timeout -k 10 300 python -u -m pytest -q -s --timeout 200 --timeout-method thread tests/test_model_gpu.py -k "dual" 2>&1 | grep -E "dual|passed|failed|Error" | head -60
