#!/bin/bash
# Stem parity cases only (tests/test_conv_pointwise_gpu.py -k stem).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/stemtests_${1:-now}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_pointwise_gpu.py -k stem > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -c PASSED $O/tests.log; tail -1 $O/tests.log
