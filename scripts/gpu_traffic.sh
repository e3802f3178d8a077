#!/bin/bash
# HBM traffic of the conv GEMM kernels (FETCH_SIZE and WRITE_SIZE need
# separate passes on gfx950), ResNet-50 b64, RUNS eager forward passes after
# the tuning run.  Summarised by rten-fork_amd/tools/pmc_traffic.py.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
RUNS=${RUNS:-2}
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/traffic -o fetch -- python3 rten-fork_amd/tools/model_once.py $RUNS > gpurun_out/traffic_fetch.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/traffic -o write -- python3 rten-fork_amd/tools/model_once.py $RUNS > gpurun_out/traffic_write.log 2>&1 || exit $?
