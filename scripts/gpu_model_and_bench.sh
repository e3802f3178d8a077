#!/bin/bash
# Run model parity then bench; stop on any fault/timeout (exit codes other than 0/1).
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests/test_model_gpu.py -x -q -m gpu > gpurun_out/model.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/model.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --timing-report --cpu-seconds 8 > gpurun_out/bench.log 2> gpurun_out/bench.err
rc=$?
echo "bench rc=$rc" >> gpurun_out/bench.err
exit $rc
