#!/bin/bash
# Full GPU check: parity tests, smoke, bench lines for the three single-GPU
# configs (ResNet-50 b64, MobileNetV2 b128, BERT-base b32).  Every GPU step
# has its own time limit; the script stops at the first failure.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u rten-fork_amd/tools/bisect_model.py > gpurun_out/bisect.log 2>&1 || { echo bisect failed; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo gpu tests failed; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench_resnet.log 2> gpurun_out/bench_resnet.err || { echo bench failed; exit 1; }
timeout -k 10 300 python bench.py --model mobilenet_v2 --batch 128 --no-cpu-baseline --timing-report > gpurun_out/bench_mnv2.log 2> gpurun_out/bench_mnv2.err || { echo bench mnv2 failed; exit 1; }
timeout -k 10 300 python bench.py --model bert --batch 32 --no-cpu-baseline --timing-report > gpurun_out/bench_bert.log 2> gpurun_out/bench_bert.err || { echo bench bert failed; exit 1; }
echo all-ok
