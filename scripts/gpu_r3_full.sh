#!/bin/bash
# Round 3: new tests first, then the whole GPU suite, the full-size BASELINE
# configs and the bench lines.  Each step has its own time limit; the script
# stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export RTEN_NUM_THREADS=8
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_parallel_gpu.py tests/test_optimizer_gpu.py tests/test_threads.py tests/test_conv_pointwise_gpu.py -k "not test_pointwise_valu_bitexact and not test_direct_valu" \
  > gpurun_out/r3_quick.log 2>&1 || { echo "quick tests failed"; tail -40 gpurun_out/r3_quick.log; exit 1; }
tail -3 gpurun_out/r3_quick.log
timeout -k 10 900 $PYT tests -m gpu --deselect tests/test_full_size_gpu.py > gpurun_out/r3_suite.log 2>&1 \
  || { echo "gpu suite failed"; tail -40 gpurun_out/r3_suite.log; exit 1; }
tail -3 gpurun_out/r3_suite.log
timeout -k 10 900 $PYT tests/test_full_size_gpu.py > gpurun_out/r3_full.log 2>&1 \
  || { echo "full-size tests failed"; tail -30 gpurun_out/r3_full.log; exit 1; }
tail -5 gpurun_out/r3_full.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err || exit 1
cat gpurun_out/r3_bench.json
timeout -k 10 300 python -u bench.py --batch 1 --steps 50 --no-cpu-baseline > gpurun_out/r3_bench_b1.json 2>> gpurun_out/r3_bench.err || exit 1
cat gpurun_out/r3_bench_b1.json
timeout -k 10 300 python -u bench.py --model mobilenet_v2 --batch 128 --no-cpu-baseline --timing-report > gpurun_out/r3_bench_mnv2.json 2>> gpurun_out/r3_bench.err || exit 1
head -c 600 gpurun_out/r3_bench_mnv2.json
timeout -k 10 300 python -u bench.py --model bert --batch 32 --no-cpu-baseline --timing-report > gpurun_out/r3_bench_bert.json 2>> gpurun_out/r3_bench.err || exit 1
head -c 600 gpurun_out/r3_bench_bert.json
RTENHIP_DIST_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/r3_bench_rehearsal2.json 2>> gpurun_out/r3_bench.err || exit 1
cat gpurun_out/r3_bench_rehearsal2.json
