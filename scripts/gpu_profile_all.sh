#!/bin/bash
# rocprofv3 kernel-trace + stats of the three single-GPU bench lines
# (ResNet-50 b64, BERT-base b32, MobileNetV2 b128).  Each step has its own
# time limit; the script stops at the first failure.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, bench args
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$name -o run --output-format csv \
    -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/prof_$name.log 2>&1
}
run resnet50 && run bert --model bert --batch 32 && run mobilenet_v2 --model mobilenet_v2 --batch 128 && echo profiles-ok
