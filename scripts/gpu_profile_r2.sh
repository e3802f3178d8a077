#!/bin/bash
# Round-2 evidence: the three single-GPU bench lines with their per-op timing
# reports, rocprofv3 kernel-trace + stats of each, and the HBM traffic passes
# (FETCH_SIZE / WRITE_SIZE, one counter per pass) of ResNet-50 b64.  Each GPU
# step has its own time limit; the script stops at the first failure.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/r2
O=gpurun_out/r2
bench() {  # name, bench args
  local name=$1; shift
  timeout -k 10 400 python3 bench.py --timing-report "$@" > $O/bench_$name.json 2> $O/timing_$name.txt \
    || { echo "bench $name failed"; tail $O/timing_$name.txt; return 1; }
  cat $O/bench_$name.json
}
prof() {  # name, bench args
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$name -o run --output-format csv \
    -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > $O/prof_$name.log 2>&1 \
    || { echo "rocprof $name failed"; tail $O/prof_$name.log; return 1; }
}
bench resnet50 &&
  bench mobilenet_v2 --model mobilenet_v2 --batch 128 --no-cpu-baseline &&
  bench bert --model bert --batch 32 --no-cpu-baseline &&
  prof resnet50 && prof mobilenet_v2 --model mobilenet_v2 --batch 128 && prof bert --model bert --batch 32 &&
  timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/traffic -o fetch \
    -- python3 rten-fork_amd/tools/model_once.py 2 > $O/traffic_fetch.log 2>&1 &&
  timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/traffic -o write \
    -- python3 rten-fork_amd/tools/model_once.py 2 > $O/traffic_write.log 2>&1 &&
  echo profile-r2-ok
