#!/bin/bash
# Round 3 profiles: rocprofv3 kernel-trace summaries of the bench (ResNet-50
# b64, b1, MobileNetV2 b128, BERT b32) and PMC HBM traffic passes (FETCH_SIZE
# and WRITE_SIZE in separate runs) for MobileNetV2 b128, BERT b32, ResNet-50 b64.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/prof3; mkdir -p $O
export RTEN_NUM_THREADS=8
prof() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$n -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { echo "rocprof $n failed"; tail $O/$n.log; exit 1; }
  f=$(find $O/$n -name 'run_kernel_stats.csv' | head -n 1); cp "$f" $O/${n}_kernel_stats.csv
  f=$(find $O/$n -name 'run_kernel_trace.csv' | head -n 1)
  python3 rten-fork_amd/tools/rocprof_per_forward.py "$f" 10 ${MINP:-4} > $O/${n}_per_forward.txt || exit 1
  [ "$n" = resnet50_b1 ] && { python3 rten-fork_amd/tools/rocprof_per_forward.py "$f" 10 4 --seq > $O/resnet50_b1_seq.txt || exit 1; }
  rm -rf $O/$n   # traces are large; gpurun copies back at most 64 MiB
  echo "== $n"; grep '^{' $O/$n.log | head -c 300; echo
}
prof resnet50_b64 --steps 20 --warmup 3
prof resnet50_b1 --batch 1 --steps 50 --warmup 5
prof mobilenet_v2_b128 --model mobilenet_v2 --batch 128 --steps 20 --warmup 3
MINP=156 prof bert_b32 --model bert --batch 32 --steps 20 --warmup 3
pmc() {  # name, model, batch
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$1 -o $(echo ${c%%_SIZE} | tr A-Z a-z) \
      -- python3 rten-fork_amd/tools/model_once.py 2 $2 $3 > $O/pmc_$1_$c.log 2>&1 || { echo "pmc $1 $c failed"; tail $O/pmc_$1_$c.log; exit 1; }
  done
  python3 rten-fork_amd/tools/pmc_traffic.py $O/pmc_$1 2 --marker > $O/pmc_$1.json 2>&1 || { echo "summary $1 failed"; cat $O/pmc_$1.json; exit 1; }
  rm -rf $O/pmc_$1; head -c 300 $O/pmc_$1.json; echo
}
pmc mobilenet_v2_b128 mobilenet_v2 128
pmc bert_b32 bert 32
pmc resnet50_b64 resnet50 64
