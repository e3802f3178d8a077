#!/bin/bash
# rocprofv3 kernel-trace summaries (per forward, steady state) of bench
# configurations, and PMC HBM traffic passes (FETCH_SIZE and WRITE_SIZE in
# separate runs, MI355X_MICROARCH.md HBM section).
# Usage: scripts/gpu_prof.sh TAG CONFIG...   CONFIG: resnet50_b64 | resnet50_b1 |
#        mobilenet_v2_b128 | bert_b32 | pmc_<model>_<batch> (e.g. pmc_bert_32)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/prof_$TAG; mkdir -p $O
prof() {  # name, min_period, bench args...
  local n=$1 mp=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$n -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-secondary "$@" > $O/$n.log 2>&1 || { echo "rocprof $n failed"; tail $O/$n.log; exit 1; }
  f=$(find $O/$n -name 'run_kernel_stats.csv' | head -n 1); cp "$f" $O/${n}_kernel_stats.csv
  f=$(find $O/$n -name 'run_kernel_trace.csv' | head -n 1)
  python3 rten-fork_amd/tools/rocprof_per_forward.py "$f" 10 $mp --seq > $O/${n}_per_forward.txt || exit 1
  rm -rf $O/$n
  echo "== $n"; head -14 $O/${n}_per_forward.txt
}
pmc() {  # model, batch
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$1 -o $(echo ${c%%_SIZE} | tr A-Z a-z) \
      -- python3 rten-fork_amd/tools/model_once.py 2 $1 $2 > $O/pmc_$1_$c.log 2>&1 || { echo "pmc $1 $c failed"; tail $O/pmc_$1_$c.log; exit 1; }
  done
  python3 rten-fork_amd/tools/pmc_traffic.py $O/pmc_$1 2 --marker > $O/pmc_traffic_$1_b$2.json 2>&1 || { echo "summary $1 failed"; cat $O/pmc_traffic_$1_b$2.json; exit 1; }
  rm -rf $O/pmc_$1; head -c 400 $O/pmc_traffic_$1_b$2.json; echo
}
for c in "$@"; do
  case $c in
    resnet50_b64) prof resnet50_b64 4 --steps 20 --warmup 3 ;;
    resnet50_b1) prof resnet50_b1 4 --batch 1 --steps 50 --warmup 5 ;;
    mobilenet_v2_b128) prof mobilenet_v2_b128 4 --model mobilenet_v2 --batch 128 --steps 20 --warmup 3 ;;
    bert_b32) prof bert_b32 85 --model bert --batch 32 --steps 20 --warmup 3 ;;
    pmc_*) m=${c#pmc_}; pmc ${m%_*} ${m##*_} ;;
  esac
done
