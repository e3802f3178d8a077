#!/bin/bash
# Conv chain session: parity tests, then ResNet-50 b1 with the chain off /
# auto / forced (bench lines, build-time timing), a stamped eager run and the
# per-forward rocprof summary of the chain build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/chain_${1:-now}; mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_chain_gpu.py > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; grep -E "^FAILED|Error" $O/tests.log | head -10
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "chain tests aborted rc=$rc"; exit 1; }
for m in 0 -1 1; do
  RTENHIP_CHAIN=$m RTENHIP_CHAIN_LOG=1 timeout -k 10 300 python -u bench.py --batch 1 --steps 300 --warmup 30 --no-secondary \
    --no-cpu-baseline --timing-report > $O/b1_$m.json 2> $O/b1_$m.err || { echo "bench chain=$m failed"; tail $O/b1_$m.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('chain', sys.argv[2], d['value'], d['ms_per_step'])" $O/b1_$m.json $m
  grep "conv chain" $O/b1_$m.err | head -3
done
RTENHIP_CHAIN=1 RTENHIP_CHAIN_NO_BVEC=1 RTENHIP_CHAIN_STAMPS=$O/stamps_nobvec.bin timeout -k 10 300 python -u rten-fork_amd/tools/model_once.py 2 resnet50 1 > $O/once_nobvec.txt 2>&1 || { echo "stamped run failed"; tail $O/once_nobvec.txt; exit 1; }
python3 rten-fork_amd/tools/chain_stamps.py $O/stamps_nobvec.bin > $O/stamps_nobvec.txt && tail -1 $O/stamps_nobvec.txt
RTENHIP_CHAIN=1 RTENHIP_CHAIN_STAMPS=$O/stamps.bin timeout -k 10 300 python -u rten-fork_amd/tools/model_once.py 2 resnet50 1 --report > $O/once.txt 2>&1 || { echo "stamped run failed"; tail $O/once.txt; exit 1; }
grep "chain of" $O/once.txt
python3 rten-fork_amd/tools/chain_stamps.py $O/stamps.bin > $O/stamps.txt && head -60 $O/stamps.txt
# Host-resident input: copy / kernel overlap of the pipelined staging.
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/hostin -o run --output-format csv \
  -- python3 bench.py --host-input --no-secondary --no-cpu-baseline --steps 20 --warmup 5 > $O/hostin.json 2> $O/hostin.err \
  || { echo "host-input trace failed"; tail $O/hostin.err; exit 1; }
python3 rten-fork_amd/tools/copy_overlap.py $O/hostin 12 > $O/hostin_overlap.txt; cat $O/hostin_overlap.txt
rm -rf $O/hostin
NO_SUITE=1 bash scripts/gpu_check.sh ${1:-now}_bench || exit 1
