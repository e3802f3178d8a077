#!/bin/bash
# Fused-block round: parity tests, per-block timing (fused / expand-only /
# apart) and MobileNetV2 b128 with every block fused vs the default policy.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/mb2_${1:-now}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_mbconv_block_gpu.py tests/test_parallel_gpu.py > $O/t.log 2>&1; rc=$?
tail -2 $O/t.log; grep -E "^FAILED|differ" $O/t.log | head; [ $rc -eq 0 ] || exit 1
for blk in 1 2 3 4 5 8 12; do
  for v in product apart; do
    env=RTENHIP_MBCONV=all; [ $v = apart ] && env=RTENHIP_MBCONV=0
    env $env timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/k -o run --output-format csv \
      -- python3 rten-fork_amd/tools/mb_bench.py $blk > $O/${blk}_$v.log 2>&1 || { echo "mb $blk $v failed"; exit 1; }
    f=$(find $O/k -name 'run_kernel_trace.csv' | head -n 1)
    # the last replay's dispatches (steady state): total kernel time of one block run
    python3 - "$f" $blk $v <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1]))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
# one replay = the trailing period of the dispatch sequence
for p in range(1, len(names) // 2 + 1):
    if names[-p:] == names[-2 * p:-p]:
        break
tail = rows[-10 * p:]
tot = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tail) / 10 / 1e3
print(sys.argv[2], sys.argv[3], "%.1f us per block run (%d kernels)" % (tot, p))
PY
    rm -rf $O/k
  done
done
for v in all default; do
  env=RTENHIP_MBCONV=all; [ $v = default ] && env=X=0
  env $env timeout -k 10 300 python -u bench.py --model mobilenet_v2 --batch 128 --no-secondary --no-cpu-baseline > $O/mnv2_$v.json 2> $O/mnv2_$v.err \
    || { echo "bench failed"; tail $O/mnv2_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('mnv2', sys.argv[2], d['value'], d['ms_per_step'])" $O/mnv2_$v.json $v
done
