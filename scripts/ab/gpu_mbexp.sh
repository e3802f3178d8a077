#!/bin/bash
# Fused-block timing experiments (tools/mb_bench.py, MobileNetV2 b128 block
# shapes): product kernel, the RTENHIP_MB_EXPERIMENT builds, and the convs
# apart (RTENHIP_MBCONV=0); average duration per kernel name.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/mbexp; mkdir -p $O
for blk in ${BLOCKS:-3 8}; do
  for v in product 1 2 3 4 apart; do
    lib=""; env=""
    [ $v != product ] && [ $v != apart ] && lib=rten-fork_amd/exp_mb/librten_hip_mb$v.so
    [ $v = apart ] && env="RTENHIP_MBCONV=0"
    [ $v != apart ] && env="RTENHIP_MBCONV=all"
    env RTENHIP_LIB=$lib $env timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv \
      -- python3 rten-fork_amd/tools/mb_bench.py $blk > $O/${blk}_$v.log 2>&1 || { echo "mb $blk $v failed"; tail $O/${blk}_$v.log; exit 1; }
    f=$(find $O/$v -name 'run_kernel_stats.csv' | head -n 1)
    python3 -c "
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'rocclr' not in r['Name']]
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
print(sys.argv[2], sys.argv[3], ' | '.join('%s %s x%s %.1fus' % (r['Name'][9:40], '', r['Calls'], float(r['AverageNs']) / 1e3) for r in rows[:4]))
" "$f" $blk $v
    rm -rf $O/$v
  done
done
