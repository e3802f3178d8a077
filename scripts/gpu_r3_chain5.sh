#!/bin/bash
# Chain with region dependencies: bit-exact tests, then the timeline and the
# b1 bench (forced and auto).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out/p8
O=gpurun_out/p8
export RTEN_NUM_THREADS=8
PYT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_conv_lat_gpu.py -k "chain" > $O/chain_tests.log 2>&1 \
  || { echo "chain tests failed"; tail -40 $O/chain_tests.log; exit 1; }
tail -3 $O/chain_tests.log
RTENHIP_CHAIN=1 RTENHIP_CHAIN_STAMPS=$O/st timeout -k 10 200 python -u bench.py --batch 1 --steps 3 --warmup 2 --no-cpu-baseline --timing-report > $O/st.json 2> $O/st.err || { tail $O/st.err; exit 1; }
for c in 0 1 2 3; do [ -f $O/st.$c ] && python3 rten-fork_amd/tools/chain_stamps.py $O/st.$c | head -4; done
timeout -k 10 200 python -u bench.py --batch 1 --steps 50 --no-cpu-baseline --timing-report > $O/b1.json 2> $O/b1.err || { tail $O/b1.err; exit 1; }
cat $O/b1.json; grep "conv chain" $O/b1.err
