set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/r6n; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_conv_pointwise_gpu.py tests/test_full_size_gpu.py tests/test_stem_pool_gpu.py -k "stem or mobilenet" > $O/t.log 2>&1; rc=$?
tail -2 $O/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/t.log | head -20; exit 1; }
for v in 1 2; do
  for st in 1 0; do
    RTENHIP_STEM=$st timeout -k 10 300 python -u bench.py --model mobilenet_v2 --batch 128 --steps 30 --warmup 3 --no-secondary --no-cpu-baseline > $O/m_${st}_$v.json 2> $O/m_${st}_$v.err || { echo "bench failed"; tail $O/m_${st}_$v.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/m_${st}_$v.json').read().strip().splitlines()[-1]); print('stem $st round $v', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 300 python -u rten-fork_amd/tools/model_once.py 1 mobilenet_v2 128 --report > $O/report.txt 2>&1 || exit 1
grep -E "^op features\.0\." $O/report.txt
