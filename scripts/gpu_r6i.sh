set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/r6i; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py tests/test_full_size_gpu.py -k "pool or gemv or gemm or batch1" > $O/t.log 2>&1; rc=$?
tail -2 $O/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/t.log | head -20; exit 1; }
bash scripts/gpu_prof.sh r6c resnet50_b1 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
grep -E "gap|gemv|forward" gpurun_out/prof_r6c/resnet50_b1_per_forward.txt | head -5
bash scripts/gpu_r6f.sh || exit 1
