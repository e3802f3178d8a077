set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/r6a; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_host_run_gpu.py tests/test_parallel_gpu.py > $O/t1.log 2>&1; rc=$?
tail -15 $O/t1.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_lat_gpu.py tests/test_full_size_gpu.py -k "batch1 or lat" > $O/t2.log 2>&1 || { tail -30 $O/t2.log; exit 1; }
tail -2 $O/t2.log
