set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; export RTEN_NUM_THREADS=8
O=gpurun_out/fcprobe; mkdir -p $O
for v in 0 91 92 41 21 11; do
  RTENHIP_LAT=$v timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --timing-report > $O/l$v.json 2> $O/l$v.txt || { tail $O/l$v.txt; exit 1; }
  echo "lat=$v $(grep -E 'op fc ' $O/l$v.txt)"
done
