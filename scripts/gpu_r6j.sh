set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/r6j; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_full_size_gpu.py tests/test_model_gpu.py -k "full_size" > $O/t.log 2>&1; rc=$?
tail -2 $O/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/t.log | head -20; exit 1; }
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("head", d["value"], d["ms_per_step"], r["frac"])
for s in d.get("secondary", []):
    print("  ", s.get("metric", s), s.get("value"), s.get("ms_per_step"), (s.get("roofline") or {}).get("frac"),
          s.get("vs_device_resident", ""), s.get("error", ""))
PY
timeout -k 10 300 python -u rten-fork_amd/tools/model_once.py 1 resnet50 64 --report > $O/report_b64.txt 2>&1 || exit 1
grep -c "split4" $O/report_b64.txt
