set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/r6l; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_host_run_gpu.py -k "timing" > $O/t.log 2>&1; rc=$?
tail -2 $O/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/t.log | head -20; exit 1; }
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("head", d["value"], d["ms_per_step"], r["frac"], r["kernel_ms_per_step"], r["kernel_ms_eager_events"], r["capped"])
for s in d.get("secondary", []):
    rr = s.get("roofline") or {}
    print("  ", s.get("metric", s), s.get("value"), s.get("ms_per_step"), rr.get("frac"), rr.get("kernel_ms_eager_events"), rr.get("capped"), s.get("error", ""))
PY
