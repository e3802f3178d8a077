set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/r6c; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_host_run_gpu.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("head", d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"].get("hold_timeouts"))
for s in d.get("secondary", []):
    print("  ", s.get("metric", s), s.get("value"), s.get("ms_per_step"), (s.get("roofline") or {}).get("frac"),
          s.get("vs_device_resident", ""), s.get("error", ""), (s.get("cpu_baseline") or {}).get("value"))
print("cpu", d["cpu_baseline"]["value"])
PY
