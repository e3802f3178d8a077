#!/bin/bash
# The driver's bench line (bench.py, N = 1, secondaries included), summarised.
# Usage: scripts/gpu_bench.sh [tag] [bench args...]   (output gpurun_out/bench_<tag>)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
T=${1:-now}; shift
O=gpurun_out/bench_$T; mkdir -p $O
timeout -k 10 600 python -u bench.py "$@" > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("head", d["value"], d["ms_per_step"], r["frac"], "rocprof", (r.get("rocprof") or {}).get("frac"), "ratio", r.get("traffic_ratio"))
for s in d.get("secondary", []):
    rr = s.get("roofline") or {}
    print("  ", s.get("metric", s), s.get("value"), s.get("ms_per_step"), rr.get("frac"), s.get("vs_device_resident", ""),
          (s.get("cpu_baseline") or {}).get("value", ""), s.get("error", ""))
if "cpu_baseline" in d: print("  cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["cores"])
PY
