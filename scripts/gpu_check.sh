#!/bin/bash
# GPU check of the current tree: the whole -m gpu suite, smoke(), and the
# driver's bench command (headline ResNet-50 b64 + the secondary configs).
# Usage: scripts/gpu_check.sh [tag]   (outputs under gpurun_out/check_<tag>)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/check_${1:-now}; mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
if [ -z "$NO_SUITE" ]; then
  timeout -k 10 900 $PYT tests -m gpu > $O/suite.log 2>&1 || { echo "gpu suite failed"; tail -40 $O/suite.log; exit 1; }
  tail -1 $O/suite.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("head", d["metric"], d["value"], d["ms_per_step"], d["roofline"]["frac"])
r = d["roofline"]; print("   roofline capped", r.get("capped"), "eager", r.get("kernel_ms_eager_events"), "rocprof", r.get("rocprof"))
for s in d.get("secondary", []):
    print("  ", s.get("metric", s), s.get("value"), s.get("ms_per_step"), (s.get("roofline") or {}).get("frac"),
          (s.get("roofline") or {}).get("capped"), (s.get("roofline") or {}).get("kernel_ms_eager_events"),
          s.get("pcie", ""), s.get("vs_device_resident", ""), s.get("error", ""))
if "cpu_baseline" in d: print("  cpu", d["cpu_baseline"]["value"], d["cpu_baseline"].get("gemm_gflops_per_core"),
                              d["cpu_baseline"].get("gemm_gflops_all_threads"), d["cpu_baseline"].get("topology"))
PY
