#!/bin/bash
# GPU session after kernel changes: the new parity tests first, then the whole
# -m gpu suite without stopping at the first failure, smoke(), the bench line
# (headline + secondaries).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/suite_${1:-now}; mkdir -p $O
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $PYT -x tests/test_vecmath_gpu.py tests/test_chain_gpu.py > $O/new.log 2>&1; rc=$?
tail -3 $O/new.log; grep -E "FAILED|Error" $O/new.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "new tests aborted rc=$rc"; exit 1; }
timeout -k 10 900 $PYT tests -m gpu > $O/suite.log 2>&1; rc=$?
tail -2 $O/suite.log; grep -E "^FAILED" $O/suite.log | head -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "suite aborted rc=$rc"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("head", d["metric"], d["value"], d["ms_per_step"], d["roofline"]["frac"])
for s in d.get("secondary", []):
    print("  ", s.get("metric", s), s.get("value"), s.get("ms_per_step"), (s.get("roofline") or {}).get("frac"), s.get("error", ""))
PY
