set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/r6e; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_stem_pool_gpu.py > $O/t.log 2>&1; rc=$?
tail -12 $O/t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py -k "batch64_full_size" > $O/t2.log 2>&1 || { tail -20 $O/t2.log; exit 1; }
tail -1 $O/t2.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("head", d["value"], d["ms_per_step"], r["frac"], r.get("bytes_per_step"), r.get("traffic_ratio"))
for s in d.get("secondary", []):
    print("  ", s.get("metric", s), s.get("value"), s.get("ms_per_step"), (s.get("roofline") or {}).get("frac"),
          s.get("vs_device_resident", ""), s.get("error", ""))
PY
timeout -k 10 300 python -u rten-fork_amd/tools/model_once.py 1 resnet50 64 --report > $O/report_b64.txt 2>&1 || exit 1
grep -E "^op (conv1|maxpool)|stem" $O/report_b64.txt | head
