set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/r6g; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_head_fusions_gpu.py tests/test_full_size_gpu.py -k "head or pool or batch1" > $O/t.log 2>&1; rc=$?
tail -3 $O/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/t.log | head -20; exit 1; }
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
timeout -k 10 300 python -u rten-fork_amd/tools/model_once.py 1 resnet50 1 --report > $O/report_b1.txt 2>&1 || exit 1
grep -E "^op (conv1|maxpool|fc|avgpool)" $O/report_b1.txt | head
