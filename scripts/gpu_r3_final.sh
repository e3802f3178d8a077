#!/bin/bash
# End-of-session check: the whole GPU suite, the full-size configs, smoke(),
# and the bench lines (ResNet-50 b64 / b1, MobileNetV2 b128, BERT b32).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
export RTEN_NUM_THREADS=8
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $PYT tests -m gpu > $O/suite.log 2>&1 || { echo "gpu suite failed"; tail -40 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
b() {  # name, args
  local n=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n', d['value'], d['ms_per_step'], d['roofline']['frac'])"
}
b resnet50_b64
b resnet50_b1 --batch 1 --steps 100 --no-cpu-baseline
b mobilenet_v2_b128 --model mobilenet_v2 --batch 128 --no-cpu-baseline
b bert_b32 --model bert --batch 32 --no-cpu-baseline
