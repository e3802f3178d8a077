#!/bin/bash
# ResNet-50 b64 dual A/B with the per-op report, then the BERT packed-A A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/big; mkdir -p $O
export RTEN_NUM_THREADS=8
for i in 1 2; do
  for v in "dual:RTENHIP_X=1" "nodual:RTENHIP_NO_DUAL=1"; do
    name=${v%%:*}
    env ${v#*:} timeout -k 10 300 python -u bench.py --no-cpu-baseline --timing-report > $O/${name}_$i.json 2> $O/${name}_$i.txt || { tail $O/${name}_$i.txt; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${name}_$i.json'));r=d['roofline'];print('$name', d['value'], d['ms_per_step'], r['frac'], r['kernel_ms_per_step'])"
  done
done
grep -E "dual|downsample|conv3" $O/dual_1.txt | head -24
bash scripts/gpu_r3_bert_ab.sh
