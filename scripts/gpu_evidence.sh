#!/bin/bash
# Evidence at the current commit: rocprofv3 per-forward kernel summaries of
# the four bench configurations, PMC HBM traffic (FETCH_SIZE / WRITE_SIZE in
# separate passes) and the per-op timing reports of ResNet-50 b64 / b1.
# Output: gpurun_out/prof_$1 (copy the summaries into profiles/ with the commit).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
T=${1:-r4}
bash scripts/gpu_prof.sh $T resnet50_b64 resnet50_b1 mobilenet_v2_b128 bert_b32 || exit 1
bash scripts/gpu_prof.sh $T pmc_resnet50_64 pmc_bert_32 pmc_mobilenet_v2_128 || exit 1
O=gpurun_out/prof_$T
for cfg in "resnet50 64" "resnet50 1"; do
  set -- $cfg
  timeout -k 10 300 python -u rten-fork_amd/tools/model_once.py 1 $1 $2 --report > $O/report_$1_b$2.txt 2>&1 || { echo "report $1 $2 failed"; exit 1; }
done
echo evidence done
