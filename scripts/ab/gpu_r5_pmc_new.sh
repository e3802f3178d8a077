#!/bin/bash
# PMC of round 5's new ResNet-50 b64 kernels (the stem and the conv pair) in the
# whole forward: one SQ pass, FETCH_SIZE and WRITE_SIZE passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/gpu_kern_pmc.sh stem conv_stem rten-fork_amd/tools/model_once.py 2 resnet50 64 > gpurun_out/r5pmc_stem.txt 2>&1 || { tail -5 gpurun_out/r5pmc_stem.txt; exit 1; }
rm -rf gpurun_out/kpmc_stem/pmc* gpurun_out/kpmc_stem/kt
bash scripts/gpu_kern_pmc.sh pair2 conv_pair rten-fork_amd/tools/model_once.py 2 resnet50 64 > gpurun_out/r5pmc_pair.txt 2>&1 || { tail -5 gpurun_out/r5pmc_pair.txt; exit 1; }
rm -rf gpurun_out/kpmc_pair2/pmc* gpurun_out/kpmc_pair2/kt
cat gpurun_out/r5pmc_stem.txt gpurun_out/r5pmc_pair.txt
