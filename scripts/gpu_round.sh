#!/bin/bash
# One GPU session: the full check (suite, smoke, bench with secondaries),
# then the attention and LayerNorm timing experiments and the tile-order A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/gpu_check.sh "${1:-now}" && bash scripts/ab/gpu_attn.sh && bash scripts/ab/gpu_ln.sh
