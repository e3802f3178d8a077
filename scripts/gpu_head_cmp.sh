#!/bin/bash
# Kernel-traced convbench: HEAD variants (var_h2/h4/h6, configs d0..d3) and the
# shipped build (d7 = 64x64 3-stage, d14 = 64x64 4-stage) on ResNet-50 shapes.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
LIBS="h2 h4 h6" CFGS=d0,d1,d2,d3 bash scripts/gpu_var.sh || exit 1
mkdir -p rten-fork_amd/var_base && cp rten-fork_amd/librten_hip.so rten-fork_amd/var_base/
LIBS="base" CFGS=d7,d14 bash scripts/gpu_var.sh || exit 1
