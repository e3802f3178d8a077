#!/bin/bash
# Timing-experiment builds of the VALU conv kernels (never shipped):
# RTENHIP_PW_EXPERIMENT=$1, linked with the regular objects into
# pwexp$1/librten_hip.so.  usage: build_pw_exp.sh MODE
set -e
cd "$(dirname "$0")"
MODE=$1
mkdir -p build/pwexp$MODE pwexp$MODE
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -c csrc/conv_pointwise.hip \
  -o build/pwexp$MODE/conv_pointwise.o -DRTENHIP_PW_EXPERIMENT=$MODE
OBJS=$(ls build/*.o | grep -v conv_pointwise)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o pwexp$MODE/librten_hip.so $OBJS build/pwexp$MODE/*.o
