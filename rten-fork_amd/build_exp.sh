#!/bin/bash
# Timing-experiment builds of the DMA GEMM (never shipped): a reduced config
# list and RTENHIP_DMA_EXPERIMENT=$1, linked with the regular objects into
# build/exp$1/librten_hip.so.  usage: build_exp.sh MODE [CONFIG_LIST_MACRO]
set -e
cd "$(dirname "$0")"
MODE=$1
CFG=${2:-"X(0, 512, 128, 128, 16, 4, 2, 2, 3) X(1, 256, 128, 128, 16, 2, 2, 2, 3) X(2, 256, 64, 64, 16, 2, 2, 4, 3) X(3, 256, 64, 64, 16, 2, 2, 4, 4)"}
mkdir -p build/exp$MODE exp$MODE
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -c csrc/gemm_dma.hip \
  -o build/exp$MODE/gemm_dma.o -DRTENHIP_DMA_EXPERIMENT=$MODE "-DRTENHIP_DMA_CONFIGS(X)=$CFG"
OBJS=$(ls build/*.o | grep -v gemm_dma.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o exp$MODE/librten_hip.so $OBJS build/exp$MODE/gemm_dma.o
