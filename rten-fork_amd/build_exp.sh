#!/bin/bash
# Timing-experiment builds of the DMA GEMM (never shipped): a reduced config
# list and RTENHIP_DMA_EXPERIMENT=$1, linked with the regular objects into
# exp$1/librten_hip.so.  usage: build_exp.sh MODE [CONFIG_LIST_MACRO]
set -e
cd "$(dirname "$0")"
MODE=$1
CFG=${2:-"X(0, 512, 128, 128, 16, 4, 2, 2, 3, 6) X(1, 256, 128, 128, 16, 2, 2, 2, 3, 6) X(2, 256, 64, 64, 16, 2, 2, 4, 3, 6) X(3, 256, 64, 64, 16, 2, 2, 4, 4, 6)"}
mkdir -p build/exp$MODE exp$MODE
for f in gemm_dma gemm_dma_p0 gemm_dma_p1 gemm_dma_p2 gemm_dma_p3; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -c csrc/$f.hip \
    -o build/exp$MODE/$f.o -DRTENHIP_DMA_EXPERIMENT=$MODE "-DRTENHIP_DMA_CONFIGS(X)=$CFG" &
done
wait
OBJS=$(ls build/*.o | grep -v gemm_dma)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o exp$MODE/librten_hip.so $OBJS build/exp$MODE/*.o
