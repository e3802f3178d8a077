#!/bin/bash
# Variant builds of the DMA GEMM for tuning experiments (never shipped):
# build_var.sh NAME "CONFIG LIST" [extra hipcc flags] -> var_NAME/librten_hip.so
set -e
cd "$(dirname "$0")"
NAME=$1; CFG=$2; shift 2
mkdir -p build/var_$NAME var_$NAME
for f in gemm_dma gemm_dma_p0 gemm_dma_p1 gemm_dma_p2 gemm_dma_p3; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -c csrc/$f.hip \
    -o build/var_$NAME/$f.o "-DRTENHIP_DMA_CONFIGS(X)=$CFG" "$@" &
done
wait
OBJS=$(ls build/*.o | grep -v gemm_dma)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o var_$NAME/librten_hip.so $OBJS build/var_$NAME/*.o
