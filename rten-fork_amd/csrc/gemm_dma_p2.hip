// Part 2 of the LDS-DMA GEMM's tile configurations (cfg % DMA_PARTS == 2),
// compiled on its own so the configurations build in parallel.
#include "gemm_dma_kernel.h"

namespace rtenhip {
template bool dma_launch_part<2>(int, const DmaDesc&, hipStream_t, const DmaDesc*);
}  // namespace rtenhip
