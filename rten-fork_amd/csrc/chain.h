// Conv chain (conv_chain.hip): a run of consecutive small-batch convs of a
// plan (ResNet-50 at batch 1: layer1.0.conv1 .. layer4.2.conv3, 52 convs)
// executed by ONE persistent launch instead of one launch per conv.
#pragma once

#include "gemm_dma.h"

namespace rtenhip {

constexpr int kChainShards = 8;        // phase-arrival counter shards (block id & 7)
constexpr int kChainShardStride = 32;  // ints between shards: one 128-byte line each
constexpr int kChainPanels = 5;        // LDS panels per workgroup: RW A panels + CW B tiles (RW + CW <= 5)

// One conv of the chain: its latency-GEMM descriptor (lat-packed weights,
// gemm_lat2's RW x CW tiles of one KC block per work item) and its items.
struct ChainLayer {
  DmaDesc d;
  int rw, cw;            // rw * cw == 4: one 16x16 chain per wave
  int bvec;              // pointwise stride-1, P % 4 == 0: 16-byte B copies (conv_chain.hip chain_item)
  int wg_m, wg_n, nkb, subs;
  int items;             // wg_m * wg_n * nkb, ordered (kb, tm, tn), tn fastest
  int item_base;         // first item of the layer within its phase
};

// Convs with no dependency among them (a bottleneck's conv1 and its
// downsample read the same input): their items form one list, and the
// launch crosses a grid-wide arrival barrier between phases.
struct ChainPhase {
  int l0, nl, items;
};

// Control words (int32): kChainShards phase-arrival counters, each on its own
// line (monotonic within a launch: shard s reaches (p + 1) * blocks_in(s)
// once every block of shard s finished phase p), the error word (a wait
// timed out), and the exit counter (the last block to leave re-zeroes every
// word, so a launch needs no memset before it).
__host__ __device__ inline int chain_error_index() { return kChainShards * kChainShardStride; }
__host__ __device__ inline int chain_exit_index() { return (kChainShards + 1) * kChainShardStride; }
constexpr int kChainCtrlInts = (kChainShards + 2) * kChainShardStride;

// Resident workgroups of the persistent grid (every one must be resident at
// once: the barrier waits for all of them): CUs x blocks per CU.
int conv_chain_grid();
// stamps (timing experiments, RTENHIP_CHAIN_STAMPS): per block and phase
// {arrive, released} s_memrealtime pairs.
rtenhip_status launch_conv_chain(const ChainLayer* layers_dev, const ChainPhase* phases_dev, int n_phases,
                                 int* ctrl, int grid, hipStream_t s, unsigned long long* stamps = nullptr);

}  // namespace rtenhip
