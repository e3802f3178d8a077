// Conv chain (conv_chain.hip): a run of consecutive small-batch convs of a
// plan executed by ONE persistent launch of latency-GEMM units.
#pragma once

#include "gemm_dma.h"

namespace rtenhip {

constexpr int kChainMaxDeps = 8;
constexpr int kChainShards = 64;       // tile-completion counter shards per layer
constexpr int kChainShardStride = 32;  // ints between shards: one 128-byte line each
constexpr int kChainReplicas = 32;     // copies of the layer word (pollers spread over them)
constexpr int kChainTileStride = 16;   // ints between column-tile counters (64 bytes)

// One conv of the chain: its latency-GEMM descriptor (lat-packed weights,
// MI = 1 units) and what its units wait for.
//   - Region dependencies (read-after-write): dep_x / dep_r, the chain layers
//     producing this conv's input / fused residual.  A unit waits only for
//     the producer's 16-column tiles its output columns read -- the input
//     rows under its kext-row window, or the same columns of the residual --
//     so consecutive layers overlap like a wavefront.
//   - Layer dependencies (deps): earlier layers that read or write the
//     storage this conv overwrites (outputs kept in shared arena storage);
//     a unit waits for those layers to complete.
struct ChainLayer {
  DmaDesc d;
  int nkb, subs, n16;
  int tiles;       // output tiles (subs * n16)
  int items;       // units = tiles * nkb, ordered (column tile, row tile, K block), K block fastest
  int item_base;   // first global item of the layer
  int ndeps;
  int deps[kChainMaxDeps];
  int dep_x, dep_r;      // producing chain layers (-1: produced before the launch)
  int in_H, in_W, in_P;  // this conv's (unpadded) input plane = dep_x's output plane
  int S, pt, kext;       // vertical stride, top pad, (kh - 1) * dh + 1
  int OW, P;             // this conv's output row and plane
  int cnt_base;          // its column-tile counters (ints into ctrl, kChainTileStride apart)
  int layer_word;        // some later layer polls this layer's completion word
};

// Control words (int32, zeroed before every launch).  Per layer, each on its
// own 128-byte line: kChainShards tile-completion counters (tile t counts
// into shard t % kChainShards) and kChainReplicas copies of a
// shard-completion counter (the wave whose add fills a shard adds 1 to every
// copy with one instruction; the layer is complete when a copy reaches its
// non-empty shard count -- one word to poll, the pollers spread over the
// copies).  Then one error word (a dependency wait timed out), the split-K
// arrival counters of all layers (d.counters point there) and the
// column-tile counters (ChainLayer::cnt_base: completed row tiles per
// 16-column tile).
__host__ __device__ inline int64_t chain_done_index(int layer) {
  return (int64_t)layer * (kChainShards + kChainReplicas) * kChainShardStride;
}
__host__ __device__ inline int64_t chain_layer_index(int layer) {
  return chain_done_index(layer) + (int64_t)kChainShards * kChainShardStride;
}
__host__ __device__ inline int64_t chain_error_index(int layers) { return chain_done_index(layers); }
__host__ __device__ inline int64_t chain_counters_base(int layers) { return chain_done_index(layers) + 32; }

// Persistent grid: resident workgroups of 4 waves; wave w runs items w,
// w + W, ... (W = 4 * grid) in order.  Every wave of the grid must be
// resident (see launch_conv_chain).
int conv_chain_grid();
// stamps (timing experiments, RTENHIP_CHAIN_STAMPS): 4 u64 per unit.
rtenhip_status launch_conv_chain(const ChainLayer* layers_dev, int n_layers, int total_items, int* ctrl,
                                 int grid, hipStream_t s, unsigned long long* stamps = nullptr);

}  // namespace rtenhip
