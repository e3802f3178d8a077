// Conv chain: consecutive small-batch convs of a plan (ResNet-50 at batch 1:
// layer1.0.conv1 .. layer4.2.conv3) as ONE persistent launch of latency-GEMM
// units (lat_unit.h), instead of one launch per conv.
//
// Why: at batch 1 every conv is a few microseconds of work, and each launch
// costs its ramp-up and drain (~3 us for an empty kernel, profiles/) plus the
// gap to the next dispatch; 52 of them are most of the forward.  In the chain
// a layer's units start as soon as the layers they depend on have completed,
// with their weight loads already issued while they wait.
//
// Work: the layers' units (16x16 output tile x KC block) in layer order form
// one list; wave w of the grid runs units w, w + W, w + 2W, ... in order (no
// queue atomics).  Before reading its input a unit waits (chain.h,
// ChainLayer) for the producer tiles under its window -- the input rows its
// 16 output columns read, the same columns of the residual -- and for whole
// earlier layers that used the storage it overwrites, by polling completion
// counters.  Progress: every dependency of a unit lies earlier in the list,
// so the lowest incomplete unit only waits on complete ones and its wave,
// which runs its units in list order, is at it -- provided every wave of the
// grid is resident, which the grid size guarantees (conv_chain_grid: at most
// the occupancy the kernel's registers allow).
// Spins are bounded; a timed-out wait sets the error word (checked by the
// graph after its eager runs).
//
// Hand-off (MI355X guide: per-XCD L2s are not coherent; the form used is the
// "valid forms" row 1): every output element is stored sc1 (write-through),
// the storing wave drains its stores (s_waitcnt vmcnt(0)) and one lane adds
// 1 to the layer's counter shard (agent-scope atomic); the consumer polls the
// shards with sc1 loads and reads the handed-off activations (x, residual)
// only with sc1 loads.  The split-K chains use 8-byte agent atomics on both
// sides (lat_unit.h).
#include <cstdlib>

#include "chain.h"
#include "lat_unit.h"

namespace rtenhip {

// Layer descriptors through the constant address space (scalar loads); the
// host pass only parses the kernel.
#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(4))) const ChainLayer CLayer;
#else
typedef const ChainLayer CLayer;
#endif

__global__ __launch_bounds__(256) void conv_chain_kernel(const ChainLayer* __restrict__ layers_g, int nl, int total,
                                                         int* ctrl, int dbg, unsigned long long* stamps) {
  __shared__ uint32_t ktl[4][LKC];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const CLayer* layers = (const CLayer*)layers_g;
  const int W = gridDim.x * 4;
  int L = 0;
  for (int i = blockIdx.x * 4 + wave; i < total; i += W) {
    while (i >= layers[L].item_base + layers[L].items) L++;
    const CLayer& ly = layers[L];
    const int u = i - ly.item_base;
    const int n16 = ly.n16, subs = ly.subs, nkb = ly.nkb;
    const int kb = u % nkb;
    const int r = u / nkb;
    const int ms = r % subs;
    const int nt = r / subs;
    const int wt = ms * n16 + nt;
    const DmaDesc d = ly.d;
    unsigned long long t0 = 0, t1 = 0;
    if (stamps) t0 = __builtin_amdgcn_s_memrealtime();
    bool timed_out = false;
    // Polls back off (64 .. 1024 cycles between them): a few thousand waves
    // polling flat out would take the memory system from the waves they wait
    // for.  `ready` is evaluated by the whole wave and must be uniform.
    auto poll = [&](auto ready) __attribute__((always_inline)) {
      int nap = 1;
      for (int spin = 0; !timed_out; spin++) {
        if (ready()) break;
        if (spin > (1 << 18)) {
          if (lane == 0) __hip_atomic_store(ctrl + chain_error_index(nl), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          timed_out = true;
          break;
        }
        if (nap == 1) __builtin_amdgcn_s_sleep(1);
        else if (nap == 2) __builtin_amdgcn_s_sleep(2);
        else if (nap == 4) __builtin_amdgcn_s_sleep(4);
        else if (nap == 8) __builtin_amdgcn_s_sleep(8);
        else __builtin_amdgcn_s_sleep(16);
        nap = nap < 16 ? nap * 2 : 16;
      }
    };
    // Column tiles t0c..t1c of layer j complete: one counter per lane, 64 a round.
    auto wait_tiles = [&](int j, int t0c, int t1c) __attribute__((always_inline)) {
      const int need = layers[j].subs;
      const int* cnt = ctrl + layers[j].cnt_base;
      for (int b = t0c; b <= t1c; b += 64) {
        const int t = b + lane;
        poll([&]() {
          const int v = t <= t1c ? __hip_atomic_load(cnt + (int64_t)t * kChainTileStride, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT)
                                 : need;
          return __builtin_amdgcn_ballot_w64(v < need) == 0;
        });
      }
    };
    auto wait = [&]() __attribute__((always_inline)) {
      // Layer dependencies (storage reuse).
      const int nd = ly.ndeps;
      for (int k = 0; k < nd; k++) {
        const int j = ly.deps[k];
        const int need = min(layers[j].tiles, kChainShards);  // non-empty shards
        const int* cnt = ctrl + chain_layer_index(j) + ((blockIdx.x * 4 + wave) % kChainReplicas) * kChainShardStride;
        poll([&]() {
          return __builtin_amdgcn_readfirstlane(__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >=
                 need;
        });
      }
      // Region dependencies: this unit's output columns p0..p1 (global n).
      const int p0 = nt * 16, p1 = min(d.N - 1, p0 + 15);
      if (ly.dep_r >= 0) wait_tiles(ly.dep_r, p0 >> 4, p1 >> 4);
      if (ly.dep_x >= 0) {
        const int P = ly.P, OW = ly.OW;
        const int img0 = p0 / P, img1 = p1 / P;
        for (int img = img0; img <= img1; img++) {
          const int q0 = img == img0 ? p0 - img * P : 0;
          const int q1 = img == img1 ? p1 - img * P : P - 1;
          const int iy0 = max(0, (q0 / OW) * ly.S - ly.pt);
          const int iy1 = min(ly.in_H - 1, (q1 / OW) * ly.S - ly.pt + ly.kext - 1);
          if (iy1 < iy0) continue;
          const int a = img * ly.in_P + iy0 * ly.in_W, b = img * ly.in_P + (iy1 + 1) * ly.in_W - 1;
          wait_tiles(ly.dep_x, a >> 4, b >> 4);
        }
      }
      if (stamps) t1 = __builtin_amdgcn_s_memrealtime();
    };
    // Tile done: count it for its column tile (region consumers) and, when a
    // later layer waits for the whole layer, in its shard; the wave that
    // fills the shard counts the shard in the layer word.
    auto done = [&]() __attribute__((always_inline)) {
      if (lane == 0)
        __hip_atomic_fetch_add(ctrl + ly.cnt_base + (int64_t)nt * kChainTileStride, 1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      if (ly.layer_word) {
        const int tiles = ly.tiles;
        const int sh = wt & (kChainShards - 1);
        const int quota = tiles / kChainShards + (sh < tiles % kChainShards ? 1 : 0);
        int prev = 0;
        if (lane == 0)
          prev = __hip_atomic_fetch_add(ctrl + chain_done_index(L) + sh * kChainShardStride, 1, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
        prev = __builtin_amdgcn_readfirstlane(prev);
        if (prev + 1 == quota && lane < kChainReplicas)
          __hip_atomic_fetch_add(ctrl + chain_layer_index(L) + lane * kChainShardStride, 1, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
      }
    };
    lat_unit<1, true>(d, ms, nt * 16, kb, nkb, subs, wt, ktl[wave], wait, done, dbg);
    if (stamps && lane == 0) {
      // timing experiments: {layer | xcc << 8 | block << 16, start, waited, end}
      const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
      const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20) & 15;
      stamps[4 * (size_t)i] = (unsigned long long)L | ((unsigned long long)xcc << 8) | ((unsigned long long)blockIdx.x << 16);
      stamps[4 * (size_t)i + 1] = t0;
      stamps[4 * (size_t)i + 2] = t1;
      stamps[4 * (size_t)i + 3] = t2;
    }
  }
}

int conv_chain_grid() {
  static int grid = 0;
  if (grid == 0) {
    int dev = 0, cus = 0, occ = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, conv_chain_kernel, 256, 0) != hipSuccess || occ <= 0)
      occ = 1;
    // At most 2 workgroups per CU, and one below the occupancy query when it
    // allows more than 2 (it can over-report by one block per CU).
    const int k = occ >= 3 ? 2 : (occ == 2 ? 2 : 1);
    grid = cus * k;
  }
  return grid;
}

rtenhip_status launch_conv_chain(const ChainLayer* layers_dev, int n_layers, int total_items, int* ctrl, int grid,
                                 hipStream_t s, unsigned long long* stamps) {
  if (n_layers <= 0 || total_items <= 0) return RTENHIP_OK;
  if (grid <= 0) return fail(RTENHIP_INVALID_VALUE, "conv chain: empty grid");
  static const int dbg = [] {
    const char* e = getenv("RTENHIP_CHAIN_DBG");  // timing experiments only
    return e ? atoi(e) : 0;
  }();
  hipLaunchKernelGGL(conv_chain_kernel, dim3((unsigned)grid), dim3(256), 0, s, layers_dev, n_layers, total_items,
                     ctrl, dbg, stamps);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

}  // namespace rtenhip
