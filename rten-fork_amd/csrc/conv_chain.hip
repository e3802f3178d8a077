// Conv chain: the batch-1 ResNet-50 convs (layer1.0.conv1 .. layer4.2.conv3)
// as ONE persistent launch instead of one launch per conv.
//
// Why: at batch 1 a conv is 25..230 MFLOP, a few microseconds of MFMA on the
// whole chip, and its launch is dominated by fixed costs
// (profiles/r4_rocprof_resnet50_b1_per_forward.txt, gpurun_out stamps):
// ~0.5 us of dispatch spread, the weight panels' first-touch latency
// (~2.5 us from the Infinity Cache), the gathered activations behind them,
// the drain at the end of the kernel and ~1 us between kernels.  Weights do
// not depend on activations, so inside one launch a workgroup loads the next
// conv's weight panel BEFORE it waits for the current conv to finish; only
// the activation loads remain after the wait.
//
// Work: the chain's convs are grouped into phases (convs that do not depend
// on each other share one: a bottleneck's conv1 and its downsample), each
// phase a list of gemm_lat2 work items (RW x CW = 4 tiles of 16 x 16 outputs
// of one KC block per item, one fma chain per wave; A panels and B tiles
// staged in LDS).  Block o of the grid (XCD-contiguous remap of the block
// id) runs items o, o + G, ... of each phase.  K-split tiles fold their KC
// blocks in K order through the workspace exactly as gemm_lat2 does (last
// arriver folds, then bias / BN / residual / activation): the bits are those
// of the per-conv kernels, which are those of the reference
// (src/gemm.rs:733-1050, src/ops/conv.rs:24-68).
//
// Between phases: every block drains its stores and adds 1 to its shard of
// the arrival counter; one wave polls the 8 shards until each holds
// (phase + 1) x its block count; the block then proceeds.  Hand-off (MI355X
// guide, "Valid forms", row 1): every element another block reads is stored
// sc1 (write-through) and drained before the add; every load of such data
// (activations, residuals, split-K partials) is an sc1 / agent-atomic load
// after the poll and a workgroup barrier.  Weights, biases and BN tables are
// constants (plain loads, prefetched across the barrier).
//
// Progress: every block of the grid is resident (conv_chain_grid sizes the
// grid to the occupancy), so every arrival happens; each wait is bounded all
// the same -- a timeout sets the error word, which every later wait sees, so
// the launch drains in bounded time and the graph falls back to per-conv
// launches (Graph::build_chains checks the word).
#include <cstdlib>

#include "chain.h"
#include "lat_unit.h"

namespace rtenhip {

namespace {

typedef unsigned int chain_u32x4 __attribute__((ext_vector_type(4)));
constexpr int kLoadSc1 = 16;  // buffer-load cache policy bit: sc1 (L1 bypassed)
constexpr int kSpinLimit = 1 << 20;

struct ItemPos {
  int tn, tm, kb;
};
__device__ __forceinline__ ItemPos chain_item_pos(const ChainLayer& ly, int it) {
  ItemPos p;
  p.tn = it % ly.wg_n;
  const int t2 = it / ly.wg_n;
  p.tm = t2 % ly.wg_m;
  p.kb = t2 / ly.wg_m;
  return p;
}

// The item's RW packed A panels ([16 groups][64 lanes] float4 each): thread
// t loads float4 t + 256 (4r + q) of panel r (zero past M / K: the packing,
// and rows past M read past the buffer).  Always 16 loads, those past the
// layer's RW panels at an out-of-range offset (they return 0 without a
// memory access): one straight-line path, so the values stay in registers
// across the phase barrier.
__device__ __forceinline__ void chain_load_a(const ChainLayer& ly, const ItemPos& ip, chain_u32x4 (&av)[16]) {
  const DmaDesc& d = ly.d;
  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(
      (void*)d.apk, 0, (int)((int64_t)ly.subs * ly.nkb * LGROUPS * 64 * 16), 0x00020000);
  const int na = ly.rw * 4;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const int r = i >> 2, gl = (int)threadIdx.x + 256 * (i & 3);
    const int sub = ip.tm * ly.rw + r;
    const uint32_t off =
        (i < na && sub < ly.subs) ? (uint32_t)(((sub * ly.nkb + ip.kb) * LGROUPS * 64 + gl) * 16) : DMA_OOB;
    av[i] = __builtin_amdgcn_raw_buffer_load_b128(ar, off, 0, 0);
  }
}

// One work item (gemm_lat2_kernel's body with the chain's hand-off loads and
// stores): B gathered by all 256 threads with sc1 loads, A from av (loaded
// by the caller, possibly before the phase barrier), both staged in LDS; one
// chain per wave; fold and epilogue with sc1 stores.
// BVEC (pointwise stride-1 convs with P % 4 == 0, ChainLayer::bvec): B is
// copied 16 bytes per lane -- 4 adjacent columns of one k row, never across
// an image -- into a [CW][256 k][16 columns] LDS tile, and the chain reads
// its B operands from it one float per step (4x fewer global loads than the
// per-element gather).
// ist (timing experiments only, null otherwise): {start, operands in LDS,
// chain done, stored and drained} of this item, s_memrealtime.
template <int RW, bool BVEC>
__device__ __forceinline__ void chain_item(const ChainLayer& ly, const ItemPos& ip, float4* lds,
                                           const chain_u32x4 (&av)[16], unsigned long long* ist) {
  if (ist && threadIdx.x == 0) ist[0] = __builtin_amdgcn_s_memrealtime();
  constexpr int CW = 4 / RW;
  const DmaDesc& d = ly.d;
  float4(*lds_a)[LGROUPS][64] = reinterpret_cast<float4(*)[LGROUPS][64]>(lds);
  float4(*lds_b)[LGROUPS][64] = reinterpret_cast<float4(*)[LGROUPS][64]>(lds + RW * LGROUPS * 64);
  float* ldsk = reinterpret_cast<float*>(lds + RW * LGROUPS * 64);  // BVEC: [CW][LKC][16]
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int K = d.K;
  const int k0 = ip.kb * LKC;
  const int ng = min(LGROUPS, (K - k0 + 15) >> 4);
  const int wr = wave / CW, wc = wave - (wave / CW) * CW;
  const int sub0 = ip.tm * RW + wr;
  const int n0 = (ip.tn * CW + wc) * 16;

  // B: thread (wave w, lane (c, h)) gathers groups 4w..4w+3 of each of the CW
  // column tiles: k = k0 + 16g + 4j + h, column n0 + c (see gemm_lat2_kernel).
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)d.x, 0, (int)d.x_bytes, 0x00020000);
  const int h = lane >> 4;
  const bool linear = d.kstride > 0;
  uint32_t k3off[9];
  const uint32_t k3step = 16u * (uint32_t)d.kt_plane;
  if (!linear) {
    const uint32_t kh0 = (uint32_t)(k0 + h + 64 * wave);
    const int c0 = (int)(__umulhi(kh0, 0x38E38E39u) >> 1);
    const int r0 = (int)kh0 - 9 * c0;
#pragma unroll
    for (int s9 = 0; s9 < 9; s9++) {
      const int kk = r0 + 4 * s9;
      const int q = (kk * 57) >> 9;
      const int rr2 = kk - 9 * q;
      const int ky = (rr2 * 11) >> 5;
      const int kx = rr2 - 3 * ky;
      k3off[s9] = (uint32_t)((c0 + q) * d.kt_plane + ky * d.kt_row + kx * d.kt_col) * 4u;
    }
  }
  float bv[CW][4][4];
  chain_u32x4 bq[CW][4];
  const int q4 = threadIdx.x & 3, kr = threadIdx.x >> 2;  // BVEC: column quad, k row (+ 64 i)
  if constexpr (BVEC) {
#pragma unroll
    for (int cw = 0; cw < CW; cw++) {
      const int n = (ip.tn * CW + cw) * 16 + 4 * q4;
      uint32_t cb = DMA_OOB;
      if (n < d.N) {
        const int img = fdiv(n, d.fdP);
        cb = (uint32_t)(((int64_t)img * d.x_img + (n - img * d.P)) * 4);
      }
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int k = k0 + kr + 64 * i;
        const uint32_t off = (k < K && cb != DMA_OOB) ? cb + (uint32_t)k * (uint32_t)d.kstride * 4u : DMA_OOB;
        bq[cw][i] = __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, kLoadSc1);
      }
    }
  } else {
    uint32_t koff[16];
#pragma unroll
    for (int st = 0; st < 16; st++) {
      const int k = k0 + 64 * wave + 4 * st + h;
      const uint32_t lin = (uint32_t)k * (uint32_t)d.kstride * 4u;
      const uint32_t win = k3off[st % 9] + (uint32_t)(st / 9) * k3step;
      koff[st] = k < K ? (linear ? lin : win) : DMA_OOB;
    }
#pragma unroll
    for (int cw = 0; cw < CW; cw++) {
      const LatCol col = lat_col(d, (ip.tn * CW + cw) * 16);
#pragma unroll
      for (int gi = 0; gi < 4; gi++)
#pragma unroll
        for (int j = 0; j < 4; j++)
          bv[cw][gi][j] =
              __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, col.vcol + koff[4 * gi + j], 0, kLoadSc1));
    }
  }
  const bool live = sub0 < ly.subs && n0 < d.N;
  const LatCol col = lat_col(d, n0);
  LatEpi<1> e;
  if (live) lat_epi_loads<1, true>(d, sub0, col, e);
#pragma unroll
  for (int i = 0; i < RW * 4; i++) {
    const int idx = (int)threadIdx.x + 256 * i;
    lds_a[idx >> 10][(idx >> 6) & 15][idx & 63] =
        make_float4(__uint_as_float(av[i].x), __uint_as_float(av[i].y), __uint_as_float(av[i].z), __uint_as_float(av[i].w));
  }
  if constexpr (BVEC) {
#pragma unroll
    for (int cw = 0; cw < CW; cw++)
#pragma unroll
      for (int i = 0; i < 4; i++)
        *reinterpret_cast<float4*>(ldsk + (cw * LKC + kr + 64 * i) * 16 + 4 * q4) =
            make_float4(__uint_as_float(bq[cw][i].x), __uint_as_float(bq[cw][i].y), __uint_as_float(bq[cw][i].z),
                        __uint_as_float(bq[cw][i].w));
  } else {
#pragma unroll
    for (int cw = 0; cw < CW; cw++)
#pragma unroll
      for (int gi = 0; gi < 4; gi++)
        lds_b[cw][4 * wave + gi][lane] = make_float4(bv[cw][gi][0], bv[cw][gi][1], bv[cw][gi][2], bv[cw][gi][3]);
  }
  __syncthreads();
  if (ist && threadIdx.x == 0) ist[1] = __builtin_amdgcn_s_memrealtime();
  if (!live) return;

  lat_f32x4 acc[1];
  acc[0] = (lat_f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int g = 0; g < LGROUPS; g++) {
    if (g < ng) {
      const float4 a4 = lds_a[wr][g][lane];
      float4 b4;
      if constexpr (BVEC) {
        const float* bp = ldsk + (wc * LKC + 16 * g + h) * 16 + (lane & 15);
        b4 = make_float4(bp[0], bp[64], bp[128], bp[192]);  // k = 16g + 4j + h, j = 0..3
      } else {
        b4 = lds_b[wc][g][lane];
      }
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.x, b4.x, acc[0], 0, 0, 0);
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.y, b4.y, acc[0], 0, 0, 0);
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.z, b4.z, acc[0], 0, 0, 0);
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.w, b4.w, acc[0], 0, 0, 0);
    }
  }
  const int wt = sub0 * (ly.wg_n * CW) + (n0 >> 4);
  if (ist && threadIdx.x == 0) {
    asm volatile("" ::"v"(acc[0][0]), "v"(acc[0][3]));
    ist[2] = __builtin_amdgcn_s_memrealtime();
  }
  LatStamps stp;
  lat_fold_finish<1, true>(d, sub0, ip.kb, ly.nkb, wt, col, e, acc, stp);
  if (ist && threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ist[3] = __builtin_amdgcn_s_memrealtime();
  }
}

// Workgroup barrier that leaves global loads in flight (__syncthreads would
// wait for vmcnt(0)): LDS traffic and the compiler's memory order settle
// first.
__device__ __forceinline__ void chain_lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

}  // namespace

// Layer / phase tables through the constant address space (scalar loads).
#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(4))) const ChainLayer CLayer;
typedef __attribute__((address_space(4))) const ChainPhase CPhase;
#else
typedef const ChainLayer CLayer;
typedef const ChainPhase CPhase;
#endif

__global__ __launch_bounds__(256) void conv_chain_kernel(const ChainLayer* __restrict__ layers_g,
                                                         const ChainPhase* __restrict__ phases_g, int nph,
                                                         int* ctrl, unsigned long long* stamps) {
  __shared__ float4 lds[kChainPanels * LGROUPS * 64];  // 80 KB: two blocks per CU
  const CLayer* layers = (const CLayer*)layers_g;
  const CPhase* phases = (const CPhase*)phases_g;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int G = gridDim.x, bid = blockIdx.x;
  // XCD-contiguous remap (dispatch is round-robin over the 8 XCDs): the
  // items of one XCD are consecutive, so neighbours sharing an A panel meet
  // in its L2.  Placement is speed only; nothing below depends on it.
  const int qq = G >> 3, rr = G & 7, xcd = bid & 7;
  const int o = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int shard = bid & (kChainShards - 1);

  chain_u32x4 av[16];
  // have_a: av holds (or is loading) this block's first A of the phase,
  // issued before the phase barrier.
  bool have_a = false;
  if (nph > 0 && o < phases[0].items) {
    int L = phases[0].l0;
    while (o >= layers[L].item_base + layers[L].items) L++;
    const ChainLayer ly = layers[L];
    chain_load_a(ly, chain_item_pos(ly, o - ly.item_base), av);
    have_a = true;
  }
  for (int ph = 0; ph < nph; ph++) {
    const ChainPhase P = phases[ph];
    bool first = true;
    for (int i = o; i < P.items; i += G) {
      int L = P.l0;
      while (i >= layers[L].item_base + layers[L].items) L++;
      const ChainLayer ly = layers[L];
      const ItemPos ip = chain_item_pos(ly, i - ly.item_base);
      if (!(first && have_a)) chain_load_a(ly, ip, av);
      if (!first) chain_lds_barrier();  // the previous item's chains are done with LDS
      first = false;
      // (timing experiments: the first item of the phase is stamped)
      unsigned long long* ist =
          stamps && i == o ? stamps + 2 * (size_t)G * nph + 4 * ((size_t)bid * nph + ph) : nullptr;
      if (ly.bvec) {
        if (ly.rw == 1) chain_item<1, true>(ly, ip, lds, av, ist);
        else if (ly.rw == 2) chain_item<2, true>(ly, ip, lds, av, ist);
        else chain_item<4, true>(ly, ip, lds, av, ist);
      } else {
        if (ly.rw == 1) chain_item<1, false>(ly, ip, lds, av, ist);
        else if (ly.rw == 2) chain_item<2, false>(ly, ip, lds, av, ist);
        else chain_item<4, false>(ly, ip, lds, av, ist);
      }
    }
    have_a = false;
    if (ph + 1 == nph) break;
    // Every store of this block is drained before its arrival (each wave
    // waits for its own stores; the barrier orders the add after all four).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // The next phase's weights (constants) stay in flight across the barrier.
    const ChainPhase Pn = phases[ph + 1];
    if (o < Pn.items) {
      int L = Pn.l0;
      while (o >= layers[L].item_base + layers[L].items) L++;
      const ChainLayer ly = layers[L];
      chain_load_a(ly, chain_item_pos(ly, o - ly.item_base), av);
      have_a = true;
    }
    chain_lds_barrier();
    unsigned long long t_arrive = 0;
    if (threadIdx.x == 0) {
      if (stamps) t_arrive = __builtin_amdgcn_s_memrealtime();
      __hip_atomic_fetch_add(ctrl + shard * kChainShardStride, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (wave == 0) {
      // Lane s < 8 polls shard s until it holds (ph + 1) x its block count.
      const int cnt = lane < kChainShards ? (G / kChainShards + (lane < G % kChainShards ? 1 : 0)) * (ph + 1) : 0;
      const int* wp = ctrl + (lane < kChainShards ? lane : 0) * kChainShardStride;
      bool failed = false;
      int spins = 0;
      while (true) {
        const int v = lane < kChainShards ? __hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : cnt;
        const int err = __hip_atomic_load(ctrl + chain_error_index(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__builtin_amdgcn_ballot_w64(v < cnt) == 0) break;
        if (__builtin_amdgcn_readfirstlane(err) || ++spins > kSpinLimit) {
          if (lane == 0 && !err)
            __hip_atomic_store(ctrl + chain_error_index(), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          failed = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      (void)failed;  // every later wait sees the error word: the launch drains in bounded time
      if (stamps && lane == 0) {
        unsigned long long* sp = stamps + 2 * ((size_t)bid * nph + ph);
        sp[0] = t_arrive;
        sp[1] = __builtin_amdgcn_s_memrealtime();
      }
    }
    chain_lds_barrier();
  }
  // Exit: the last block re-zeroes the control words for the next launch.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int prev =
        __hip_atomic_fetch_add(ctrl + chain_exit_index(), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == G - 1) {
      const int err = __hip_atomic_load(ctrl + chain_error_index(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int s = 0; s < kChainShards; s++)
        __hip_atomic_store(ctrl + s * kChainShardStride, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctrl + chain_exit_index(), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // The error word stays set for the host to read (it re-zeroes it).
      (void)err;
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
    static const int per_cu = getenv("RTENHIP_CHAIN_PER_CU") ? atoi(getenv("RTENHIP_CHAIN_PER_CU")) : 2;
    grid = cus * std::max(1, std::min(occ, per_cu));
  }
  return grid;
}

rtenhip_status launch_conv_chain(const ChainLayer* layers_dev, const ChainPhase* phases_dev, int n_phases, int* ctrl,
                                 int grid, hipStream_t s, unsigned long long* stamps) {
  if (n_phases <= 0) return RTENHIP_OK;
  if (grid <= 0) return fail(RTENHIP_INVALID_VALUE, "conv chain: empty grid");
  hipLaunchKernelGGL(conv_chain_kernel, dim3((unsigned)grid), dim3(256), 0, s, layers_dev, phases_dev, n_phases, ctrl,
                     stamps);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

}  // namespace rtenhip
