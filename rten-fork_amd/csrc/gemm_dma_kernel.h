// Kernel template and launch helpers of the LDS-DMA GEMM, included by
// gemm_dma.hip (host side) and the gemm_dma_p*.hip parts that instantiate
// the tile configurations (split for parallel builds).
#pragma once
// f32 MFMA GEMM with LDS-DMA staging for gfx950 — the fast path of the
// implicit-GEMM engine (see gemm_mfma.hip for the general kernel and the
// summation-order contract it shares: KC = 256 blocks, fma chains from +0,
// bias after block 0, src/gemm.rs:733-1050).
//
// Why a second kernel: v_mfma_f32_32x32x2_f32 issues at the f32 VALU rate and
// PMC counters show it never co-executes with VALU instructions
// (SQ_VALU_MFMA_COEXEC_CYCLES = 0), so every address/bounds instruction of a
// register-staged im2col gather is taken straight out of MFMA time.  This
// kernel issues NO per-element VALU work in its K loop:
//   - A (weights) is pre-packed once into [tiles_m][tiles_k][BK][BM] tiles
//     (zero padded), copied into LDS by buffer_load_dwordx4 ... lds;
//   - B is gathered with buffer_load_dword ... lds where each lane's VGPR
//     offset (its output pixel's input corner) is fixed for the whole kernel
//     and the k-dependent part is a scalar offset from a per-k table.  This
//     is exact for convolutions whose input needs no bounds checks: pointwise
//     and unpadded strided convs, and padded convs whose input the graph
//     executor materialised with its zero border.  Out-of-range n / k are
//     pushed past the buffer's num_records and read as 0 by the hardware.
#include <type_traits>

#include "common.h"
#include "gemm_dma.h"
#include "fastdiv_dev.h"
#include "packed_a.h"
#include "vecmath.h"

namespace rtenhip {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void_t;
// Constant address space: uniform loads through it become s_load (SMEM,
// lgkmcnt) instead of vector loads that would drain vmcnt and with it the
// whole DMA pipeline.
typedef __attribute__((address_space(4))) const int const_int_t;
// The kernel's descriptor argument as it sits in the kernarg segment (the
// host pass only parses the kernel: plain const there).
#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(4))) const DmaDesc KDesc;
#else
typedef const DmaDesc KDesc;
#endif

constexpr int DKC = 256;

// Timing experiments only (separate builds, never the shipped library):
// 1 = no DMA inside the K loop, 2 = no MFMA, 3 = 1 without the per-tile
// barrier, 4 = 3 without the per-tile LDS reads.  Results are wrong under all.
#ifndef RTENHIP_DMA_EXPERIMENT
#define RTENHIP_DMA_EXPERIMENT 0
#endif

// LDS-DMA helpers (buffer_load_dword{,x4} ... lds), issued as inline asm.
// With the compiler builtin, the waitcnt pass treats every LDS read as
// possibly aliasing every DMA still in flight; once a wave has more DMAs
// outstanding than it can track individually (wave tiles above 32x32: 10+ per
// K tile) it drains the whole ring with an s_waitcnt vmcnt(0) before each
// tile's LDS reads, exposing the full DMA latency every K tile.  As asm the
// DMAs are invisible to that pass; the kernel orders them itself with counted
// s_waitcnt vmcnt + s_barrier (wait_dma) and drains them before the epilogue
// reuses the LDS.  (Loads the compiler does track stay correctly waited for:
// vmcnt retires in issue order, so extra untracked loads only make its waits
// stricter.)  M0 holds the wave-uniform LDS destination; one wait state
// separates the M0 write from the DMA.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4 make_rsrc(const void* base, uint32_t num_records) {
  const uint64_t a = (uint64_t)base;
  return (u32x4){(uint32_t)a, (uint32_t)(a >> 32) & 0xffffu, num_records, 0x00020000u};
}
__device__ __forceinline__ uint32_t lds_addr(const float* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)p;
}
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void lds_dma16(u32x4 r, uint32_t dst, uint32_t voff, uint32_t soff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               ::"s"(__builtin_amdgcn_readfirstlane(dst)), "v"(voff), "s"(r), "s"(soff)
               : "memory", "m0");
}
__device__ __forceinline__ void lds_dma4(u32x4 r, uint32_t dst, uint32_t voff, uint32_t soff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dword %1, %2, %3 offen lds"
               ::"s"(__builtin_amdgcn_readfirstlane(dst)), "v"(voff), "s"(r), "s"(soff)
               : "memory", "m0");
}
#pragma clang diagnostic pop

__device__ __forceinline__ float f4_at(const float4& v, int j) {
  return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
}

// One block computes a BM x BN tile with WAVES_M x WAVES_N waves, each owning
// a (BM/WAVES_M) x (BN/WAVES_N) sub-tile of 32x32 MFMA accumulators.
//
// DUAL (d.dual): two GEMMs over the same output tile, summed in the
// epilogue -- ResNet's conv3 + downsample pair, y = act((W3·h + b3) + (Wd·x
// + bd)).  Segment 1 (d2: the downsample) runs its whole K fold first and
// keeps the folded value (bias included) in registers; segment 2 (d: conv3)
// then runs its own K loop and adds it where the unfused graph adds the
// residual: the same per-element operations as the two convs and the Add,
// without the downsample output's round trip through HBM.  With d.dual_one
// both segments run as one K loop (mode 3 below); with BVEC (both segments
// pointwise stride-1) only that way.
template <int NT, int BM, int BN, int BK, int WAVES_M, int WAVES_N, int MINW, int STAGES, int HEAD_,
          bool MULTI_KB, bool BVEC, bool DUAL = false>
__global__ __launch_bounds__(NT, MINW) void gemm_dma_kernel(DmaDesc d, DmaDesc d2, int tiles_m, int tiles_n) {
  static_assert(!DUAL || MULTI_KB, "dual GEMMs fold through the multi-block path");
  static_assert(STAGES >= 2 && STAGES <= 4, "2..4 stages");
  constexpr int NW = NT / 64;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int MI = WM / 32, NI = WN / 32;
  // A tile copy: dwordx4 per lane when there is enough data for every wave,
  // else dword.
  constexpr int A_LB = BM * BK * 4 >= NT * 16 ? 16 : 4;  // bytes per lane
  constexpr int A_CHUNK = 64 * A_LB;                     // bytes per wave-instruction
  constexpr int A_INSTR = BM * BK * 4 / A_CHUNK;
  // B tile copy: dword per lane (one k row of 64 columns per instruction), or
  // with BVEC dwordx4 (4 k rows x 64 columns per instruction; pointwise convs
  // whose 4-pixel groups are contiguous and whose k stride is linear).
  constexpr int B_INSTR = BVEC ? BK * BN / 256 : BK * (BN / 64);
  constexpr int A_PER_W = A_INSTR / NW;
  constexpr int B_PER_W = B_INSTR / NW;
  constexpr int STAGE = (BM + BN) * BK;      // floats per stage
  constexpr int KSTEPS = BK / 2;
  static_assert(WAVES_M * WAVES_N == NW, "wave grid");
  static_assert(A_INSTR % NW == 0 && B_INSTR % NW == 0, "even DMA split");
  static_assert(BN % 64 == 0 && DKC % BK == 0 && BK <= DMA_KTAB_PAD, "tile shape");
  static_assert(MI >= 1 && NI >= 1, "wave tile");
  static_assert(!BVEC || (NI == 1 && BN == 64 && BK % 4 == 0),
                "BVEC needs the identity B column layout and 64-column rows");

  __shared__ float lds[STAGES * STAGE];

  const int tid_o = threadIdx.x;

  // Work items are whole tiles and, with a KC split, single K blocks of the
  // split tiles; see the dispatch at the end of the kernel.
  const int bid = blockIdx.x;
  const int n_full = d.n_full;
  // Placement experiment (separate builds only): wave 0 records where and
  // when this block ran into a debug buffer of its own (vector stores).
  unsigned long long t_start = 0, t_kend = 0, t_sync = 0, t_bias = 0;
  if constexpr (RTENHIP_DMA_EXPERIMENT == 5) t_start = __builtin_amdgcn_s_memrealtime();
  auto stamp = [&]() __attribute__((always_inline)) {
    if constexpr (RTENHIP_DMA_EXPERIMENT == 5) {
      if (d.stamps && threadIdx.x == 0) {
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
        volatile unsigned long long* p = d.stamps + 8 * (size_t)bid;
        p[0] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
        p[1] = t_start;
        p[2] = t_end;
        p[3] = t_kend;  // end of the (last) item's K loop
        p[4] = t_sync;  // vectorised epilogue: after its drain + barrier
        p[5] = t_bias;  //   after the first accumulator block is in the LDS slot
      }
    }
  };
  __shared__ int last_arrival;  // split tiles: this block folds (see process)

  // One work item: output tile wg (kb_split < 0), or K block kb_split of split
  // tile split_idx (wg = n_full + split_idx).
  // Dual: segment 1's folded values, carried into segment 2's epilogue.
  f32x16 carry[DUAL ? MI : 1][DUAL ? NI : 1];
  // mode 0: one GEMM; 1: dual segment 1 (fold into carry, no epilogue);
  // 2: dual segment 2 (epilogue adds carry).
  // mode 3 (DUAL): both segments in one pipelined K loop -- segment 1's
  // tiles (desc e: the downsample) then segment 2's (desc d: conv3), the
  // refill DMAs running on across the boundary, so segment 2's first tiles
  // are in flight while segment 1 finishes; segment 1's fold is the carry.
  auto process = [&](const KDesc& d, const int wg, const int kb_split, const int split_idx, const int mode,
                     const KDesc& e) __attribute__((always_inline)) {
  // Lane-derived values are recomputed per item: hoisted out of the item loop
  // they would stay live across it and spill.
  int tid = tid_o;
  asm volatile("" : "+v"(tid));
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = (wave / WAVES_N) * WM;
  const int wn = (wave % WAVES_N) * WN;
  const int M = d.M, N = d.N, K = d.K;
  int tmi, tni;
  if (d.swz > 0) {  // strips of swz tile columns, n fastest within a strip (see DmaDesc::swz)
    const int tiles_n = (N + BN - 1) / BN, sw = d.swz * tiles_m;
    const int st = wg / sw, r = wg - st * sw;
    const int gw = min(d.swz, tiles_n - st * d.swz);
    tmi = r / gw;
    tni = st * d.swz + (r - tmi * gw);
  } else {
    tmi = wg % tiles_m;
    tni = wg / tiles_m;
  }
  const int tm = tmi * BM;
  const int tn = tni * BN;
  const int tiles_k = (K + BK - 1) / BK;
  constexpr int TPB = DKC / BK;  // K tiles per KC block
  // Dual, mode 3: segment 1 (e) occupies virtual K tiles [0, tk1), segment 2
  // (d) [tk1, tk1 + tiles_k).  (Same M, N and tile; both 4-byte B copies.)
  const bool seg2 = DUAL && mode == 3;
  const int tk1 = seg2 ? (e.K + BK - 1) / BK : 0;
  const int kt_lo = kb_split >= 0 ? kb_split * TPB : 0;
  const int kt_hi = kb_split >= 0 ? min(tiles_k, kt_lo + TPB) : tk1 + tiles_k;

  const u32x4 ra = make_rsrc(d.apk, 0x7fffffffu);
  const u32x4 rb = make_rsrc(d.x, d.x_bytes);

  // Per-lane B offsets: one per 64-column group this wave loads.
  constexpr int NG = BN / 64;
  uint32_t vb[NG];
#pragma unroll
  for (int g = 0; g < NG; g++) {
    // LDS position p of a B row holds column wn' + ni*32 + l where p = wn' + l*NI + ni,
    // so a lane's NI B values for one k are adjacent (one ds_read).
    const int pos = g * 64 + lane;
    const int q = pos % WN;
    const int n = tn + (pos - q) + (q % NI) * 32 + q / NI;
    uint32_t off = DMA_OOB;
    if (n < N) {
      const int img = fdiv(n, d.fdP);
      const int p = n - img * d.P;
      const int oy = fdiv(p, d.fdOW);
      const int ox = p - oy * d.OW;
      off = (uint32_t)(((int64_t)img * d.x_img + (int64_t)oy * d.ystride + (int64_t)ox * d.xstride) * 4);
    }
    vb[g] = off;
  }
  // BVEC: instruction i of this wave covers k rows 4*(wave*B_PER_W+i) .. +3 of
  // the tile; lane -> row (lane >> 4), columns 4*(lane & 15) .. +3.
  uint32_t vb4[BVEC ? B_PER_W : 1];
  if constexpr (BVEC) {
#pragma unroll
    for (int i = 0; i < B_PER_W; i++) {
      const int gi = wave * B_PER_W + i;
      const int kk = gi * 4 + (lane >> 4);
      const int n = tn + (lane & 15) * 4;
      uint32_t off = DMA_OOB;
      if (n < N) {
        const int img = fdiv(n, d.fdP);
        const int p = n - img * d.P;
        off = (uint32_t)(((int64_t)img * d.x_img + p) * 4 + (int64_t)kk * d.kstride * 4);
      }
      vb4[i] = off;
    }
  }
  const uint32_t va = (uint32_t)(wave * A_PER_W * A_CHUNK + lane * A_LB);
  const uint32_t a_row_base = (uint32_t)tmi * (uint32_t)tiles_k * (BM * BK * 4);
  const_int_t* ktab4 = (const_int_t*)d.ktab4;
  const uint32_t lds0 = lds_addr(lds);
  u32x4 ra1 = ra, rb1 = rb;  // segment 1's resources (mode 3)
  uint32_t vb1[DUAL ? NG : 1];
  uint32_t a_row_base1 = 0;
  const_int_t* ktab41 = ktab4;
  uint32_t vb41[BVEC && DUAL ? B_PER_W : 1];
  if constexpr (DUAL) {
    if (seg2) {
      ra1 = make_rsrc(e.apk, 0x7fffffffu);
      rb1 = make_rsrc(e.x, e.x_bytes);
      a_row_base1 = (uint32_t)tmi * (uint32_t)tk1 * (BM * BK * 4);
      ktab41 = (const_int_t*)e.ktab4;
      if constexpr (BVEC) {
#pragma unroll
        for (int i = 0; i < B_PER_W; i++) {
          const int kk = (wave * B_PER_W + i) * 4 + (lane >> 4);
          const int n = tn + (lane & 15) * 4;
          uint32_t off = DMA_OOB;
          if (n < N) {
            const int img = fdiv(n, e.fdP);
            const int p = n - img * e.P;
            off = (uint32_t)(((int64_t)img * e.x_img + p) * 4 + (int64_t)kk * e.kstride * 4);
          }
          vb41[i] = off;
        }
      }
#pragma unroll
      for (int g = 0; g < NG; g++) {
        const int pos = g * 64 + lane;
        const int q = pos % WN;
        const int n = tn + (pos - q) + (q % NI) * 32 + q / NI;
        uint32_t off = DMA_OOB;
        if (n < N) {
          const int img = fdiv(n, e.fdP);
          const int p = n - img * e.P;
          const int oy = fdiv(p, e.fdOW);
          const int ox = p - oy * e.OW;
          off = (uint32_t)(((int64_t)img * e.x_img + (int64_t)oy * e.ystride + (int64_t)ox * e.xstride) * 4);
        }
        vb1[g] = off;
      }
    }
  }

  // K-table offsets of the tile about to be issued, loaded at the start of
  // the tile body that issues it, so the scalar load's latency hides under
  // that body's first MFMAs.
  // Two sets (by register-set parity): the steady-state body loads the next
  // body's offsets right after its barrier, a whole K tile before they are
  // used, so the pre-barrier lgkmcnt(0) never waits on a fresh scalar load.
  constexpr int KPRE = BVEC ? 1 : B_PER_W;
  uint32_t kpre[2][KPRE];
  auto load_k = [&](int kt, int slot) __attribute__((always_inline)) {
    if constexpr (!BVEC) {
      if (DUAL && kt < tk1) {  // (tk1 = 0 unless mode 3)
#pragma unroll
        for (int i = 0; i < B_PER_W; i++) kpre[slot][i] = (uint32_t)ktab41[kt * BK + (wave * B_PER_W + i) / NG];
        return;
      }
      kt = min(kt - tk1, tiles_k - 1);
#pragma unroll
      for (int i = 0; i < B_PER_W; i++) kpre[slot][i] = (uint32_t)ktab4[kt * BK + (wave * B_PER_W + i) / NG];
    }
  };

  // An empty asm reading the prefetched offsets, placed after the MFMAs:
  // keeps the load from being sunk into the conditional issue block.
  auto pin_k = [&](int slot) __attribute__((always_inline)) {
    if constexpr (!BVEC) {
#pragma unroll
      for (int i = 0; i < B_PER_W; i++) asm volatile("" ::"s"(kpre[slot][i]));
    }
  };

  // DMA j (0 <= j < A_PER_W + B_PER_W) of this wave's share of tile kt, into
  // stage `stage`: the A pieces first, then the B rows.
  auto issue_j = [&](int stage, int kt, int j, int slot) __attribute__((always_inline)) {
    const uint32_t As = lds0 + (uint32_t)(stage * STAGE * 4);
    const uint32_t Bs = As + BM * BK * 4;
    const bool s1 = DUAL && kt < tk1;  // wave-uniform
    if (j < A_PER_W) {
      const uint32_t a_soff = s1 ? a_row_base1 + (uint32_t)kt * (BM * BK * 4)
                                 : a_row_base + (uint32_t)(kt - tk1) * (BM * BK * 4);
      const uint32_t dst = As + (uint32_t)((wave * A_PER_W + j) * A_CHUNK);
      if constexpr (A_LB == 16)
        lds_dma16(s1 ? ra1 : ra, dst, va + j * A_CHUNK, a_soff);
      else
        lds_dma4(s1 ? ra1 : ra, dst, va + j * A_CHUNK, a_soff);
      return;
    }
    const int i = j - A_PER_W;
    if constexpr (BVEC) {
      const int gi = wave * B_PER_W + i;  // rows 4*gi .. 4*gi+3: 1 KB of LDS
      if constexpr (DUAL) {
        const uint32_t b_soff = s1 ? (uint32_t)kt * (uint32_t)(BK * e.kstride * 4)
                                   : (uint32_t)(kt - tk1) * (uint32_t)(BK * d.kstride * 4);
        lds_dma16(s1 ? rb1 : rb, Bs + gi * 1024, s1 ? vb41[i] : vb4[i], b_soff);
      } else {
        const uint32_t b_soff = (uint32_t)kt * (uint32_t)(BK * d.kstride * 4);
        lds_dma16(rb, Bs + gi * 1024, vb4[i], b_soff);
      }
    } else {
      const int gi = wave * B_PER_W + i;  // wave-uniform
      const int kl = gi / NG, g = gi % NG;
      if constexpr (DUAL)
        lds_dma4(s1 ? rb1 : rb, Bs + (uint32_t)((kl * BN + g * 64) * 4), s1 ? vb1[g] : vb[g], kpre[slot][i]);
      else
        lds_dma4(rb, Bs + (uint32_t)((kl * BN + g * 64) * 4), vb[g], kpre[slot][i]);
    }
  };
  auto issue = [&](int stage, int kt) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < A_PER_W + B_PER_W; j++) issue_j(stage, kt, j, 0);
  };

  f32x16 acc[MI][NI];
#pragma unroll
  for (int mi = 0; mi < MI; mi++)
#pragma unroll
    for (int ni = 0; ni < NI; ni++) acc[mi][ni] = (f32x16){0};

  const int half = lane >> 5;
  const int l32 = lane & 31;
  const int m_lim = M - 1 - tm;
  const int n_lim = N - 1 - tn;
  auto lrow = [&](int mi, int j) __attribute__((always_inline)) { return wm + mi * 32 + (j & 3) + 8 * (j >> 2) + 4 * half; };

  // Bias of accumulator row j, read through the constant address space: the
  // row index without the lane's half-wave offset is wave-uniform, so both
  // candidates (rows r and r + 4) are scalar loads (lgkmcnt, no interaction
  // with the counted DMA waits) and the lane selects one.  Nothing is held
  // across the K loop.
  typedef __attribute__((address_space(4))) const float cfloat_t;
  auto bias_row = [&](int mi, int j) __attribute__((always_inline)) {
    cfloat_t* cb = (cfloat_t*)d.bias;
    const int r = tm + wm + mi * 32 + (j & 3) + 8 * (j >> 2);
    const float lo = cb[min(r, M - 1)], hi = cb[min(r + 4, M - 1)];
    return half ? hi : lo;
  };

  // End of K block 0: v = alpha*acc (+ beta*C) + bias (gemm.rs:1004-1050).
  // with_bias false: the caller adds the bias itself, next in the same order
  // (the vectorised epilogue, after its LDS transpose).
  auto first_block = [&](f32x16& v, const f32x16& a, int mi, int ni, bool with_bias = true) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const int ml = min(lrow(mi, j), m_lim);
      float x;
      if (d.cin) {
        const int nl = min(wn + ni * 32 + l32, n_lim);
        const float c = d.cin[(int64_t)(tm + ml) * d.out_c + tn + nl];
        x = __fmaf_rn(a[j], d.alpha, __fmul_rn(c, d.beta));
      } else {
        x = d.alpha == 1.f ? a[j] : __fmul_rn(a[j], d.alpha);  // x * 1 == x exactly
      }
      if (with_bias && d.bias) x = __fadd_rn(x, bias_row(mi, j));
      v[j] = x;
    }
  };

  // LDS read offsets of this lane (floats, relative to a stage): its MI A
  // values and NI B values of one k row are contiguous (see pack_a_kernel and
  // the B column permutation above).
  // A tiles are packed k-quad major (see pack_a_kernel): a lane's A values of
  // 4 consecutive k steps (k = 2*(4*sq + j) + half, j = 0..3) are one float4,
  // so each 32-row group costs one ds_read_b128 per 4 MFMA steps.
  const int a_lane = (half * BM + wm + l32) * 4;
  const int b_lane = BM * BK + half * BN + wn + l32 * NI;

  // Software pipeline over K tiles.  A tile's operands are read from LDS
  // into one of two register sets in a single burst; the next tile's burst is
  // issued before the last two MFMA steps of the current one, so LDS latency
  // hides behind MFMAs.  As soon as every wave holds its operands of tile kt
  // (barrier), tile kt's stage is refilled with tile kt+STAGES.  Waits are
  // counted and the barrier is a raw s_barrier, so later tiles' DMAs stay in
  // flight across it (__syncthreads would drain vmcnt).
  constexpr int PER_TILE = A_PER_W + B_PER_W;
  static_assert(KSTEPS % 4 == 0, "A k-quads");
  typedef float vb_t __attribute__((ext_vector_type(NI)));
  float4 av[2][KSTEPS / 4][MI];
  vb_t bv[2][KSTEPS];

  auto wait_dma = [&](int allowed_tiles) __attribute__((always_inline)) {
    if (STAGES >= 4 && allowed_tiles >= 3) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_TILE * 3) : "memory");
    } else if (STAGES >= 3 && allowed_tiles >= 2) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_TILE * 2) : "memory");
    } else if (allowed_tiles >= 1) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_TILE) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  };
  auto read_tile = [&](auto set_tag, int stage) __attribute__((always_inline)) {
    constexpr int SET = decltype(set_tag)::value;
    if constexpr (RTENHIP_DMA_EXPERIMENT == 4) {
      if (stage != 0) return;  // keep only the prologue's read
    }
    const float* As = lds + stage * STAGE + a_lane;
    const float* Bs = lds + stage * STAGE + b_lane;
#pragma unroll
    for (int s = 0; s < KSTEPS; s++) {
      if (s % 4 == 0) {
#pragma unroll
        for (int mi = 0; mi < MI; mi++) av[SET][s / 4][mi] = *(const float4*)(As + (s / 2 * BM + mi * 32) * 4);
      }
      bv[SET][s] = *(const vb_t*)(Bs + 2 * s * BN);
    }
  };
  auto mfma_steps = [&](auto set_tag, auto s0_tag, auto s1_tag) __attribute__((always_inline)) {
    constexpr int SET = decltype(set_tag)::value;
    if constexpr (RTENHIP_DMA_EXPERIMENT == 2) return;
#pragma unroll
    for (int s = decltype(s0_tag)::value; s < decltype(s1_tag)::value; s++)
#pragma unroll
      for (int mi = 0; mi < MI; mi++)
#pragma unroll
        for (int ni = 0; ni < NI; ni++)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4_at(av[SET][s / 4][mi], s % 4), bv[SET][s][ni],
                                                             acc[mi][ni], 0, 0, 0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  // Each K tile: HEAD MFMA steps, the DMA wait + barrier, the next tile's
  // LDS reads, then the TAIL steps with the refill DMAs interleaved (a few
  // after each MFMA, inside its 64-cycle shadow) instead of one burst that
  // the wave's own MFMAs cannot cover.
  // HEAD_ is a configuration parameter: an early barrier (2) suits the
  // long-K layer3 / layer4 convs, a late one (6) the 56x56 ones.
  constexpr int HEAD = KSTEPS > HEAD_ ? HEAD_ : KSTEPS / 2;
  constexpr int TAIL = KSTEPS - HEAD;
  using IMid = std::integral_constant<int, HEAD>;
  using IEnd = std::integral_constant<int, KSTEPS>;
  // The tail steps of register set SET, refilling stage `rs` with tile `rkt`
  // when `refill`.
  auto tail_steps = [&](auto set_tag, int rs, int rkt, bool refill) __attribute__((always_inline)) {
    constexpr int SET = decltype(set_tag)::value;
#pragma unroll
    for (int t = 0; t < TAIL; t++) {
      const int s = HEAD + t;
#pragma unroll
      for (int mi = 0; mi < MI; mi++)
#pragma unroll
        for (int ni = 0; ni < NI; ni++)
          if constexpr (RTENHIP_DMA_EXPERIMENT != 2)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4_at(av[SET][s / 4][mi], s % 4),
                                                               bv[SET][s][ni], acc[mi][ni], 0, 0, 0);
      if (refill && (RTENHIP_DMA_EXPERIMENT == 0 || RTENHIP_DMA_EXPERIMENT == 2)) {
#pragma unroll
        for (int j = t * PER_TILE / TAIL; j < (t + 1) * PER_TILE / TAIL; j++) issue_j(rs, rkt, j, SET);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  int stage = 0;  // stage holding tile kt
  auto body = [&](auto set_tag, int kt) __attribute__((always_inline)) {
    constexpr int SET = decltype(set_tag)::value;
    load_k(kt + STAGES, SET);  // unconditional (clamped): no phi, so no early wait
    __builtin_amdgcn_sched_barrier(0);  // keep the scalar load ahead of the MFMAs
    mfma_steps(set_tag, I0{}, IMid{});
    pin_k(SET);
    const int refill_stage = stage;
    const bool refill = kt + 1 < kt_hi && kt + STAGES < kt_hi;
    if (kt + 1 < kt_hi) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      wait_dma(min(STAGES - 2, kt_hi - kt - 2));
      if constexpr (RTENHIP_DMA_EXPERIMENT < 3) __builtin_amdgcn_s_barrier();
      stage = stage + 1 == STAGES ? 0 : stage + 1;
      read_tile(std::integral_constant<int, SET ^ 1>{}, stage);
    }
    tail_steps(set_tag, refill_stage, kt + STAGES, refill);
  };
  // Steady state (STAGES = 2 or 4, whose ring period divides both the
  // register-set period 2 and the KC block): a group of STAGES tiles with
  // compile-time stage and register-set indices, fixed DMA wait counts and
  // no bounds tests -- LDS addresses become immediates and the per-tile
  // scalar/vector bookkeeping disappears.  Valid while every tile of the
  // group still has a refill to issue (kt + STAGES - 1 + STAGES < kt_hi).
  constexpr bool FAST = STAGES == 2 || STAGES == 4;
  auto body_fast = [&](auto set_tag, auto stg_tag, int kt) __attribute__((always_inline)) {
    constexpr int SET = decltype(set_tag)::value;
    constexpr int STG = decltype(stg_tag)::value;
    mfma_steps(set_tag, I0{}, IMid{});
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_TILE * (STAGES - 2)) : "memory");
    if constexpr (RTENHIP_DMA_EXPERIMENT < 3) __builtin_amdgcn_s_barrier();
    load_k(kt + 1 + STAGES, SET ^ 1);  // the next body's refill offsets (this body's: kpre[SET])
    read_tile(std::integral_constant<int, SET ^ 1>{}, (STG + 1) % STAGES);
    tail_steps(set_tag, STG, kt + STAGES, true);
  };
  // Tiles [kt0, kt1) with kt0 even (register set = tile parity) and
  // (kt0 - kt_lo) % STAGES == 0 (stage of tile kt0 is 0).
  auto run = [&](int kt0, int kt1) __attribute__((always_inline)) {
    int kt = kt0;
    if constexpr (FAST) {
      if (kt + STAGES <= kt1 && kt + 2 * STAGES - 1 < kt_hi) load_k(kt + STAGES, 0);
      for (; kt + STAGES <= kt1 && kt + 2 * STAGES - 1 < kt_hi; kt += STAGES) {
        body_fast(I0{}, std::integral_constant<int, 0>{}, kt);
        body_fast(I1{}, std::integral_constant<int, 1>{}, kt + 1);
        if constexpr (STAGES == 4) {
          body_fast(I0{}, std::integral_constant<int, 2>{}, kt + 2);
          body_fast(I1{}, std::integral_constant<int, 3>{}, kt + 3);
        }
      }
    }
    for (; kt < kt1; kt += 2) {
      body(I0{}, kt);
      if (kt + 1 < kt1) body(I1{}, kt + 1);
    }
  };

  // Vectorised epilogue geometry (see the epilogue) and, for short-K small
  // wave tiles (memory-bound pointwise convs with a residual), the residual
  // prefetched now so its latency hides under the K loop (it does not depend
  // on the GEMM).  Not with MULTI_KB: held across the long K loop, its 16
  // registers push the kernel into spills.
  constexpr bool VEC_FITS = NW * 1024 <= STAGES * STAGE;
  constexpr bool RES_PRE = VEC_FITS && !MULTI_KB && MI * NI == 1 && BK == 16 && MINW <= 4;
  const int rr = lane >> 3;        // row within an 8-row group
  const int c4 = (lane & 7) * 4;   // first of this lane's 4 columns
  float4 rpre[RES_PRE ? 4 : 1];
  // With RES_PRE the bias of the lane's 4 epilogue rows is prefetched too.
  float bpre[RES_PRE ? 4 : 1];
  if constexpr (RES_PRE) {
    if (d.vec4 && d.bias && !d.cin) {
#pragma unroll
      for (int i = 0; i < 4; i++) bpre[i] = d.bias[min(tm + wm + i * 8 + rr, M - 1)];
    }
    if (d.vec4 && d.residual) {
      const int n = tn + wn + c4;
      const bool ncol_ok = n <= N - 1;
      const int nn = ncol_ok ? n : 0;
      const int img = fdiv(nn, d.fdP);
      const int64_t rbase = (int64_t)img * d.res_img + (nn - img * d.P);
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int m = tm + wm + i * 8 + rr;
        rpre[i] = (ncol_ok && m < M) ? *(const float4*)(d.residual + rbase + (int64_t)m * d.res_c)
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }


  // Prologue: fill every stage, wait for the first tile, read it.
#pragma unroll
  for (int s = 0; s < STAGES; s++)
    if (kt_lo + s < kt_hi) {
      load_k(kt_lo + s, 0);
      issue(s, kt_lo + s);
    }
  wait_dma(min(STAGES, kt_hi - kt_lo) - 1);
  __builtin_amdgcn_s_barrier();
  read_tile(I0{}, 0);

  f32x16 sum[MULTI_KB ? MI : 1][MULTI_KB ? NI : 1];
  if constexpr (!MULTI_KB) {
    run(0, tiles_k);
  } else if (kb_split >= 0) {
    // One KC block of a split tile: its chain goes to the workspace; the
    // last of the tile's nkb blocks to arrive folds all chains in K order
    // exactly as the whole-tile path does, then runs the epilogue.
    run(kt_lo, kt_hi);
    // Hand-off without L2 write-back fences (MI355X guide, Guideline 16 /
    // "Valid forms" row 1): chains are stored write-through (sc1, as 8-byte
    // agent-scope atomic stores), every storing wave drains (vmcnt(0)) before
    // the workgroup barrier, one lane adds to the tile's counter (agent scope)
    // and the workgroup whose add returns nkb-1 reads the chains with sc1
    // loads only.
    constexpr int CH = MI * NI * 16 * NT;  // floats per chain (whole block)
    // 8-byte granules, stored and loaded as agent-scope relaxed atomics
    // (global_store/load_dwordx2 sc1).  Layout per chain: [(mi*NI+ni)*8 + jp][tid].
    // (__float_as_uint, not __builtin_bit_cast: clang 22 folds a bit_cast of
    // an ext_vector element to element 0.)
    unsigned long long* wsq =
        reinterpret_cast<unsigned long long*>(d.ws + (int64_t)split_idx * d.nkb * CH);
    auto qidx = [&](int kb, int mi, int ni, int jp) {
      return ((int64_t)kb * (CH / 2)) + (((mi * NI + ni) * 8 + jp) * NT + tid);
    };
#pragma unroll
    for (int mi = 0; mi < MI; mi++)
#pragma unroll
      for (int ni = 0; ni < NI; ni++)
#pragma unroll
        for (int jp = 0; jp < 8; jp++) {
          const unsigned long long q =
              (unsigned long long)__float_as_uint(acc[mi][ni][2 * jp]) |
              ((unsigned long long)__float_as_uint(acc[mi][ni][2 * jp + 1]) << 32);
          __hip_atomic_store(wsq + qidx(kb_split, mi, ni, jp), q, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const int prev = __hip_atomic_fetch_add(d.counters + split_idx, 1, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
      last_arrival = prev == d.nkb - 1;
    }
    __syncthreads();
    if (!last_arrival) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only
    auto ldq = [&](int kb, int mi, int ni, int jp) {
      return __hip_atomic_load(wsq + qidx(kb, mi, ni, jp), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    };
    auto lo = [](unsigned long long q) { return __uint_as_float((unsigned)(q & 0xffffffffu)); };
    auto hi = [](unsigned long long q) { return __uint_as_float((unsigned)(q >> 32)); };
#pragma unroll
    for (int mi = 0; mi < MI; mi++)
#pragma unroll
      for (int ni = 0; ni < NI; ni++) {
        f32x16 c;
#pragma unroll
        for (int jp = 0; jp < 8; jp++) {
          const unsigned long long q = ldq(0, mi, ni, jp);
          c[2 * jp] = lo(q);
          c[2 * jp + 1] = hi(q);
        }
        first_block(sum[mi][ni], c, mi, ni);
      }
    // Remaining chains in K order; loads of a group of blocks are issued
    // together so the fold is not latency-bound.
    constexpr int G = MI * NI == 1 ? 2 : 1;
    for (int kb0 = 1; kb0 < d.nkb; kb0 += G) {
      f32x16 cg[G][MI][NI];
#pragma unroll
      for (int gi = 0; gi < G; gi++) {
        if (kb0 + gi >= d.nkb) break;
#pragma unroll
        for (int mi = 0; mi < MI; mi++)
#pragma unroll
          for (int ni = 0; ni < NI; ni++)
#pragma unroll
            for (int jp = 0; jp < 8; jp++) {
              const unsigned long long q = ldq(kb0 + gi, mi, ni, jp);
              cg[gi][mi][ni][2 * jp] = lo(q);
              cg[gi][mi][ni][2 * jp + 1] = hi(q);
            }
      }
#pragma unroll
      for (int gi = 0; gi < G; gi++) {
        if (kb0 + gi >= d.nkb) break;
#pragma unroll
        for (int mi = 0; mi < MI; mi++)
#pragma unroll
          for (int ni = 0; ni < NI; ni++)
#pragma unroll
            for (int j = 0; j < 16; j++)
              sum[mi][ni][j] = __fmaf_rn(cg[gi][mi][ni][j], d.alpha, sum[mi][ni][j]);
      }
    }
    if (tid == 0)
      __hip_atomic_store(d.counters + split_idx, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if (DUAL && seg2) {
    // Segment 1's KC blocks (virtual tiles [0, tk1)): block 0 + e's bias,
    // later blocks added in K order -> the carry; then segment 2's blocks
    // from tile tk1, folded as one GEMM (the epilogue adds the carry).
    // tk1 and TPB are even (register-set parity) and multiples of STAGES for
    // the fast path (K1 a multiple of 64: the ResNet downsample widths).
    run(0, min(TPB, tk1));
#pragma unroll
    for (int mi = 0; mi < MI; mi++)
#pragma unroll
      for (int ni = 0; ni < NI; ni++) {
#pragma unroll
        for (int j = 0; j < 16; j++) {
          float x = e.alpha == 1.f ? acc[mi][ni][j] : __fmul_rn(acc[mi][ni][j], e.alpha);
          if (e.bias) {
            cfloat_t* cb = (cfloat_t*)e.bias;
            const int r = tm + wm + mi * 32 + (j & 3) + 8 * (j >> 2);
            const float lo = cb[min(r, M - 1)], hi = cb[min(r + 4, M - 1)];
            x = __fadd_rn(x, half ? hi : lo);
          }
          sum[mi][ni][j] = x;
        }
        acc[mi][ni] = (f32x16){0};
      }
    for (int kt = TPB; kt < tk1; kt += TPB) {
      run(kt, min(kt + TPB, tk1));
#pragma unroll
      for (int mi = 0; mi < MI; mi++)
#pragma unroll
        for (int ni = 0; ni < NI; ni++) {
#pragma unroll
          for (int j = 0; j < 16; j++) sum[mi][ni][j] = __fmaf_rn(acc[mi][ni][j], e.alpha, sum[mi][ni][j]);
          acc[mi][ni] = (f32x16){0};
        }
    }
#pragma unroll
    for (int mi = 0; mi < MI; mi++)
#pragma unroll
      for (int ni = 0; ni < NI; ni++) carry[mi][ni] = sum[mi][ni];
    run(tk1, tk1 + min(TPB, tiles_k));
#pragma unroll
    for (int mi = 0; mi < MI; mi++)
#pragma unroll
      for (int ni = 0; ni < NI; ni++) {
        first_block(sum[mi][ni], acc[mi][ni], mi, ni);
        acc[mi][ni] = (f32x16){0};
      }
    for (int kt = TPB; kt < tiles_k; kt += TPB) {
      run(tk1 + kt, tk1 + min(kt + TPB, tiles_k));
#pragma unroll
      for (int mi = 0; mi < MI; mi++)
#pragma unroll
        for (int ni = 0; ni < NI; ni++) {
#pragma unroll
          for (int j = 0; j < 16; j++) sum[mi][ni][j] = __fmaf_rn(acc[mi][ni][j], d.alpha, sum[mi][ni][j]);
          acc[mi][ni] = (f32x16){0};
        }
    }
  } else {
    // K > DKC: block 0 is peeled so the bias/beta fold sits outside the loop.
    static_assert(TPB % 2 == 0, "register-set parity across K blocks");
    run(0, DUAL ? min(TPB, tiles_k) : TPB);  // (only a dual segment can have K <= DKC here)
#pragma unroll
    for (int mi = 0; mi < MI; mi++)
#pragma unroll
      for (int ni = 0; ni < NI; ni++) {
        first_block(sum[mi][ni], acc[mi][ni], mi, ni);
        acc[mi][ni] = (f32x16){0};
      }
    for (int kt = TPB; kt < tiles_k; kt += TPB) {
      run(kt, min(kt + TPB, tiles_k));
#pragma unroll
      for (int mi = 0; mi < MI; mi++)
#pragma unroll
        for (int ni = 0; ni < NI; ni++) {
#pragma unroll
          for (int j = 0; j < 16; j++) sum[mi][ni][j] = __fmaf_rn(acc[mi][ni][j], d.alpha, sum[mi][ni][j]);
          acc[mi][ni] = (f32x16){0};
        }
    }
  }

  if constexpr (DUAL) {
    if (mode == 1) {
#pragma unroll
      for (int mi = 0; mi < MI; mi++)
#pragma unroll
        for (int ni = 0; ni < NI; ni++) carry[mi][ni] = sum[mi][ni];
      return;
    }
  }
  if constexpr (RTENHIP_DMA_EXPERIMENT == 5) t_kend = __builtin_amdgcn_s_memrealtime();
  // ---- epilogue ----
  auto apply_act = [&](float x) __attribute__((always_inline)) {
    if (d.act == RTENHIP_ACT_RELU) {
      x = fmaxf(x, 0.f);
    } else if (d.act == RTENHIP_ACT_CLIP) {
      x = rust_clamp(x, d.act_lo, d.act_hi);
    } else if (d.act == RTENHIP_ACT_GELU) {
      x = vm_gelu(x);
    }
    return x;
  };
  // Relu / Clip / none as selects (no per-element branches); Gelu separately.
  const bool act_relu = d.act == RTENHIP_ACT_RELU, act_clip = d.act == RTENHIP_ACT_CLIP;
  const float clip_lo = d.act_lo, clip_hi = d.act_hi;
  auto apply_act_sel = [&](float x) __attribute__((always_inline)) {
    const float r = fmaxf(x, 0.f);
    const float c = rust_clamp(x, clip_lo, clip_hi);
    return act_relu ? r : (act_clip ? c : x);
  };
  if (VEC_FITS && d.vec4) {
    // Row-contiguous outputs (P % 4 == 0, unpadded): each 32x32 accumulator
    // block is transposed through this wave's LDS slot so every lane stores
    // (and loads the residual as) 16-byte row segments: 4 dwordx4 per block
    // instead of 16 dword accesses.  Same per-element arithmetic as below.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land in the slots
    __syncthreads();  // every wave is done reading the K stages
    if constexpr (RTENHIP_DMA_EXPERIMENT == 5) t_sync = __builtin_amdgcn_s_memrealtime();
    float* slot = lds + wave * 1024;
    // Without a C input the bias is added after the transpose: a lane then
    // needs the bias of its 4 rows only (vector loads issued together),
    // instead of two scalar loads per accumulator element.
    const bool bias_late = !MULTI_KB && d.bias && !d.cin;
    const bool gelu = d.act == RTENHIP_ACT_GELU;
#pragma unroll
    for (int mi = 0; mi < MI; mi++)
#pragma unroll
      for (int ni = 0; ni < NI; ni++) {
        // Every load of this block is issued before its stores: vmcnt
        // retires in order, so a load issued after a store would wait for it.
        // Addresses are clamped in range; rows / columns out of range are
        // computed but not stored.
        const int n = tn + wn + ni * 32 + c4;
        const bool ncol_ok = n <= N - 1;  // N % 4 == 0: the whole segment is in range
        const int nn = ncol_ok ? n : 0;
        const int img = fdiv(nn, d.fdP);
        const int p = nn - img * d.P;
        const int64_t obase = (int64_t)img * d.out_img + p;
        const int64_t rbase = (int64_t)img * d.res_img + p;
        float bl[4] = {0.f, 0.f, 0.f, 0.f};
        if (bias_late) {
#pragma unroll
          for (int i = 0; i < 4; i++)
            bl[i] = RES_PRE ? bpre[i] : d.bias[min(tm + wm + mi * 32 + i * 8 + rr, M - 1)];
        }
        float4 cb = make_float4(0.f, 0.f, 0.f, 0.f);
        if (d.colbias) cb = *(const float4*)(d.colbias + nn);  // (colbias over all N columns)
        float bnm[4] = {0.f, 0.f, 0.f, 0.f}, bns[4] = {0.f, 0.f, 0.f, 0.f}, bnb[4] = {0.f, 0.f, 0.f, 0.f};
        if (d.bn) {
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const int mr = min(tm + wm + mi * 32 + i * 8 + rr, M - 1);
            bnm[i] = d.bn[mr];
            bns[i] = d.bn[d.bn_c + mr];
            bnb[i] = d.bn[2 * d.bn_c + mr];
          }
        }
        float4 rl[RES_PRE ? 1 : 4];
        if constexpr (!RES_PRE) {
          if (d.residual) {
#pragma unroll
            for (int i = 0; i < 4; i++)
              rl[i] = *(const float4*)(d.residual + rbase + (int64_t)min(tm + wm + mi * 32 + i * 8 + rr, M - 1) * d.res_c);
          }
        }
        f32x16 v;
        if constexpr (MULTI_KB) {
          v = sum[mi][ni];
        } else if (!d.cin && d.alpha == 1.f) {
          v = acc[mi][ni];  // first_block without C, alpha and (late) bias: the values as they are
          if (!bias_late && d.bias) first_block(v, acc[mi][ni], mi, ni);
        } else {
          first_block(v, acc[mi][ni], mi, ni, !bias_late);
        }
        if constexpr (DUAL) {
          // (the bias is in v already: MULTI_KB; no column bias or residual)
#pragma unroll
          for (int j = 0; j < 16; j++) v[j] = __fadd_rn(v[j], carry[mi][ni][j]);
        }
#pragma unroll
        for (int j = 0; j < 16; j++) slot[((j & 3) + 8 * (j >> 2) + 4 * half) * 32 + l32] = v[j];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (RTENHIP_DMA_EXPERIMENT == 5) t_bias = __builtin_amdgcn_s_memrealtime();
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const int row = i * 8 + rr;
          const int m = tm + wm + mi * 32 + row;
          const bool ok = ncol_ok && m < M;
          float4 x = *(const float4*)(slot + row * 32 + c4);
          if (bias_late) {
            x.x = __fadd_rn(x.x, bl[i]);
            x.y = __fadd_rn(x.y, bl[i]);
            x.z = __fadd_rn(x.z, bl[i]);
            x.w = __fadd_rn(x.w, bl[i]);
          }
          if (d.colbias) {
            x.x = __fadd_rn(x.x, cb.x);
            x.y = __fadd_rn(x.y, cb.y);
            x.z = __fadd_rn(x.z, cb.z);
            x.w = __fadd_rn(x.w, cb.w);
          }
          if (d.bn) {  // (x - mean) * s + beta, each step rounded (norm.rs:49)
            x.x = __fadd_rn(__fmul_rn(__fsub_rn(x.x, bnm[i]), bns[i]), bnb[i]);
            x.y = __fadd_rn(__fmul_rn(__fsub_rn(x.y, bnm[i]), bns[i]), bnb[i]);
            x.z = __fadd_rn(__fmul_rn(__fsub_rn(x.z, bnm[i]), bns[i]), bnb[i]);
            x.w = __fadd_rn(__fmul_rn(__fsub_rn(x.w, bnm[i]), bns[i]), bnb[i]);
          }
          if (d.residual) {
            float4 r;
            if constexpr (RES_PRE)
              r = rpre[i];
            else
              r = rl[i];
            x.x = __fadd_rn(x.x, r.x);
            x.y = __fadd_rn(x.y, r.y);
            x.z = __fadd_rn(x.z, r.z);
            x.w = __fadd_rn(x.w, r.w);
          }
          if (gelu) {
            const vm_f32x2 g0 = vm_gelu2((vm_f32x2){x.x, x.y}), g1 = vm_gelu2((vm_f32x2){x.z, x.w});
            x = make_float4(g0[0], g0[1], g1[0], g1[1]);
          } else {
            x.x = apply_act_sel(x.x);
            x.y = apply_act_sel(x.y);
            x.z = apply_act_sel(x.z);
            x.w = apply_act_sel(x.w);
          }
          if (ok) {
            if (d.pk_out) {  // the consumer MatMul's packed A (row m, k = n .. n + 3)
              store_packed_a4(d.pk_out, d.pk_lbm, d.pk_lbk, d.pk_tiles_k, m, n, x);
            } else {
              *(float4*)(d.out + obase + (int64_t)m * d.out_c) = x;
            }
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
    return;
  }
  const bool full_tile = m_lim >= BM - 1 && n_lim >= BN - 1;
  const bool gelu_any = d.act == RTENHIP_ACT_GELU;
#pragma unroll
  for (int ni = 0; ni < NI; ni++) {
    const int nl = wn + ni * 32 + l32;
    const bool ncol_ok = nl <= n_lim;
    const int n = tn + min(nl, n_lim);
    const int img = fdiv(n, d.fdP);
    const int p = n - img * d.P;
    const int oy = fdiv(p, d.fdOW);
    const int ox = p - oy * d.OW;
    const int64_t obase = (int64_t)img * d.out_img + (int64_t)oy * d.out_row + ox + d.out_off;
    const int64_t rbase = (int64_t)img * d.res_img + p;
    // As in the vectorised path: this block's loads (bias rows, the column
    // bias, the residual) are issued together before its stores -- vmcnt
    // retires in order, so a load behind a store would wait for the store.
    const bool bias_late = !MULTI_KB && d.bias && !d.cin;
    const float cbv = d.colbias ? d.colbias[n] : 0.f;
#pragma unroll
    for (int mi = 0; mi < MI; mi++) {
      float bv[16], rv[16];
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const int ml = lrow(mi, j);
        const bool ok = full_tile || (ncol_ok && ml <= m_lim);
        bv[j] = bias_late ? d.bias[min(tm + ml, M - 1)] : 0.f;
        rv[j] = d.residual ? d.residual[ok ? rbase + (int64_t)(tm + ml) * d.res_c : 0] : 0.f;
      }
      f32x16 v;
      if constexpr (MULTI_KB) {
        v = sum[mi][ni];
      } else if (!d.cin && d.alpha == 1.f) {
        v = acc[mi][ni];
      } else {
        first_block(v, acc[mi][ni], mi, ni, !bias_late);
      }
      if constexpr (DUAL) {
#pragma unroll
        for (int j = 0; j < 16; j++) v[j] = __fadd_rn(v[j], carry[mi][ni][j]);
      }
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const int ml = lrow(mi, j);
        const bool ok = full_tile || (ncol_ok && ml <= m_lim);
        float x = v[j];
        if (bias_late) x = __fadd_rn(x, bv[j]);
        if (d.colbias) x = __fadd_rn(x, cbv);
        if (d.bn) {  // (x - mean) * s + beta (norm.rs:49); loaded here: BN-fused convs only
          const int mr = min(tm + ml, M - 1);
          x = __fadd_rn(__fmul_rn(__fsub_rn(x, d.bn[mr]), d.bn[d.bn_c + mr]), d.bn[2 * d.bn_c + mr]);
        }
        if (d.residual) x = __fadd_rn(x, rv[j]);
        x = gelu_any ? apply_act(x) : apply_act_sel(x);
        if (ok) d.out[obase + (int64_t)(tm + ml) * d.out_c] = x;
      }
    }
  }
  };  // process

  // Work items.  Without persistence, one per block: blocks [0, n_full) each
  // own a whole tile (XCD-aware bijective remap, see gemm_mfma.hip) and, with
  // a KC split (d.split_tiles > 0), the remaining tiles -- the ones that would
  // leave CUs idle in a last partial round -- are cut at the reference's
  // KC = 256 boundaries: block n_full + t*nkb + kb computes only K block kb of
  // split tile t and the last of the nkb blocks to finish folds them in order.
  //
  // Persistent (d.persist_k > 0): the grid is exactly persist_k resident
  // blocks per CU (LDS padding caps the slots, see persistent_shape), and the
  // items are dealt out statically.  XCD x (the blocks b with b % 8 == x) owns
  // a contiguous range of the full tiles -- neighbouring tiles share A rows
  // and B columns in that XCD's L2 -- followed by a contiguous range of the
  // split tiles' K-block units, so the small units come last; its blocks take
  // positions r, r + G/8, r + 2G/8, ... of that range.  With every CU holding
  // the same number of blocks, every CU gets the same work (one block per
  // item lets the dispatcher stack an extra full tile on some CUs: on a
  // 784-tile layer 72 CUs ran 4 tiles and 184 ran 3).  No atomics: a pulled
  // queue position is a vector-memory op older than the DMAs, and the counted
  // DMA waits would stall on its round trip.
  const bool persistent = d.persist_k > 0;
  const int G = gridDim.x;
  const int nq = G < 8 ? G : 8;
  const int q = bid % nq;
  const int stride = G / nq + (q < G % nq ? 1 : 0);  // blocks serving queue q
  auto part = [&](int n, int& lo, int& cnt) {
    const int per = n / nq, r = n % nq;
    lo = q * per + (q < r ? q : r);
    cnt = per + (q < r ? 1 : 0);
  };
  int f_lo = 0, f_n = 1, st_lo = 0, st_n = 0;
  int p = 0;
  if (persistent) {
    part(n_full, f_lo, f_n);
    part(d.split_tiles, st_lo, st_n);
    p = bid / nq;
  }
  const int len = persistent ? f_n + st_n * d.nkb : 1;
  for (; p < len; p += stride) {
    int wg, kbs = -1, si = -1;
    if (!persistent) {
      if (bid < n_full) {
        const int qq = n_full >> 3, r = n_full & 7, xcd = bid & 7;
        wg = (xcd < r ? xcd * (qq + 1) : r * (qq + 1) + (xcd - r) * qq) + (bid >> 3);
      } else {
        const int u = bid - n_full;
        si = u / d.nkb;
        kbs = u - si * d.nkb;
        wg = n_full + si;
      }
    } else if (p < f_n) {
      wg = f_lo + p;
    } else {
      const int u = p - f_n;
      si = st_lo + u / d.nkb;
      kbs = u % d.nkb;
      wg = n_full + si;
    }
    // The descriptor is re-read through a laundered kernarg pointer per item:
    // values derived from it are not hoisted out of the item loop (live
    // across it, they spill).
    const KDesc* dp = (const KDesc*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(dp));
    if constexpr (DUAL && BVEC) {
      process(dp[0], wg, -1, -1, 3, dp[1]);  // (16-byte B copies: one K loop only)
    } else if constexpr (DUAL) {
      if (dp[0].dual_one) {
        process(dp[0], wg, -1, -1, 3, dp[1]);  // d2 (the second kernel argument): segment 1
      } else {
        process(dp[1], wg, -1, -1, 1, dp[1]);  // segment 1
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // segment 1's LDS stages are free
        process(dp[0], wg, -1, -1, 2, dp[1]);
      }
    } else {
      process(*dp, wg, kbs, si, 0, *dp);
    }
    if (!persistent) break;
    // Every wave is done with this item's LDS before the next item's DMAs.
    __syncthreads();
  }
  stamp();
}

// Whether a configuration has a BVEC (16-byte B copy) variant.
template <int NT, int BM, int BN, int BK, int WM_, int WN_>
constexpr bool dma_bvec_ok() {
  return BN == 64 && BN / WN_ == 32 && (BK * BN / 256) % (NT / 64) == 0 && BK % 4 == 0;
}

// Persistent grid of one kernel variant: k resident blocks on every CU.  The
// dispatcher fills free slots unevenly (on a 784-tile layer with 4 slots per
// CU, 72 CUs ran 4 full tiles and 184 ran 3), so the slot count per CU is made
// exactly k: dynamic LDS padding brings a block's LDS above 160 KiB / (k + 1)
// (and at most 160 KiB / k), and the grid fills every slot.
constexpr int kLdsPerCu = 160 * 1024;
template <typename Kern>
static void persistent_shape(Kern kern, int nt, int static_lds, int want_k, int& grid, size_t& pad) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, nt, 0) != hipSuccess || occ <= 0) occ = 1;
  int k = want_k > 0 && want_k < occ ? want_k : occ;
  pad = 0;
  if (k < occ) {
    const int need = kLdsPerCu / (k + 1) + 16;  // > 160 KiB / (k + 1)
    if (need > static_lds) pad = (size_t)(need - static_lds);
  }
  grid = k * cus;
}

template <int NT, int BM, int BN, int BK, int WM_, int WN_, int MINW, int STAGES, int HD, bool MKB, bool BV,
          bool DUAL = false>
static void launch_dma_variant(const DmaDesc& d, int tiles_m, int tiles_n, hipStream_t s,
                               const DmaDesc* d2 = nullptr) {
  auto kern = gemm_dma_kernel<NT, BM, BN, BK, WM_, WN_, MINW, STAGES, HD, MKB, BV, DUAL>;
  const int items = d.n_full + d.split_tiles * d.nkb;
  int grid = items;
  size_t pad = 0;
  if (d.persist_k > 0) {
    constexpr int static_lds = STAGES * (BM + BN) * BK * 4 + 16;  // stages + last_arrival
    persistent_shape(kern, NT, static_lds, d.persist_k, grid, pad);
    if (items < grid) grid = items;
  }
  hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), pad, s, d, d2 ? *d2 : d, tiles_m, tiles_n);
}

// Configurations with a dual-GEMM instance (64x64 tiles, 4 waves).
template <int NT, int BM, int BN, int BK, int WM_, int WN_>
constexpr bool dma_dual_ok() {
  return NT == 256 && BM == 64 && BN == 64;
}

template <int NT, int BM, int BN, int BK, int WM_, int WN_, int MINW, int STAGES, int HD>
static bool launch_dma_cfg(const DmaDesc& d, hipStream_t s, const DmaDesc* d2) {
  const int tiles_m = (d.M + BM - 1) / BM, tiles_n = (d.N + BN - 1) / BN;
  if (d2) {
    if constexpr (dma_dual_ok<NT, BM, BN, BK, WM_, WN_>()) {
      if constexpr (dma_bvec_ok<NT, BM, BN, BK, WM_, WN_>()) {
        if (d.bvec) {  // (both segments; launch_gemm_dma checked)
          launch_dma_variant<NT, BM, BN, BK, WM_, WN_, MINW, STAGES, HD, true, true, true>(d, tiles_m, tiles_n, s, d2);
          return true;
        }
      }
      launch_dma_variant<NT, BM, BN, BK, WM_, WN_, MINW, STAGES, HD, true, false, true>(d, tiles_m, tiles_n, s, d2);
      return true;
    }
    return false;
  }
  if constexpr (dma_bvec_ok<NT, BM, BN, BK, WM_, WN_>()) {
    if (d.bvec) {
      if (d.K > DKC)
        launch_dma_variant<NT, BM, BN, BK, WM_, WN_, MINW, STAGES, HD, true, true>(d, tiles_m, tiles_n, s);
      else
        launch_dma_variant<NT, BM, BN, BK, WM_, WN_, MINW, STAGES, HD, false, true>(d, tiles_m, tiles_n, s);
      return true;
    }
  }
  if (d.K > DKC)
    launch_dma_variant<NT, BM, BN, BK, WM_, WN_, MINW, STAGES, HD, true, false>(d, tiles_m, tiles_n, s);
  else
    launch_dma_variant<NT, BM, BN, BK, WM_, WN_, MINW, STAGES, HD, false, false>(d, tiles_m, tiles_n, s);
  return true;
}

// DMA tile configurations:
//   X(id, threads, BM, BN, BK, WAVES_M, WAVES_N, min waves/SIMD, stages, head steps)
// (head steps: MFMA steps of a K tile before its barrier; the rest carry the
// interleaved refill DMAs)
// The wave tile is (BM/WAVES_M) x (BN/WAVES_N).  All configurations produce
// bit-identical results (same KC-block summation order), so the choice is
// purely a performance one: dma_default_cfg below, or plan-time tuning.
#ifndef RTENHIP_DMA_CONFIGS  // (overridable for ISA inspection builds of one config)
#define RTENHIP_DMA_CONFIGS(X)          \
  X(0, 512, 128, 128, 16, 4, 2, 2, 3, 6)   \
  X(1, 256, 128, 128, 16, 2, 2, 2, 3, 6)   \
  X(2, 256, 64, 256, 16, 1, 4, 2, 3, 6)    \
  X(3, 128, 128, 64, 16, 2, 1, 2, 3, 6)    \
  X(4, 128, 64, 128, 16, 1, 2, 2, 3, 6)    \
  X(5, 64, 64, 64, 16, 1, 1, 2, 3, 6)      \
  X(6, 512, 256, 128, 16, 4, 2, 2, 3, 6)   \
  X(7, 256, 64, 64, 16, 2, 2, 4, 3, 6)     \
  X(8, 128, 64, 64, 16, 2, 1, 2, 3, 6)     \
  X(9, 256, 128, 64, 16, 4, 1, 2, 3, 6)    \
  X(10, 256, 64, 128, 16, 2, 2, 2, 3, 6)   \
  X(11, 512, 128, 128, 16, 4, 2, 2, 4, 6)  \
  X(12, 256, 128, 128, 16, 2, 2, 2, 4, 6)  \
  X(13, 256, 64, 64, 32, 2, 2, 3, 2, 6)    \
  X(14, 256, 64, 64, 16, 2, 2, 4, 4, 6)    \
  X(15, 512, 128, 64, 16, 4, 2, 4, 3, 6)   \
  X(16, 512, 64, 128, 16, 2, 4, 4, 3, 6)   \
  X(17, 128, 32, 64, 16, 1, 2, 4, 3, 6)    \
  X(18, 1024, 128, 128, 16, 4, 4, 4, 3, 6) \
  X(19, 256, 64, 64, 16, 2, 2, 5, 3, 6) \
  X(20, 256, 64, 64, 16, 2, 2, 4, 4, 2) \
  X(21, 256, 64, 64, 16, 2, 2, 4, 3, 2) \
  X(22, 256, 64, 64, 16, 2, 2, 4, 4, 4) \
  X(23, 128, 64, 64, 16, 2, 1, 2, 3, 2) \
  X(24, 256, 64, 64, 16, 2, 2, 6, 3, 6)
#endif

// Launch configuration cfg if it belongs to part PART of the split build
// (cfg % DMA_PARTS == PART; each gemm_dma_p*.hip instantiates one part).
constexpr int DMA_PARTS = 4;
template <int PART>
bool dma_launch_part(int cfg, const DmaDesc& d, hipStream_t s, const DmaDesc* d2) {
  switch (cfg) {
#define RTENHIP_DMA_PART_CASE(id, NT, BM, BN, BK, WMW, WNW, MINW, ST, HD) \
  case id:                                                              \
    if constexpr ((id) % DMA_PARTS == PART) {                            \
      return launch_dma_cfg<NT, BM, BN, BK, WMW, WNW, MINW, ST, HD>(d, s, d2); \
    } else {                                                            \
      return false;                                                     \
    }
    RTENHIP_DMA_CONFIGS(RTENHIP_DMA_PART_CASE)
#undef RTENHIP_DMA_PART_CASE
    default:
      return false;
  }
}
extern template bool dma_launch_part<0>(int, const DmaDesc&, hipStream_t, const DmaDesc*);
extern template bool dma_launch_part<1>(int, const DmaDesc&, hipStream_t, const DmaDesc*);
extern template bool dma_launch_part<2>(int, const DmaDesc&, hipStream_t, const DmaDesc*);
extern template bool dma_launch_part<3>(int, const DmaDesc&, hipStream_t, const DmaDesc*);

}  // namespace rtenhip
