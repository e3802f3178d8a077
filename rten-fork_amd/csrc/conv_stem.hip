// Small-C convolutions on MFMA with the im2col formed in LDS: the network
// stems -- ResNet-50's 7x7 / 2 (C = 3, K = 147, M = 64) and MobileNetV2's
// 3x3 / 2 (C = 3, K = 27, M = 32).
//
// The DMA GEMM runs a stem as an implicit GEMM whose B operand is gathered
// from HBM / L2 one k row of 64 columns per LDS-DMA instruction, through a
// per-k offset table: at K = 147 that is 10 K tiles of tiny, table-driven
// gathers per 64 x 64 tile, and each input value is fetched once per
// overlapping window.  The VALU direct kernel (conv_direct_lds_kernel) stages
// the input rows in LDS but spends 27 fma per output on the vector ALUs.
//
// Here a persistent workgroup (4 waves, two per CU) keeps the packed weights
// in LDS and walks bands of TR output rows of one image (band b, b + grid,
// ...):
//   1. the band's C x R input rows sit in LDS, zero outside the image (a
//      buffer load at an out-of-range offset returns 0), so padding is free;
//      the next band's rows are loaded into registers after this band's
//      MFMA chains, ahead of its stores, and written to LDS after them;
//   2. a band is TR * OW pixels = tiles of 32 pixels x MT tiles of 32
//      channels; item (tile, m) = tile * MT + m, wave w takes items w, w + 4,
//      ... (NT of them, one channel tile m per wave), each a
//      v_mfma_f32_32x32x2_f32 chain over k = (c, ky, kx): the A operand of
//      lane (pixel j, half h) at step s is the LDS word
//      pix(j) + off(2 s + h), off(k) = c R LW + ky LW + kx, with (c, ky, kx)
//      compile-time constants (the step loop is unrolled; k = K reads a zero
//      slot), the B operand one LDS word of the weights packed
//      [k pair][half][channel]; operands are loaded PD steps ahead;
//   3. bias, activation, and (MT = 2) 4 stores per lane and item of 4
//      adjacent pixels: pixels are the MFMA's rows (A and B above swap), so
//      an accumulator register group holds 4 of them; with MT = 1, 16 stores
//      per lane of 32 contiguous pixels.
// The host picks TR so that a band is at most 4 NT items (ResNet-50: TR = 4,
// 14 tiles x 2 -- seven items per wave; MobileNetV2: TR = 7, 25 tiles x 1).
// Measured (ResNet-50 b64 stem, profiles/r5_stem_mfma.txt): 0.194 ms per
// replayed conv vs 0.214 for the best DMA configuration; the MobileNetV2
// stem stays on the VALU direct kernel (the tuner times both).
// Summation contract (the GEMM's, src/gemm.rs:733-1050, as the DMA kernel
// states it): K <= 256 is one KC block, one fma chain per output from +0 over
// k in im2col order (VirtualIm2Col: k = (c * kh + ky) * kw + kx, padding
// read as 0), v_mfma_f32_32x32x2_f32 being bitwise that chain; then + bias,
// then the fused activation -- bit-identical to every other configuration.
#include <algorithm>
#include <type_traits>
#include <utility>

#include "common.h"
#include "ctx.h"
#include "vecmath.h"

namespace rtenhip {

namespace {

typedef float stem_f32x16 __attribute__((ext_vector_type(16)));

struct StemDesc {
  const float* x;   // [N, C, H, W] (unpadded)
  const float* wp;  // packed weights [KP / 2][2][MT * 32]
  const float* bias;
  float* y;         // [N, M, OH, OW]
  int M, H, W, OH, OW, pt, pl;
  int TR, R, LW;    // output rows per band, staged input rows, staged row width
  int tiles_y;      // bands per image
  int nbands;       // N * tiles_y
  int stage_n;      // C * R * LW staged floats
  int act;
  float lo, hi;
  int vec;          // OW % 4 == 0 and y 16-byte aligned: 4-pixel vector stores
  float* halo;      // POOL: [N, M, tiles_y, OW / 2] row-pooled last conv row of each band
};

constexpr int kStemThreads = 256;
// Items (32 x 32 output tiles) per wave and band: 7 for large batches; 2 when
// the batch has too few TR-row bands to fill the chip (batch 1: one output
// row per band, 112 workgroups instead of 28).
constexpr int kStemNT = 7, kStemNTSmall = 2;
// Staged rows per wave (a bound on C R / 4, in registers while the next band
// is loaded): ResNet-50's band (TR = 4, 3 x 13 rows of 232) needs 10;
// MobileNetV2's gets TR = 7 (3 x 15 rows) within 12.
constexpr int stem_rows_cap(int kh) { return kh == 7 ? 10 : 12; }
constexpr int kStemLdsFloats = 20480;  // 80 KiB: two workgroups per CU

template <int... Is, class F>
__device__ __forceinline__ void stem_static_for(std::integer_sequence<int, Is...>, F&& f) {
  (f(std::integral_constant<int, Is>{}), ...);
}

template <int C, int KH, int KW, int S, int MT, int NT, bool POOL = false>
__global__ __launch_bounds__(kStemThreads, 2) void conv_stem_kernel(StemDesc d) {
  constexpr int K = C * KH * KW;
  constexpr int KP = (K + 1) & ~1;  // k pairs of the 32x32x2 MFMA
  constexpr int NS = KP / 2;
  constexpr int MW = MT * 32;       // packed channel rows
  constexpr int SR = stem_rows_cap(KH);
  // Pixels as the MFMA's rows (vector stores in the epilogue) with two
  // channel tiles; with one, the 4-pixel groups' addresses and guards spill.
  constexpr bool PXR = MT == 2;
  extern __shared__ float4 stem_lds4[];
  float* lds = reinterpret_cast<float*>(stem_lds4);
  float* wl = lds;                  // [NS][2][MW]
  float* xs = lds + KP * MW;        // [C][R][LW], then one zero slot
  float* bl = xs + d.stage_n + 1;   // [MW] bias (0 past M, or without bias)
  float* ex = bl + MW;              // POOL: [MT][4 rows][32 channels] column exchange
  const int zs = d.stage_n;         // the zero slot (index into xs)
  const int t = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int lane = t & 63;
  const int half = lane >> 5, j = lane & 31;
  const int RL = d.R * d.LW;

  // Staging: staged row q = c R + r (of C R) goes to wave q % 4, its lanes
  // covering columns lane + 64 jj (LW <= 256).  The row's image offset and
  // validity are wave-uniform (scalar ALU); a column outside the image gets
  // an out-of-range offset (the load returns 0).
  auto band_loads = [&](int b, float (&xv)[SR][4]) __attribute__((always_inline)) {
    const int img = b / d.tiles_y;
    const int iy0 = (b - img * d.tiles_y) * d.TR * S - d.pt;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(d.x + (int64_t)img * C * d.H * d.W), 0, C * d.H * d.W * 4, 0x00020000);
    // (opaque per band, so the per-column terms are formed here rather than
    // hoisted out of the band loop and held through the MFMA chains)
    int ix0 = lane - d.pl;
    asm volatile("" : "+v"(ix0));
#pragma unroll
    for (int i = 0; i < SR; i++) {
      const int q = wave + 4 * i;
      const int c = (q >= d.R) + (C > 2 && q >= 2 * d.R);
      const int iy = iy0 + q - c * d.R;
      const bool row_ok = q < C * d.R && iy >= 0 && iy < d.H;
      const int rowoff = (c * d.H + iy) * d.W;
#pragma unroll
      for (int jj = 0; jj < 4; jj++) {
        const int ix = ix0 + 64 * jj;
        const bool ok = row_ok && ix >= 0 && ix < d.W;
        const uint32_t off = ok ? (uint32_t)(rowoff + ix) * 4u : 0x80000000u;
        xv[i][jj] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, off, 0, 0));
      }
    }
  };
  auto band_store = [&](const float (&xv)[SR][4]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < SR; i++) {
      const int q = wave + 4 * i;
      if (q < C * d.R) {
#pragma unroll
        for (int jj = 0; jj < 4; jj++)
          if (lane + 64 * jj < d.LW) xs[q * d.LW + lane + 64 * jj] = xv[i][jj];
      }
    }
  };

  // Weights and the first band.
  float xv[SR][4];
  int b = blockIdx.x;
  {
    // Weights straight into LDS (global_load_lds_dwordx4: 1 KiB per wave
    // instruction, no registers), overlapping the first band's loads.
    constexpr int NWF = KP * MW;  // a multiple of 32 floats
#pragma unroll
    for (int c0 = 0; c0 < NWF; c0 += 4 * 256) {
      const int idx = c0 + wave * 256 + lane * 4;
      if (idx < NWF)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(d.wp + idx),
                                         (__attribute__((address_space(3))) void*)(wl + c0 + wave * 256), 16, 0, 0);
    }
    band_loads(b, xv);
    band_store(xv);
    if (t == 0) xs[zs] = 0.f;
    // (the epilogue reads the bias from LDS: a global load there would wait,
    // through the in-order vmcnt, for every store issued before it)
    if (t < MW) bl[t] = (d.bias && t < d.M) ? d.bias[t] : 0.f;
    // this wave's weight DMAs have landed before the barrier below
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }

  // This wave's channel tile.
  const int m = MT == 1 ? 0 : (wave & 1);

  for (; b < d.nbands; b += gridDim.x) {
    __syncthreads();  // xs holds band b
    const int img = b / d.tiles_y;
    const int oy0 = (b - img * d.tiles_y) * d.TR;
    const int opb = min(d.TR, d.OH - oy0) * d.OW;  // output pixels of the band

    int pb[NT];
    bool pok[NT];
#pragma unroll
    for (int i = 0; i < NT; i++) {
      if constexpr (POOL) {
        // Tile t = 4 rows x 8 columns (the band's rows; waves 0 / 1 take
        // tiles 0..6, waves 2 / 3 tiles 7..13), pixel j = (row j / 8,
        // column 8 t + j % 8): an accumulator lane then holds a 4 x 4 patch.
        const int t = (wave >> 1) * NT + i;
        pok[i] = true;
        pb[i] = (j >> 3) * S * d.LW + (8 * t + (j & 7)) * S;
      } else {
        const int p = ((wave / MT) + (4 / MT) * i) * 32 + j;
        pok[i] = p < opb;
        const int pc = pok[i] ? p : 0;
        const int oyl = pc / d.OW, ox = pc - oyl * d.OW;
        pb[i] = oyl * S * d.LW + ox * S;
      }
    }
    stem_f32x16 acc[NT];
#pragma unroll
    for (int i = 0; i < NT; i++) acc[i] = (stem_f32x16){0};
    // Operands of step s (k = 2 s + half) land in slot s % (PD + 1), PD
    // steps ahead of their MFMAs.
    constexpr int PD = 2;
    float bq[PD + 1][NT], aq[PD + 1];
    // The per-step offset selects below depend on the lane's half; redefined
    // here each band so they are not all hoisted out of the band loop (74
    // live registers) but formed one per step.
    int hsel = half;
    asm volatile("" : "+v"(hsel));
    auto load = [&](auto s_) __attribute__((always_inline)) {
      constexpr int s = decltype(s_)::value;
      if constexpr (s < NS) {
        constexpr int k0 = 2 * s, k1 = 2 * s + 1;
        constexpr int c0 = k0 / (KH * KW), y0 = (k0 / KW) % KH, x0 = k0 % KW;
        constexpr int c1 = k1 / (KH * KW), y1 = (k1 / KW) % KH, x1 = k1 % KW;
        const int off0 = c0 * RL + y0 * d.LW + x0;
        const int off1 = c1 * RL + y1 * d.LW + x1;
        int off = hsel ? off1 : off0;
        // (opaque per step: no per-(tile, c, ky) row bases kept live across steps)
        asm volatile("" : "+v"(off));
#pragma unroll
        for (int i = 0; i < NT; i++) {
          // k = K (odd K, last step) reads the zero slot.
          const int addr = (k1 >= K && hsel) ? zs : pb[i] + off;
          bq[s % (PD + 1)][i] = xs[addr];
        }
        aq[s % (PD + 1)] = wl[(s * 2 + half) * MW + m * 32 + j];
      }
    };
    stem_static_for(std::make_integer_sequence<int, PD>{}, load);
    stem_static_for(std::make_integer_sequence<int, NS>{}, [&](auto s_) __attribute__((always_inline)) {
      constexpr int s = decltype(s_)::value;
      load(std::integral_constant<int, s + PD>{});
#pragma unroll
      for (int i = 0; i < NT; i++)
        if constexpr (PXR)
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(bq[s % (PD + 1)][i], aq[s % (PD + 1)], acc[i], 0, 0, 0);
        else
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(aq[s % (PD + 1)], bq[s % (PD + 1)][i], acc[i], 0, 0, 0);
      // (keeps the scheduler from sinking the loads ahead to their MFMAs)
      __builtin_amdgcn_sched_barrier(0);
    });

    // The next band's rows are loaded now, ahead of this band's stores (a
    // load issued after them would wait for them all: vmcnt is in order),
    // and written to LDS once every wave is done with this band.
    const int nb = b + (int)gridDim.x;
    if (nb < d.nbands) band_loads(nb, xv);

    // Epilogue: pixels are the MFMA's rows (A = the im2col tile), so element
    // 4 q + r of lane (j, half) is pixel 8 q + 4 half + r of the tile,
    // channel m 32 + j: four adjacent pixels of one channel per q, one
    // 16-byte store when d.vec (band pixels are contiguous in the plane).
    const int64_t oplane = (int64_t)d.OH * d.OW;
    float* yb = d.y + (int64_t)img * d.M * oplane + (int64_t)oy0 * d.OW;
    if constexpr (POOL) {
      // MaxPool 3x3 / 2, pads 1 (pooling.rs:104-238) on the band's Relu'd
      // conv outputs, in registers.  Lane (channel j, half h) of item i holds
      // rows 0..3 x columns 8 t + 4 h .. + 3; pooled column 4 t + 2 h + u
      // takes columns 8 t + 4 h + 2 u - 1 .. + 1, the left one from the
      // other half (h = 1) or the previous tile (h = 0: the previous item, or
      // for tile 7 wave 0 / 1's tile 6 through LDS; tile 0 has only padding
      // there).  Pooled row 2 b + 1 (conv rows 4 b + 1 .. 3) is complete in
      // the band; row 2 b gets rows 4 b, 4 b + 1 here and conv row 4 b - 1
      // from band b - 1's halo row (stem_pool_finish_kernel).  The values are
      // Relu outputs -- never NaN, never -0 -- so their max does not depend
      // on the order of the folds: the reference's (ky, kx) fold gives the
      // same bits.
      const int ch = m * 32 + j;  // (M == 64 == MT * 32)
      const float bv = bl[ch];
      const int PW = d.OW >> 1;
      const int band = b - img * d.tiles_y;
      float* yc = d.y + ((int64_t)img * d.M + ch) * (int64_t)(d.OH >> 1) * PW + (int64_t)(2 * band) * PW;
      float* hc = d.halo + (((int64_t)img * d.M + ch) * d.tiles_y + band) * PW;
      auto relu_v = [&](const stem_f32x16& a, int q, int r) __attribute__((always_inline)) {
        float v = a[4 * q + r];
        if (d.bias) v = __fadd_rn(v, bv);
        return rust_max(v, 0.f);
      };
      float prev[4];
      if (wave < 2) {  // publish column 55 (tile 6's last) for tile 7's left neighbour
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const float sw = __shfl_xor(relu_v(acc[NT - 1], q, 3), 32);
          if (half == 0) ex[(m * 4 + q) * 32 + j] = sw;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
      for (int q = 0; q < 4; q++) prev[q] = wave >= 2 ? ex[(m * 4 + q) * 32 + j] : 0.f;
#pragma unroll
      for (int i = 0; i < NT; i++) {
        const int t = (wave >> 1) * NT + i;
        float hm[4][2];
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const float v0 = relu_v(acc[i], q, 0), v1 = relu_v(acc[i], q, 1);
          const float v2 = relu_v(acc[i], q, 2), v3 = relu_v(acc[i], q, 3);
          const float sw = __shfl_xor(v3, 32);  // h = 1: column 8 t + 3; h = 0: 8 t + 7 (next tile's left)
          const float left = half ? sw : prev[q];
          float h0 = fmaxf(v0, v1);
          if (half || t > 0) h0 = fmaxf(left, h0);
          hm[q][0] = h0;
          hm[q][1] = fmaxf(fmaxf(v1, v2), v3);
          prev[q] = sw;
        }
        const int px = 4 * t + 2 * half;
        *reinterpret_cast<float2*>(yc + PW + px) =
            make_float2(fmaxf(fmaxf(hm[1][0], hm[2][0]), hm[3][0]), fmaxf(fmaxf(hm[1][1], hm[2][1]), hm[3][1]));
        *reinterpret_cast<float2*>(yc + px) = make_float2(fmaxf(hm[0][0], hm[1][0]), fmaxf(hm[0][1], hm[1][1]));
        if (band + 1 < d.tiles_y) *reinterpret_cast<float2*>(hc + px) = make_float2(hm[3][0], hm[3][1]);
      }
    } else if constexpr (!PXR) {
      // (channels as rows: element 4 q + r is channel m 32 + 8 q + 4 half + r,
      // pixel j of the tile)
#pragma unroll
      for (int i = 0; i < NT; i++) {
        if (!pok[i]) continue;
        float* yp = yb + ((wave / MT) + (4 / MT) * i) * 32 + j;
#pragma unroll
        for (int e = 0; e < 16; e++) {
          const int c = m * 32 + 8 * (e >> 2) + 4 * half + (e & 3);
          if (c < d.M) {
            float v = acc[i][e];
            if (d.bias) v = __fadd_rn(v, bl[c]);
            if (d.act == RTENHIP_ACT_RELU) v = rust_max(v, 0.f);
            else if (d.act == RTENHIP_ACT_CLIP) v = rust_clamp(v, d.lo, d.hi);
            yp[(int64_t)c * oplane] = v;
          }
        }
      }
    } else if (m * 32 + j < d.M) {
      const int ch = m * 32 + j;
      const float bv = bl[ch];
      float* yc = yb + (int64_t)ch * oplane;
#pragma unroll
      for (int i = 0; i < NT; i++) {
        const int tp = ((wave / MT) + (4 / MT) * i) * 32;
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int p0 = tp + 8 * q + 4 * half;
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; r++) {
            v[r] = acc[i][4 * q + r];
            if (d.bias) v[r] = __fadd_rn(v[r], bv);
            if (d.act == RTENHIP_ACT_RELU) v[r] = rust_max(v[r], 0.f);
            else if (d.act == RTENHIP_ACT_CLIP) v[r] = rust_clamp(v[r], d.lo, d.hi);
          }
          if (d.vec) {
            if (p0 < opb) *reinterpret_cast<float4*>(yc + p0) = make_float4(v[0], v[1], v[2], v[3]);
          } else {
#pragma unroll
            for (int r = 0; r < 4; r++)
              if (p0 + r < opb) yc[p0 + r] = v[r];
          }
        }
      }
    }
    if (nb < d.nbands) {
      __syncthreads();  // every wave is done with band b
      band_store(xv);
    }
  }
}

// Pooled row 2 b of every (image, channel), b >= 1: the band's partial (conv
// rows 4 b, 4 b + 1) and band b - 1's halo (conv row 4 b - 1, row-pooled),
// 16 bytes per thread.  (Pooled row 0's window has only padding above.)
__global__ void stem_pool_finish_kernel(float* __restrict__ y, const float* __restrict__ halo, int64_t n4,
                                        int PW4, int tiles_y) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const int c4 = (int)(i % PW4);
  const int64_t r = i / PW4;                  // (image, channel) * (tiles_y - 1) + b - 1
  const int64_t plane = r / (tiles_y - 1);
  const int b = (int)(r - plane * (tiles_y - 1)) + 1;
  float4* yp = reinterpret_cast<float4*>(y) + (plane * (2 * tiles_y) + 2 * b) * PW4 + c4;
  const float4 h = reinterpret_cast<const float4*>(halo)[(plane * tiles_y + b - 1) * PW4 + c4];
  float4 v = *yp;
  v.x = fmaxf(v.x, h.x);
  v.y = fmaxf(v.y, h.y);
  v.z = fmaxf(v.z, h.z);
  v.w = fmaxf(v.w, h.w);
  *yp = v;
}

// w [M][K] -> [KP / 2][2][MT * 32], zero past M and K.
__global__ void pack_stem_kernel(const float* __restrict__ w, float* __restrict__ out, int M, int K, int KP, int MW) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= KP * MW) return;
  const int kk = i / MW, m = i - kk * MW;  // kk = 2 s + half = k
  out[i] = (m < M && kk < K) ? w[(int64_t)m * K + kk] : 0.f;
}

struct StemShape {
  int TR, R, LW, tiles_y, stage_n, NT;
};
int stem_mt(int64_t M) { return M <= 32 ? 1 : (M <= 64 ? 2 : 0); }

// Output rows per band: the most whose tiles fit 4 waves x NT items, with the
// staged rows within the per-thread register stage and the LDS budget; the
// small-item variant when the large one leaves fewer bands than 2 per CU.
StemShape stem_shape(int C, int kh, int kw, int S, int OH, int OW, int64_t M, int64_t N, int cus) {
  StemShape e{};
  const int mt = stem_mt(M);
  if (mt == 0 || OW < 1 || OH < 1) return e;
  const int wfloats = ((C * kh * kw + 1) & ~1) * mt * 32;
  const int lw = ((OW - 1) * S + kw + 3) & ~3;
  auto fits = [&](int tr, int nt) {
    const int tiles = (tr * OW + 31) / 32;
    const int staged = C * ((tr - 1) * S + kh) * lw;
    return tiles * mt <= 4 * nt && C * ((tr - 1) * S + kh) <= 4 * stem_rows_cap(kh) && lw <= 256 &&
           wfloats + staged + 1 + mt * 32 <= kStemLdsFloats;
  };
  auto rows_for = [&](int nt) {
    int r = 0;
    while (r < OH && fits(r + 1, nt)) r++;
    return r;
  };
  int nt = kStemNT, tr = rows_for(nt);
  if (tr >= 1 && N * ((OH + tr - 1) / tr) < 2 * (int64_t)cus) {
    const int trs = rows_for(kStemNTSmall);
    if (trs >= 1) {
      nt = kStemNTSmall;
      tr = trs;
    }
  }
  e.NT = nt;
  if (tr < 1) return e;
  e.TR = tr;
  e.R = (tr - 1) * S + kh;
  e.LW = lw;
  e.tiles_y = (OH + tr - 1) / tr;
  e.stage_n = C * e.R * lw;
  return e;
}

int stem_grid_cap() {
  static int cap = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    return 2 * cus;  // two workgroups per CU
  }();
  return cap;
}

}  // namespace

// Stem + MaxPool 3x3 / 2 / pads 1 in one pass (conv_stem_kernel<..., POOL>):
// ResNet-50's 7x7 / 2 stem (C = 3, M = 64, 112 x 112 outputs) with a fused
// Relu, at batches whose bands are 4 output rows of 7 items per wave.
bool conv_stem_pool_eligible(const ConvPlan& g) {
  if (!(g.C == 3 && g.kh == 7 && g.kw == 7 && g.sh == 2 && g.sw == 2 && g.O == 64 && g.groups == 1 && g.dh == 1 &&
        g.dw == 1 && g.ow == 112 && g.oh % 4 == 0 && !g.one_d))
    return false;
  const StemShape e = stem_shape((int)g.C, (int)g.kh, (int)g.kw, (int)g.sh, (int)g.oh, (int)g.ow, g.O, g.N,
                                 stem_grid_cap() / 2);
  const int64_t KP = 148;
  return e.TR == 4 && e.NT == kStemNT && KP * 64 + e.stage_n + 1 + 64 + 256 <= kStemLdsFloats &&
         g.C * g.H * g.W < (int64_t(1) << 29) && g.N * e.tiles_y < (int64_t(1) << 31);
}

int64_t stem_pool_halo_floats(const ConvPlan& g) { return g.N * g.O * (g.oh / 4) * (g.ow / 2); }

rtenhip_status conv_stem_pool(const ConvDmaArgs& a, float* pooled, float* halo, hipStream_t s) {
  ConvPlan g{};
  g.N = a.N;
  g.C = a.C;
  g.H = a.H;
  g.W = a.W;
  g.O = a.O;
  g.kh = a.kh;
  g.kw = a.kw;
  g.sh = a.sh;
  g.sw = a.sw;
  g.dh = a.dh;
  g.dw = a.dw;
  g.oh = a.oh;
  g.ow = a.ow;
  g.groups = a.groups;
  if (!conv_stem_pool_eligible(g) || !a.x_unpadded || a.residual || a.bn || a.act != RTENHIP_ACT_RELU ||
      ((uintptr_t)pooled & 15) || ((uintptr_t)halo & 15))
    return fail(RTENHIP_INVALID_VALUE, "stem + max pool: unsupported layout");
  const StemShape e = stem_shape((int)a.C, (int)a.kh, (int)a.kw, (int)a.sh, (int)a.oh, (int)a.ow, a.O, a.N,
                                 stem_grid_cap() / 2);
  StemDesc d{};
  d.x = a.x_unpadded;
  d.wp = a.packed_w;
  d.bias = a.bias;
  d.y = pooled;
  d.halo = halo;
  d.M = (int)a.O;
  d.H = (int)a.H;
  d.W = (int)a.W;
  d.OH = (int)a.oh;
  d.OW = (int)a.ow;
  d.pt = (int)a.pad_t;
  d.pl = (int)a.pad_l;
  d.TR = e.TR;
  d.R = e.R;
  d.LW = e.LW;
  d.tiles_y = e.tiles_y;
  d.nbands = (int)(a.N * e.tiles_y);
  d.stage_n = e.stage_n;
  d.act = a.act;
  d.vec = 1;
  const size_t lds = (size_t)(148 * 64 + e.stage_n + 1 + 64 + 256) * 4;
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_stem_kernel<3, 7, 7, 2, 2, kStemNT, true>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, kStemLdsFloats * 4);
  RTENHIP_HIP_CHECK(attr);
  hipLaunchKernelGGL((conv_stem_kernel<3, 7, 7, 2, 2, kStemNT, true>),
                     dim3((unsigned)std::min(d.nbands, stem_grid_cap())), dim3(kStemThreads), lds, s, d);
  RTENHIP_LAUNCH_CHECK();
  const int PW4 = (int)(a.ow / 2 / 4);
  const int64_t n4 = a.N * a.O * (e.tiles_y - 1) * PW4;
  if (n4 > 0) {
    hipLaunchKernelGGL(stem_pool_finish_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, pooled, halo,
                       n4, PW4, e.tiles_y);
    RTENHIP_LAUNCH_CHECK();
  }
  return RTENHIP_OK;
}

bool conv_stem_eligible(const ConvPlan& g, bool padded_out) {
  const bool resnet = g.C == 3 && g.kh == 7 && g.kw == 7 && g.sh == 2 && g.sw == 2;
  const bool mnv2 = g.C == 3 && g.kh == 3 && g.kw == 3 && g.sh == 2 && g.sw == 2;
  if (!(resnet || mnv2) || g.groups != 1 || g.dh != 1 || g.dw != 1 || padded_out) return false;
  const StemShape e = stem_shape((int)g.C, (int)g.kh, (int)g.kw, (int)g.sh, (int)g.oh, (int)g.ow, g.O, g.N,
                                 stem_grid_cap() / 2);
  return e.TR > 0 && g.C * g.H * g.W < (int64_t(1) << 29) && g.N * e.tiles_y < (int64_t(1) << 31) &&
         g.N * g.O * g.oh * g.ow < (int64_t(1) << 40);
}

int64_t stem_weight_floats(int64_t M, int64_t K) { return ((K + 1) & ~int64_t(1)) * stem_mt(M) * 32; }

rtenhip_status pack_stem_weights(const float* w, int64_t M, int64_t K, float* out, hipStream_t s) {
  const int KP = (int)((K + 1) & ~int64_t(1)), MW = stem_mt(M) * 32;
  if (MW == 0) return fail(RTENHIP_UNSUPPORTED_VALUE, "stem conv: more than 64 output channels");
  hipLaunchKernelGGL(pack_stem_kernel, dim3((unsigned)((KP * MW + 255) / 256)), dim3(256), 0, s, w, out, (int)M,
                     (int)K, KP, MW);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

rtenhip_status conv_stem(const ConvDmaArgs& a, hipStream_t s) {
  const bool resnet = a.C == 3 && a.kh == 7 && a.kw == 7 && a.sh == 2 && a.sw == 2;
  const bool mnv2 = a.C == 3 && a.kh == 3 && a.kw == 3 && a.sh == 2 && a.sw == 2;
  const int mt = stem_mt(a.O);
  if (!(resnet || mnv2) || a.groups != 1 || a.dh != 1 || a.dw != 1 || mt == 0 || !a.x_unpadded || a.residual ||
      a.bn || a.y_off != 0 || (a.y_row != 0 && a.y_row != a.ow) || a.y_img != a.O * a.oh * a.ow)
    return fail(RTENHIP_INVALID_VALUE, "stem conv: unsupported layout");
  const StemShape e = stem_shape((int)a.C, (int)a.kh, (int)a.kw, (int)a.sh, (int)a.oh, (int)a.ow, a.O, a.N,
                                 stem_grid_cap() / 2);
  if (e.TR == 0 || a.C * a.H * a.W >= (int64_t(1) << 29) || a.N * e.tiles_y >= (int64_t(1) << 31))
    return fail(RTENHIP_UNSUPPORTED_VALUE, "stem conv: shape outside the kernel's bounds");
  StemDesc d{};
  d.x = a.x_unpadded;
  d.wp = a.packed_w;
  d.bias = a.bias;
  d.y = a.y;
  d.M = (int)a.O;
  d.H = (int)a.H;
  d.W = (int)a.W;
  d.OH = (int)a.oh;
  d.OW = (int)a.ow;
  d.pt = (int)a.pad_t;
  d.pl = (int)a.pad_l;
  d.TR = e.TR;
  d.R = e.R;
  d.LW = e.LW;
  d.tiles_y = e.tiles_y;
  d.nbands = (int)(a.N * e.tiles_y);
  d.stage_n = e.stage_n;
  d.act = a.act;
  d.lo = a.lo;
  d.hi = a.hi;
  d.vec = a.ow % 4 == 0 && ((uintptr_t)a.y & 15) == 0;
  const int64_t K = a.C * a.kh * a.kw, KP = (K + 1) & ~int64_t(1);
  const size_t lds = (size_t)(KP * mt * 32 + e.stage_n + 1 + mt * 32) * 4;
  const dim3 grid((unsigned)std::min(d.nbands, stem_grid_cap())), blk(kStemThreads);
  // (over 64 KiB of dynamic LDS: opted in once per instantiation)
#define STEM_LAUNCH(KH, MT, NT)                                                                            \
  {                                                                                                        \
    static const hipError_t attr = hipFuncSetAttribute((const void*)conv_stem_kernel<3, KH, KH, 2, MT, NT>, \
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,         \
                                                       kStemLdsFloats * 4);                                \
    RTENHIP_HIP_CHECK(attr);                                                                               \
    hipLaunchKernelGGL((conv_stem_kernel<3, KH, KH, 2, MT, NT>), grid, blk, lds, s, d);                    \
  }
  const bool small = e.NT == kStemNTSmall;
  if (resnet && mt == 2) {
    if (small) STEM_LAUNCH(7, 2, kStemNTSmall) else STEM_LAUNCH(7, 2, kStemNT)
  } else if (resnet) {
    if (small) STEM_LAUNCH(7, 1, kStemNTSmall) else STEM_LAUNCH(7, 1, kStemNT)
  } else if (mt == 1) {
    if (small) STEM_LAUNCH(3, 1, kStemNTSmall) else STEM_LAUNCH(3, 1, kStemNT)
  } else {
    if (small) STEM_LAUNCH(3, 2, kStemNTSmall) else STEM_LAUNCH(3, 2, kStemNT)
  }
#undef STEM_LAUNCH
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

}  // namespace rtenhip
