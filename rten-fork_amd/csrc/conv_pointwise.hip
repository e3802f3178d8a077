// Pointwise (1x1, stride 1, unpadded, ungrouped) convolution on the vector
// ALUs, for the thin layers where a 64x64 MFMA tile is mostly padding and
// the layer is bound by its activation traffic (MobileNetV2's expand /
// project convs: M or K of 16..64 over 0.4..1.6 M pixels).
//
// Reference: conv_2d_pointwise (src/ops/conv.rs:24-68) runs, per image,
// gemm_uninit_bias(W[O, C], X_n[C, HW], bias); with K = C <= 256 the GEMM
// has one KC block (gemm.rs:546-571), so each output is the k-ordered fma
// chain from zero (kernels.rs:206-316), then + bias (gemm.rs:1034-1047).
// The fused residual Add and Relu / Clip / Gelu follow, as in the DMA GEMM's
// epilogue (gemm_dma_kernel.h), so both paths give bit-identical outputs.
//
// Layout: a lane owns 4 consecutive pixels of one image (P % 4 == 0) and
// MC output channels per pass: MC x 4 accumulators in VGPRs, one 16-byte x
// load per k (coalesced: a wave reads 1 KB of one channel row), the MC
// weights of that k as scalar operands (weights are transposed to [K][M]
// once at plan time so one k's weights are contiguous), packed f32 FMAs on
// pixel pairs.  Outputs are 16-byte stores, 1 KB per wave-instruction.
// Passes over further channel chunks re-read x from L2.
#include <algorithm>

#include "common.h"
#include "ctx.h"
#include "fastdiv_dev.h"
#include "vecmath.h"

// Timing-experiment builds only (build_pw_exp.sh, never shipped): 1 = stores
// skipped (kept live by an impossible condition), 2 = one FMA chain per
// pass instead of MC (the others copy it).
#ifndef RTENHIP_PW_EXPERIMENT
#define RTENHIP_PW_EXPERIMENT 0
#endif

namespace rtenhip {

typedef float f32x2 __attribute__((ext_vector_type(2)));

// Pointers are separate __restrict__ kernel arguments: the weight reads are
// then provably unclobbered by the output stores and become scalar loads.
struct PwDesc {
  int M, Mpad, K, P4;  // wt row stride Mpad (M rounded up to 32, zero columns); P4 = P / 4
  int groups4;       // N * P / 4
  int act;
  float lo, hi;
};

__device__ __forceinline__ float pw_act(float x, int act, float lo, float hi) {
  if (act == RTENHIP_ACT_RELU) {
    x = fmaxf(x, 0.f);
  } else if (act == RTENHIP_ACT_CLIP) {
    x = rust_clamp(x, lo, hi);
  } else if (act == RTENHIP_ACT_GELU) {
    x = vm_gelu(x);
  }
  return x;
}

// KX > 0: K <= KX, the lane's x column (K float4) is loaded once into VGPRs
// and every channel chunk reuses it (expand convs: K 16..32, M up to 192);
// KX == 0: x streamed per chunk, KU loads in flight.
template <int MC, int KX>
__global__ __launch_bounds__(256) void conv_pw_valu_kernel(
    const float* __restrict__ x,         // [N][K][P]
    const float* __restrict__ wt,        // [K][Mpad] (transposed weights)
    const float* __restrict__ bias,      // [M] or null
    const float* __restrict__ residual,  // [N][M][P] or null
    float* __restrict__ y,               // [N][M][P]
    PwDesc d) {
  constexpr int KU = 8;  // x loads in flight per lane
  const int gi = (int)blockIdx.x * 256 + (int)threadIdx.x;  // < 2^31 (eligibility)
  if (gi >= d.groups4) return;
  const int img = (int)((uint32_t)gi / (uint32_t)d.P4);
  const int p = (gi - img * d.P4) * 4;
  const int64_t P = (int64_t)d.P4 * 4;
  const float* __restrict__ xp = x + (int64_t)img * d.K * P + p;
  const int nchunk = (d.M + MC - 1) / MC;
  float4 xr[KX > 0 ? KX : 1];
  if constexpr (KX > 0) {
#pragma unroll
    for (int j = 0; j < KX; j++)  // unconditional (clamped) loads: all in flight together
      xr[j] = *(const float4*)(xp + (int64_t)min(j, d.K - 1) * P);
    // Opaque to the optimizer: the column stays in VGPRs instead of being
    // re-loaded in every chunk pass.
#pragma unroll
    for (int j = 0; j < KX; j++) {
      float e0 = xr[j].x, e1 = xr[j].y, e2 = xr[j].z, e3 = xr[j].w;
      asm volatile("" : "+v"(e0), "+v"(e1), "+v"(e2), "+v"(e3));
      xr[j] = make_float4(e0, e1, e2, e3);
    }
  }
  for (int ch = blockIdx.y; ch < nchunk; ch += gridDim.y) {
    const int o0 = ch * MC;
    f32x2 acc[MC][2];
#pragma unroll
    for (int o = 0; o < MC; o++) acc[o][0] = acc[o][1] = (f32x2){0.f, 0.f};
    // The last partial chunk reads the zero padding columns of wt (their
    // results are not stored).
    const float* __restrict__ wk = wt + o0;
    const int olim = d.M - 1 - o0;
    if constexpr (KX > 0) {
#pragma unroll
      for (int j = 0; j < KX; j++) {
        if (j < d.K) {
          const f32x2 xa = {xr[j].x, xr[j].y}, xb = {xr[j].z, xr[j].w};
          const float* __restrict__ wr = wk + j * d.Mpad;
#pragma unroll
          for (int o = 0; o < MC; o++) {
            const f32x2 wv = {wr[o], wr[o]};
            acc[o][0] = __builtin_elementwise_fma(wv, xa, acc[o][0]);
            acc[o][1] = __builtin_elementwise_fma(wv, xb, acc[o][1]);
          }
        }
      }
    }
    for (int k0 = 0; KX == 0 && k0 < d.K; k0 += KU) {
      float4 xv[KU];
#pragma unroll
      for (int j = 0; j < KU; j++)
        xv[j] = *(const float4*)(xp + (int64_t)min(k0 + j, d.K - 1) * P);
#pragma unroll
      for (int j = 0; j < KU; j++) {
        if (k0 + j >= d.K) break;
        const f32x2 xa = {xv[j].x, xv[j].y}, xb = {xv[j].z, xv[j].w};
        const float* __restrict__ wr = wk + (k0 + j) * d.Mpad;
#pragma unroll
        for (int o = 0; o < MC; o++) {
          const f32x2 wv = {wr[o], wr[o]};
          acc[o][0] = __builtin_elementwise_fma(wv, xa, acc[o][0]);
          acc[o][1] = __builtin_elementwise_fma(wv, xb, acc[o][1]);
        }
      }
    }
    float* __restrict__ yp = y + ((int64_t)img * d.M + o0) * P + p;
    const float* __restrict__ rp = residual ? residual + ((int64_t)img * d.M + o0) * P + p : nullptr;
#pragma unroll
    for (int o = 0; o < MC; o++) {
      if (o > olim) continue;
      float4 v = make_float4(acc[o][0].x, acc[o][0].y, acc[o][1].x, acc[o][1].y);
      if (bias) {
        const float b = bias[o0 + o];
        v.x = __fadd_rn(v.x, b);
        v.y = __fadd_rn(v.y, b);
        v.z = __fadd_rn(v.z, b);
        v.w = __fadd_rn(v.w, b);
      }
      if (rp) {
        const float4 r = *(const float4*)(rp + (int64_t)o * P);
        v.x = __fadd_rn(v.x, r.x);
        v.y = __fadd_rn(v.y, r.y);
        v.z = __fadd_rn(v.z, r.z);
        v.w = __fadd_rn(v.w, r.w);
      }
      v.x = pw_act(v.x, d.act, d.lo, d.hi);
      v.y = pw_act(v.y, d.act, d.lo, d.hi);
      v.z = pw_act(v.z, d.act, d.lo, d.hi);
      v.w = pw_act(v.w, d.act, d.lo, d.hi);
      *(float4*)(yp + (int64_t)o * P) = v;
    }
  }
}

// Direct small-K convolution on the vector ALUs (MobileNetV2's stem: 3x3 /
// stride 2 over 3 channels, K = 27, M = 32, 1.6 M output pixels at batch
// 128): the im2col GEMM's B operand is mostly gather and its output pass is
// bound by the stores, so a lane computes 4 consecutive output pixels of one
// row for MC channels straight from the input rows, with the padding handled
// in place (no padded copy of the input).  Chain order is the reference's
// im2col row order k = (c, ky, kx) (im2col.rs:104-124); padding positions
// contribute fma(w, 0, acc) exactly as the masked zeros of VirtualIm2Col
// do in the GEMM kernel.
struct DirDesc {
  int C, H, W, kh, sh, dh, pt, pl, OH, OW4;
  int64_t x_elems;
  int M, Mpad, groups4;  // groups4 = N * OH * OW / 4
  int act;
  float lo, hi;
};

// CC, KH > 0: channel count and kernel height known at compile time (the
// 3-channel image stems), so all C*KH input rows are loaded up front.
template <int MC, int KW, int SW, int CC, int KH>
__global__ __launch_bounds__(256) void conv_direct_valu_kernel(const float* __restrict__ x,
                                                               const float* __restrict__ wt,
                                                               const float* __restrict__ bias,
                                                               const float* __restrict__ residual,
                                                               float* __restrict__ y, DirDesc d) {
  constexpr int SEG = 3 * SW + KW;  // input columns under 4 outputs
  const int gi = (int)blockIdx.x * 256 + (int)threadIdx.x;
  if (gi >= d.groups4) return;
  const int per_img = d.OH * d.OW4;
  const int img = (int)((uint32_t)gi / (uint32_t)per_img);
  const int r = gi - img * per_img;
  const int oy = (int)((uint32_t)r / (uint32_t)d.OW4);
  const int ox0 = (r - oy * d.OW4) * 4;
  const int64_t HW = (int64_t)d.H * d.W;
  // Input through a buffer resource over the whole tensor (< 2 GiB, see
  // conv_direct_valu_eligible): 32-bit offsets, and padding positions get an
  // out-of-range offset, which the buffer load returns as 0.
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, (int)(d.x_elems * 4), 0x00020000);
  const uint32_t img_off = (uint32_t)img * (uint32_t)d.C * (uint32_t)HW * 4u;
  const int ix0 = ox0 * SW - d.pl;
  const int nchunk = (d.M + MC - 1) / MC;
  const int64_t OP = (int64_t)d.OH * d.OW4 * 4;
  for (int ch = blockIdx.y; ch < nchunk; ch += gridDim.y) {
    const int o0 = ch * MC;
    f32x2 acc[MC][2];
#pragma unroll
    for (int o = 0; o < MC; o++) acc[o][0] = acc[o][1] = (f32x2){0.f, 0.f};
    const float* __restrict__ wk = wt + o0;
    int k = 0;
    const int nc = CC > 0 ? CC : d.C, nkh = KH > 0 ? KH : d.kh;
    constexpr int UC = CC > 0 ? CC : 1, UKH = KH > 0 ? KH : 1;
#pragma unroll UC
    for (int c = 0; c < nc; c++) {
#pragma unroll UKH
      for (int ky = 0; ky < nkh; ky++, k += KW) {
        const int iy = oy * d.sh - d.pt + ky * d.dh;
        const bool row_ok = iy >= 0 && iy < d.H;
        const uint32_t row_off = img_off + (uint32_t)(c * (int)HW + iy * d.W) * 4u;
        float seg[SEG];
#pragma unroll
        for (int t = 0; t < SEG; t++) {
          const int ix = ix0 + t;
          const uint32_t off = row_ok && ix >= 0 && ix < d.W ? row_off + (uint32_t)ix * 4u : 0x80000000u;
          seg[t] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xrs, off, 0, 0));
        }
#pragma unroll
        for (int kx = 0; kx < KW; kx++) {
          const f32x2 xa = {seg[kx], seg[SW + kx]}, xb = {seg[2 * SW + kx], seg[3 * SW + kx]};
          const float* __restrict__ wr = wk + (k + kx) * d.Mpad;
#pragma unroll
          for (int o = 0; o < (RTENHIP_PW_EXPERIMENT == 2 ? 1 : MC); o++) {
            const f32x2 wv = {wr[o], wr[o]};
            acc[o][0] = __builtin_elementwise_fma(wv, xa, acc[o][0]);
            acc[o][1] = __builtin_elementwise_fma(wv, xb, acc[o][1]);
          }
        }
      }
    }
    if constexpr (RTENHIP_PW_EXPERIMENT == 2) {
#pragma unroll
      for (int o = 1; o < MC; o++) acc[o][0] = acc[0][0] + (float)o, acc[o][1] = acc[0][1];
    }
    const int64_t pix = (int64_t)oy * d.OW4 * 4 + ox0;
    float* __restrict__ yp = y + ((int64_t)img * d.M + o0) * OP + pix;
    const float* __restrict__ rp = residual ? residual + ((int64_t)img * d.M + o0) * OP + pix : nullptr;
    const int olim = d.M - 1 - o0;
#pragma unroll
    for (int o = 0; o < MC; o++) {
      if (o > olim) continue;
      float4 v = make_float4(acc[o][0].x, acc[o][0].y, acc[o][1].x, acc[o][1].y);
      if (bias) {
        const float b = bias[o0 + o];
        v.x = __fadd_rn(v.x, b);
        v.y = __fadd_rn(v.y, b);
        v.z = __fadd_rn(v.z, b);
        v.w = __fadd_rn(v.w, b);
      }
      if (rp) {
        const float4 q = *(const float4*)(rp + (int64_t)o * OP);
        v.x = __fadd_rn(v.x, q.x);
        v.y = __fadd_rn(v.y, q.y);
        v.z = __fadd_rn(v.z, q.z);
        v.w = __fadd_rn(v.w, q.w);
      }
      v.x = pw_act(v.x, d.act, d.lo, d.hi);
      v.y = pw_act(v.y, d.act, d.lo, d.hi);
      v.z = pw_act(v.z, d.act, d.lo, d.hi);
      v.w = pw_act(v.w, d.act, d.lo, d.hi);
      if (RTENHIP_PW_EXPERIMENT != 1 || v.x == 1234.5f) *(float4*)(yp + (int64_t)o * OP) = v;
    }
  }
}

// The same direct conv with the block's input rows staged in LDS (variant mc
// + 100; MobileNetV2's stem: 3 channels, 3x3, stride 2, pad 1).  A block owns
// TR output rows x the whole output width of one image for all channel
// chunks; its C x R input rows (R = (TR - 1) * SW + kh) are copied into LDS
// once, zero-filled where the window leaves the image, by coalesced 4-byte
// loads all in flight together (no per-channel round trips, no padded copy of
// the input).  LDS row layout: position j holds input column j - 4, so a
// lane's 4 outputs read their window as three aligned 16-byte LDS reads.
// Same chain order k = (c, ky, kx) and the same fma(w, 0, acc) at padding
// positions as conv_direct_valu_kernel, so the two are bit-identical.
constexpr int kDirLdsQ = 52;  // staged floats per thread: 52 KB of LDS, three blocks per CU
struct DirLdsDesc {
  int TR, R, LROW, tiles_y;
  FastDiv fdLROW, fdR;
};

template <int MC, int SW, int PL>
__global__ __launch_bounds__(256) void conv_direct_lds_kernel(const float* __restrict__ x,
                                                              const float* __restrict__ wt,
                                                              const float* __restrict__ bias,
                                                              const float* __restrict__ residual,
                                                              float* __restrict__ y, DirDesc d, DirLdsDesc e) {
  extern __shared__ float4 dir_lds4[];
  float* lds = reinterpret_cast<float*>(dir_lds4);
  const int tid = threadIdx.x;
  const int img = (int)blockIdx.x / e.tiles_y;
  const int oy0 = ((int)blockIdx.x - img * e.tiles_y) * e.TR;
  const int64_t HW = (int64_t)d.H * d.W;
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, (int)(d.x_elems * 4), 0x00020000);
  const uint32_t img_off = (uint32_t)img * (uint32_t)d.C * (uint32_t)HW * 4u;
  const int iy0 = oy0 * SW - d.pt;
  const int total = d.C * e.R * e.LROW;
  // Stage: element i = (c * R + r) * LROW + j <- x[img][c][iy0 + r][j - 4].
  float v[kDirLdsQ];
#pragma unroll
  for (int q = 0; q < kDirLdsQ; q++) {
    const int i = tid + 256 * q;
    const int cr = fdiv(i, e.fdLROW);
    const int j = i - cr * e.LROW;
    const int c = fdiv(cr, e.fdR);
    const int iy = iy0 + cr - c * e.R, ix = j - 4;
    const bool ok = i < total && iy >= 0 && iy < d.H && ix >= 0 && ix < d.W;
    const uint32_t off = ok ? img_off + (uint32_t)(c * (int)HW + iy * d.W + ix) * 4u : 0x80000000u;
    v[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xrs, off, 0, 0));
  }
#pragma unroll
  for (int q = 0; q < kDirLdsQ; q++)
    if (tid + 256 * q < total) lds[tid + 256 * q] = v[q];
  __syncthreads();

  const int tr = tid / d.OW4, t = tid - tr * d.OW4;
  const int oy = oy0 + tr;
  if (tr >= e.TR || oy >= d.OH) return;
  // Window of output column 4t + i, tap kx: LDS position SW * (4t + i) + kx
  // + 4 - PL = base + o + SW * i + kx.
  constexpr int o = (4 - PL) & 3;
  const int base = SW * 4 * t + 4 - PL - o;
  const int nchunk = (d.M + MC - 1) / MC;
  const int64_t OP = (int64_t)d.OH * d.OW4 * 4;
  for (int ch = 0; ch < nchunk; ch++) {
    const int o0 = ch * MC;
    f32x2 acc[MC][2];
#pragma unroll
    for (int m = 0; m < MC; m++) acc[m][0] = acc[m][1] = (f32x2){0.f, 0.f};
    // (Weights as scalar operands: staged in LDS and read as broadcast
    // 16-byte loads instead, the stem conv measured 0.104 -> 0.153 ms.)
    const float* __restrict__ wk = wt + o0;
    int k = 0;
    for (int c = 0; c < d.C; c++) {
      // (ky not unrolled: 160 VGPRs, three waves per SIMD)
      for (int ky = 0; ky < d.kh; ky++, k += 3) {
        // (LROW and base are multiples of 4: 16-byte reads)
        const float4* rp = dir_lds4 + (((c * e.R + tr * SW + ky) * e.LROW + base) >> 2);
        const float4 s0 = rp[0], s1 = rp[1], s2 = rp[2];
        const float seg[12] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w, s2.x, s2.y, s2.z, s2.w};
#pragma unroll
        for (int kx = 0; kx < 3; kx++) {
          const f32x2 xa = {seg[o + kx], seg[o + SW + kx]}, xb = {seg[o + 2 * SW + kx], seg[o + 3 * SW + kx]};
          const float* __restrict__ wr = wk + (k + kx) * d.Mpad;
#pragma unroll
          for (int m = 0; m < MC; m++) {
            const f32x2 wv = {wr[m], wr[m]};
            acc[m][0] = __builtin_elementwise_fma(wv, xa, acc[m][0]);
            acc[m][1] = __builtin_elementwise_fma(wv, xb, acc[m][1]);
          }
        }
      }
    }
    const int64_t pix = (int64_t)oy * d.OW4 * 4 + 4 * t;
    float* __restrict__ yp = y + ((int64_t)img * d.M + o0) * OP + pix;
    const float* __restrict__ rq = residual ? residual + ((int64_t)img * d.M + o0) * OP + pix : nullptr;
    const int olim = d.M - 1 - o0;
#pragma unroll
    for (int m = 0; m < MC; m++) {
      if (m > olim) continue;
      float4 r = make_float4(acc[m][0].x, acc[m][0].y, acc[m][1].x, acc[m][1].y);
      if (bias) {
        const float b = bias[o0 + m];
        r.x = __fadd_rn(r.x, b);
        r.y = __fadd_rn(r.y, b);
        r.z = __fadd_rn(r.z, b);
        r.w = __fadd_rn(r.w, b);
      }
      if (rq) {
        const float4 q = *(const float4*)(rq + (int64_t)m * OP);
        r.x = __fadd_rn(r.x, q.x);
        r.y = __fadd_rn(r.y, q.y);
        r.z = __fadd_rn(r.z, q.z);
        r.w = __fadd_rn(r.w, q.w);
      }
      r.x = pw_act(r.x, d.act, d.lo, d.hi);
      r.y = pw_act(r.y, d.act, d.lo, d.hi);
      r.z = pw_act(r.z, d.act, d.lo, d.hi);
      r.w = pw_act(r.w, d.act, d.lo, d.hi);
      if (RTENHIP_PW_EXPERIMENT != 1 || r.x == 1234.5f) *(float4*)(yp + (int64_t)m * OP) = r;
    }
  }
}

// Rows per block of the LDS-staged direct conv (0: not eligible).
static DirLdsDesc dir_lds_plan(int64_t C, int64_t kh, int64_t sh, int64_t oh, int64_t ow, int64_t M) {
  DirLdsDesc e{};
  const int64_t ow4 = ow / 4;
  (void)M;
  if (ow4 < 1 || ow4 > 256) return e;
  const int64_t lrow = sh * 4 * ow4 + 12;
  int64_t tr = std::min<int64_t>(oh, 256 / ow4);
  auto rows = [&](int64_t t) { return C * ((t - 1) * sh + kh) * lrow; };
  while (tr >= 1 && rows(tr) > 256 * kDirLdsQ) tr--;
  if (tr < 1) return e;
  e.TR = (int)tr;
  e.R = (int)((tr - 1) * sh + kh);
  e.LROW = (int)lrow;
  e.tiles_y = (int)((oh + tr - 1) / tr);
  e.fdLROW = make_fastdiv((uint32_t)lrow);
  e.fdR = make_fastdiv((uint32_t)e.R);
  return e;
}

bool conv_direct_lds_eligible(const ConvPlan& g, bool padded_out) {
  return conv_direct_valu_eligible(g, padded_out) && g.kh <= 3 && g.dh == 1 && g.sh == g.sw &&
         (g.pads[1] == 0 || g.pads[1] == 1) && dir_lds_plan(g.C, g.kh, g.sh, g.oh, g.ow, g.O).TR > 0;
}

// w [M][K] -> wt [K][Mpad], zero columns M..Mpad-1
__global__ void transpose_weights_kernel(const float* __restrict__ w, float* __restrict__ wt, int M,
                                         int Mpad, int K) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)Mpad * K) return;
  const int k = (int)(i / Mpad), m = (int)(i - (int64_t)k * Mpad);
  wt[i] = m < M ? w[(int64_t)m * K + k] : 0.f;
}

bool conv_pw_valu_eligible(const ConvPlan& g, int64_t Hp, int64_t Wp, bool padded_out) {
  const int64_t P = g.oh * g.ow;
  return g.kh == 1 && g.kw == 1 && g.sh == 1 && g.sw == 1 && g.groups == 1 && g.dh == 1 &&
         g.dw == 1 && !g.pads[0] && !g.pads[1] && !g.pads[2] && !g.pads[3] && Hp == g.oh &&
         Wp == g.ow && !padded_out && P % 4 == 0 && g.C >= 1 && g.C <= 256 && g.O >= 1 &&
         g.N * P < (int64_t(1) << 31);
}

bool conv_direct_valu_eligible(const ConvPlan& g, bool padded_out) {
  return g.groups == 1 && g.kw == 3 && g.dw == 1 && (g.sw == 1 || g.sw == 2) && g.kh >= 1 &&
         g.C * g.kh * g.kw <= 64 && g.ow % 4 == 0 && !padded_out &&
         g.N * g.oh * g.ow < (int64_t(1) << 31) && g.N * g.C * g.H * g.W < (int64_t(1) << 29);
}

int64_t pw_weight_floats(int64_t M, int64_t K) { return (M + 31) / 32 * 32 * K; }

rtenhip_status pack_pw_weights(const float* w, int64_t M, int64_t K, float* wt, hipStream_t s) {
  const int64_t n = pw_weight_floats(M, K);
  transpose_weights_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(w, wt, (int)M,
                                                                      (int)((M + 31) / 32 * 32), (int)K);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

// variant = mc + 100 * (KX / 16): mc in {8, 16, 32}; KX 0 (streamed x), 16 or 32
bool pw_variant_ok(int variant, int64_t K) {
  const int mc = variant % 100, kx = variant / 100 * 16;
  return (mc == 8 || mc == 16 || mc == 32) && (kx == 0 || ((kx == 16 || kx == 32) && K <= kx && mc <= 16));
}

rtenhip_status conv_direct_valu(const ConvDmaArgs& a, int mc, hipStream_t s) {
  const bool lds = mc >= 100;
  if (lds) mc -= 100;
  if (a.groups != 1 || a.kw != 3 || a.dw != 1 || (a.sw != 1 && a.sw != 2) || a.ow % 4 ||
      a.C * a.kh * a.kw > 64 || (uintptr_t)a.y % 16 || (a.residual && (uintptr_t)a.residual % 16) ||
      !a.x_unpadded || (mc != 16 && mc != 32))
    return fail(RTENHIP_INVALID_VALUE, "direct VALU conv: unsupported layout");
  DirLdsDesc e{};
  if (lds) {
    e = dir_lds_plan(a.C, a.kh, a.sh, a.oh, a.ow, a.O);
    if (e.TR == 0 || a.kh > 3 || a.dh != 1 || a.sh != a.sw || (a.pad_l != 0 && a.pad_l != 1))
      return fail(RTENHIP_INVALID_VALUE, "direct VALU conv (LDS rows): unsupported layout");
  }
  DirDesc d{};
  d.C = (int)a.C;
  d.x_elems = a.N * a.C * a.H * a.W;
  d.H = (int)a.H;
  d.W = (int)a.W;
  d.kh = (int)a.kh;
  d.sh = (int)a.sh;
  d.dh = (int)a.dh;
  d.pt = (int)a.pad_t;
  d.pl = (int)a.pad_l;
  d.OH = (int)a.oh;
  d.OW4 = (int)(a.ow / 4);
  d.M = (int)a.O;
  d.Mpad = (int)((a.O + 31) / 32 * 32);
  d.groups4 = (int)(a.N * a.oh * a.ow / 4);
  d.act = a.act;
  d.lo = a.lo;
  d.hi = a.hi;
  if (lds) {
    const unsigned blocks = (unsigned)(a.N * e.tiles_y);
    const size_t bytes = (size_t)a.C * e.R * e.LROW * 4;
#define DIR_LDS_LAUNCH(MC, SW, PL)                                                                      \
  conv_direct_lds_kernel<MC, SW, PL><<<blocks, 256, bytes, s>>>(a.x_unpadded, a.packed_w, a.bias, a.residual, \
                                                                a.y, d, e)
#define DIR_LDS_PL(MC, SW) \
  if (a.pad_l == 1) { DIR_LDS_LAUNCH(MC, SW, 1); } else { DIR_LDS_LAUNCH(MC, SW, 0); }
#define DIR_LDS_SW(MC) \
  if (a.sw == 2) { DIR_LDS_PL(MC, 2); } else { DIR_LDS_PL(MC, 1); }
    if (mc == 32) {
      DIR_LDS_SW(32);
    } else {
      DIR_LDS_SW(16);
    }
#undef DIR_LDS_SW
#undef DIR_LDS_PL
#undef DIR_LDS_LAUNCH
    RTENHIP_LAUNCH_CHECK();
    return RTENHIP_OK;
  }
  const int64_t gx = (d.groups4 + 255) / 256;
  const int nchunk = (d.M + mc - 1) / mc;
  int gy = 1;
  while (gy < nchunk && gx * gy < 2048) gy++;
  const dim3 grid((unsigned)gx, (unsigned)gy);
#define DIR_LAUNCH(MC, SW, CC, KH)                                                                   \
  conv_direct_valu_kernel<MC, 3, SW, CC, KH><<<grid, 256, 0, s>>>(a.x_unpadded, a.packed_w, a.bias, \
                                                                  a.residual, a.y, d)
  const bool stem = a.C == 3 && a.kh == 3;
  if (mc == 16 && a.sw == 1) DIR_LAUNCH(16, 1, 0, 0);
  else if (mc == 16 && stem) DIR_LAUNCH(16, 2, 0, 3);
  else if (mc == 16) DIR_LAUNCH(16, 2, 0, 0);
  else if (a.sw == 1) DIR_LAUNCH(32, 1, 0, 0);
  else if (stem) DIR_LAUNCH(32, 2, 0, 3);
  else DIR_LAUNCH(32, 2, 0, 0);
#undef DIR_LAUNCH
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

rtenhip_status conv_pw_valu(const ConvDmaArgs& a, int variant, hipStream_t s) {
  const int64_t P = a.oh * a.ow;
  if (P % 4 || a.C > 256 || ((uintptr_t)a.xin | (uintptr_t)a.y) % 16 ||
      (a.residual && (uintptr_t)a.residual % 16) || !pw_variant_ok(variant, a.C))
    return fail(RTENHIP_INVALID_VALUE, "pointwise VALU conv: unsupported layout");
  PwDesc d{};
  d.M = (int)a.O;
  d.Mpad = (int)((a.O + 31) / 32 * 32);
  d.K = (int)a.C;
  d.P4 = (int)(P / 4);
  d.groups4 = (int)(a.N * P / 4);
  d.act = a.act;
  d.lo = a.lo;
  d.hi = a.hi;
  const int mc = variant % 100, kx = variant / 100 * 16;
  const int64_t gx = (d.groups4 + 255) / 256;
  const int nchunk = (d.M + mc - 1) / mc;
  // Small layers: channel chunks across blocks too, so the grid fills the
  // 256 CUs (streamed x is then re-read per chunk from L2 either way).
  int gy = 1;
  while (gy < nchunk && gx * gy < 2048) gy++;
  const dim3 grid((unsigned)gx, (unsigned)gy);
#define PW_LAUNCH(MC, KX)                                                                       \
  conv_pw_valu_kernel<MC, KX><<<grid, 256, 0, s>>>(a.xin, a.packed_w, a.bias, a.residual, a.y, d)
  switch (variant) {
    case 8: PW_LAUNCH(8, 0); break;
    case 16: PW_LAUNCH(16, 0); break;
    case 32: PW_LAUNCH(32, 0); break;
    case 108: PW_LAUNCH(8, 16); break;
    case 116: PW_LAUNCH(16, 16); break;
    case 208: PW_LAUNCH(8, 32); break;
    case 216: PW_LAUNCH(16, 32); break;
    default: return fail(RTENHIP_INVALID_VALUE, "pointwise VALU conv: unknown variant");
  }
#undef PW_LAUNCH
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

}  // namespace rtenhip
