// Pooling and depthwise convolution kernels (HBM-bound).
//
//  - MaxPool / AveragePool: pool_impl (src/ops/pooling.rs:104-238) folds the
//    window in (ky, kx) order from -inf / 0 and divides by the non-padding
//    count (or the kernel size with count_include_pad).
//  - GlobalAveragePool (pooling.rs:294-342): row-major sum per channel / HW.
//  - Depthwise conv: conv_2d_depthwise_block (src/ops/conv/depthwise.rs:49-120)
//    initialises each output row with the bias and adds in*w (separately
//    rounded) per (ky, kx); the valid output-x range per kx is the
//    reference's min_max_out_x_coords (depthwise.rs:24-38), reproduced
//    exactly.  The Clip/Relu/Add that follow in MobileNetV2 can be fused.
#include "common.h"
#include <cstdlib>
#include "vecmath.h"
#include "fastdiv_dev.h"
#include "stage.h"

namespace rtenhip {

template <bool IS_MAX, typename IDX>
__global__ void pool_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t total_,
                            int H, int W, int OH, int OW, int kh, int kw, int sh, int sw, int pt,
                            int pl, int count_include_pad) {
  const IDX total = (IDX)total_;
  const IDX stride = (IDX)gridDim.x * blockDim.x;
  for (IDX i = (IDX)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int ox = (int)(i % OW);
    const int oy = (int)((i / OW) % OH);
    const IDX plane = i / ((IDX)OW * OH);
    const float* xp = x + (int64_t)plane * H * W;
    float acc = IS_MAX ? -__builtin_huge_valf() : 0.f;
    int cnt = 0;
    for (int ky = 0; ky < kh; ky++) {
      const int iy = oy * sh + ky;
      if (iy < pt || iy >= H + pt) continue;
      for (int kx = 0; kx < kw; kx++) {
        const int ix = ox * sw + kx;
        if (ix < pl || ix >= W + pl) continue;
        const float v = xp[(iy - pt) * W + (ix - pl)];
        acc = IS_MAX ? rust_max(acc, v) : __fadd_rn(acc, v);
        cnt++;
      }
    }
    if (!IS_MAX) acc = __fdiv_rn(acc, count_include_pad ? (float)(kh * kw) : (float)cnt);
    y[i] = acc;
  }
}

// One workgroup per (n, c) plane staged in LDS with 16-byte loads; each
// output then reads its window from LDS.  Same per-window (ky, kx) order and
// arithmetic as pool_kernel: taps in the padding are skipped (for max a
// skipped tap and a -inf tap are the same, for avg the add is predicated so a
// -0.0 sum is kept).  KH/KW > 0: compile-time window, fully unrolled.
template <bool IS_MAX, int KH, int KW>
__global__ __launch_bounds__(256) void pool_plane_kernel(const float* __restrict__ x,
                                                         float* __restrict__ y, int H, int W,
                                                         int OH, int OW, FastDiv fd_ow, int kh_,
                                                         int kw_, int sh, int sw, int pt, int pl,
                                                         int count_include_pad, int rb) {
  extern __shared__ float plane[];
  const int kh = KH > 0 ? KH : kh_, kw = KW > 0 ? KW : kw_;
  const int64_t pidx = blockIdx.x;
  // Output rows [oy0, oy1) of this block and the input rows [r_lo, r_hi) they read.
  const int oy0 = blockIdx.y * rb, oy1 = min(OH, oy0 + rb);
  const int r_lo = max(0, oy0 * sh - pt), r_hi = min(H, (oy1 - 1) * sh - pt + kh);
  const float* xp = x + pidx * H * W + (int64_t)r_lo * W;
  const int n = max(0, r_hi - r_lo) * W;
  if ((W & 3) == 0) {
    stage_batched<4, float4>(n >> 2, [&](int e) { return *(const float4*)(xp + 4 * e); },
                             [&](int e, const float4& v) { *(float4*)(plane + 4 * e) = v; });
  } else {
    stage_batched<8, float>(n, [&](int e) { return xp[e]; }, [&](int e, float v) { plane[e] = v; });
  }
  __syncthreads();
  float* yp = y + pidx * OH * OW;
  for (int o = oy0 * OW + threadIdx.x; o < oy1 * OW; o += 256) {
    const int oy = fdiv(o, fd_ow), ox = o - oy * OW;
    const int iy0 = oy * sh - pt, ix0 = ox * sw - pl;
    float acc = IS_MAX ? -__builtin_huge_valf() : 0.f;
    int cnt = 0;
#pragma unroll
    for (int ky = 0; ky < (KH > 0 ? KH : 1); ky++) {
      for (int kyr = (KH > 0 ? ky : 0); kyr < (KH > 0 ? ky + 1 : kh); kyr++) {
        const int iy = iy0 + kyr;
        const bool row_ok = iy >= 0 && iy < H;
#pragma unroll
        for (int kx = 0; kx < (KW > 0 ? KW : 1); kx++) {
          for (int kxr = (KW > 0 ? kx : 0); kxr < (KW > 0 ? kx + 1 : kw); kxr++) {
            const int ix = ix0 + kxr;
            const bool ok = row_ok && ix >= 0 && ix < W;
            const float v = plane[ok ? (iy - r_lo) * W + ix : 0];
            if (IS_MAX) {
              acc = ok ? rust_max(acc, v) : acc;
            } else {
              acc = ok ? __fadd_rn(acc, v) : acc;
              cnt += ok;
            }
          }
        }
      }
    }
    if (!IS_MAX) acc = __fdiv_rn(acc, count_include_pad ? (float)(kh * kw) : (float)cnt);
    yp[o] = acc;
  }
}

template <bool IS_MAX>
static void launch_pool_plane(const float* x, float* y, int64_t NC, int H, int W, int OH, int OW,
                              int kh, int kw, int sh, int sw, int pt, int pl, int cip,
                              hipStream_t s) {
  // Row bands of rb output rows whose input rows fit ~16 KB of LDS (more
  // resident blocks per CU, so staging overlaps other blocks' compute).
  const int rows_in = std::max(kh, 4096 / W);
  const int rb = std::max(1, std::min(OH, (rows_in - kh) / sh + 1));
  const int bands = (OH + rb - 1) / rb;
  const int max_rows = std::min(H, (rb - 1) * sh + kh);
  const size_t bytes = (size_t)max_rows * W * sizeof(float);
  const FastDiv fd = make_fastdiv((uint32_t)OW);
  const dim3 grid((unsigned)NC, (unsigned)bands);
  if (kh == 3 && kw == 3)
    hipLaunchKernelGGL((pool_plane_kernel<IS_MAX, 3, 3>), grid, dim3(256), bytes, s, x, y, H, W,
                       OH, OW, fd, kh, kw, sh, sw, pt, pl, cip, rb);
  else if (kh == 2 && kw == 2)
    hipLaunchKernelGGL((pool_plane_kernel<IS_MAX, 2, 2>), grid, dim3(256), bytes, s, x, y, H, W,
                       OH, OW, fd, kh, kw, sh, sw, pt, pl, cip, rb);
  else
    hipLaunchKernelGGL((pool_plane_kernel<IS_MAX, 0, 0>), grid, dim3(256), bytes, s, x, y, H, W,
                       OH, OW, fd, kh, kw, sh, sw, pt, pl, cip, rb);
}

rtenhip_status launch_pool(int is_max, const float* x, float* y, int64_t NC, int H, int W,
                           int OH, int OW, int kh, int kw, int sh, int sw, int pt, int pl,
                           int count_include_pad, hipStream_t s) {
  const int64_t total = NC * OH * OW;
  if (total == 0) return RTENHIP_OK;
  const size_t plane_bytes = (size_t)H * W * sizeof(float);
  if (plane_bytes <= 64 * 1024 && OH * OW >= 256 && NC < (int64_t(1) << 31) && sh >= 1 &&
      kh >= 1 && ((uintptr_t)x % 16) == 0) {
    if (is_max)
      launch_pool_plane<true>(x, y, NC, H, W, OH, OW, kh, kw, sh, sw, pt, pl, count_include_pad, s);
    else
      launch_pool_plane<false>(x, y, NC, H, W, OH, OW, kh, kw, sh, sw, pt, pl, count_include_pad, s);
    RTENHIP_LAUNCH_CHECK();
    return RTENHIP_OK;
  }
  int64_t blocks32 = (total + 255) / 256;
  if (blocks32 > 8192) blocks32 = 8192;
  if (total + blocks32 * 256 < (int64_t(1) << 31) && NC * H * W < (int64_t(1) << 31)) {
    // 32-bit index math (the 64-bit divisions dominate the 64-bit variant).
    if (is_max)
      hipLaunchKernelGGL((pool_kernel<true, int>), dim3((unsigned)blocks32), dim3(256), 0, s, x, y,
                         total, H, W, OH, OW, kh, kw, sh, sw, pt, pl, count_include_pad);
    else
      hipLaunchKernelGGL((pool_kernel<false, int>), dim3((unsigned)blocks32), dim3(256), 0, s, x, y,
                         total, H, W, OH, OW, kh, kw, sh, sw, pt, pl, count_include_pad);
    RTENHIP_LAUNCH_CHECK();
    return RTENHIP_OK;
  }
  int64_t blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (is_max)
    hipLaunchKernelGGL((pool_kernel<true, int64_t>), dim3((unsigned)blocks), dim3(256), 0, s, x, y, total, H,
                       W, OH, OW, kh, kw, sh, sw, pt, pl, count_include_pad);
  else
    hipLaunchKernelGGL((pool_kernel<false, int64_t>), dim3((unsigned)blocks), dim3(256), 0, s, x, y, total, H,
                       W, OH, OW, kh, kw, sh, sw, pt, pl, count_include_pad);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

// One thread per (n, c): the reference's sum is a sequential chain over the
// plane, so it is kept sequential; planes are small (7x7 in ResNet/MobileNet)
// and the wave's 64 planes are contiguous, so the loads stay L1/L2-served.
__global__ void gap_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t NC,
                           int64_t HW) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= NC) return;
  const float* p = x + i * HW;
  float s = 0.f;
  for (int64_t k = 0; k < HW; k++) s = __fadd_rn(s, p[k]);
  y[i] = __fdiv_rn(s, (float)HW);
}

// Same sequential chain per plane, with the block's planes (contiguous in
// memory) first staged through LDS by coalesced loads.
__global__ __launch_bounds__(256) void gap_lds_kernel(const float* __restrict__ x,
                                                      float* __restrict__ y, int64_t NC, int HW,
                                                      int ppb) {
  extern __shared__ float buf[];
  const int64_t p0 = (int64_t)blockIdx.x * ppb;
  const int np = (int)min((int64_t)ppb, NC - p0);
  const float* src = x + p0 * HW;
  const int n = np * HW;
  stage_batched<8, float>(n, [&](int e) { return src[e]; }, [&](int e, float v) { buf[e] = v; });
  __syncthreads();
  if ((int)threadIdx.x < np) {
    const float* p = buf + threadIdx.x * HW;
    float acc = 0.f;
    for (int k = 0; k < HW; k++) acc = __fadd_rn(acc, p[k]);
    y[p0 + threadIdx.x] = __fdiv_rn(acc, (float)HW);
  }
}

rtenhip_status launch_gap(const float* x, float* y, int64_t NC, int64_t HW, hipStream_t s) {
  if (NC == 0) return RTENHIP_OK;
  // Planes per block: at most 256 and 12288 floats of LDS; fewer when that
  // would leave most CUs idle (ResNet-50's 2048 planes of 7 x 7 at batch 1:
  // 64 blocks of 32 planes, one memory round trip each, instead of 9 blocks
  // staging 12250 floats in six).
  int64_t ppb = std::min<int64_t>(256, HW > 0 ? 12288 / HW : 0);
  if (ppb >= 32 && NC < 256 * ppb) ppb = std::max<int64_t>(32, std::min(ppb, (NC + 255) / 256));
  if (HW > 0 && ppb >= 32 && NC / ppb < (int64_t(1) << 31)) {
    const int64_t blocks = (NC + ppb - 1) / ppb;
    hipLaunchKernelGGL(gap_lds_kernel, dim3((unsigned)blocks), dim3(256),
                       (size_t)(ppb * HW * sizeof(float)), s, x, y, NC, (int)HW, (int)ppb);
    RTENHIP_LAUNCH_CHECK();
    return RTENHIP_OK;
  }
  hipLaunchKernelGGL(gap_kernel, dim3((unsigned)((NC + 255) / 256)), dim3(256), 0, s, x, y, NC,
                     HW);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

__global__ void depthwise_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                 const float* __restrict__ bias, float* __restrict__ y,
                                 int64_t total, int C, int H, int W, int OH, int OW, int kh,
                                 int kw, int sh, int sw, int dh, int dw, int pt, int pl,
                                 const float* __restrict__ residual, int act, float lo,
                                 float hi) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int ox = (int)(i % OW);
    const int oy = (int)((i / OW) % OH);
    const int64_t plane = i / ((int64_t)OW * OH);  // n*C + c
    const int c = (int)(plane % C);
    const float* xp = x + plane * H * W;
    const float* kp = w + (int64_t)c * kh * kw;
    float acc = bias ? bias[c] : 0.f;
    for (int ky = 0; ky < kh; ky++) {
      const int iy = oy * sh + ky * dh;
      if (iy < pt || iy >= H + pt) continue;
      const float* row = xp + (int64_t)(iy - pt) * W;
      for (int kx = 0; kx < kw; kx++) {
        // min_max_out_x_coords (depthwise.rs:24-38)
        const int kxd = kx * dw;
        const int omin = pl - kxd > 0 ? pl - kxd : 0;
        const int t = W + pl - kxd > 0 ? W + pl - kxd : 0;
        int omax = (t + sw - 1) / sw;
        if (omax > OW) omax = OW;
        if (ox < omin || ox >= omax) continue;
        const float v = row[ox * sw + kxd - pl];
        acc = __fadd_rn(acc, __fmul_rn(v, kp[ky * kw + kx]));
      }
    }
    if (residual) acc = __fadd_rn(acc, residual[i]);
    if (act == RTENHIP_ACT_RELU) acc = rust_max(acc, 0.f);
    else if (act == RTENHIP_ACT_CLIP) acc = rust_clamp(acc, lo, hi);
    y[i] = acc;
  }
}

// Same arithmetic as depthwise_kernel (per output: bias, then + v*w in ky, kx
// order, separately rounded mul and add as conv_2d_depthwise_block does), for
// outputs that fit 32-bit indexing and kernels at most 8 wide: index math by
// invariant-divisor multiplies and the per-kx valid output-x range
// (min_max_out_x_coords, depthwise.rs:24-38, incl. its undivided lower
// bound) precomputed on the host.
struct DwBounds {
  int omin[8], omax[8];
};

__global__ __launch_bounds__(256) void depthwise32_kernel(
    const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
    float* __restrict__ y, int total, int C, int H, int W, int OH, int OW, int kh, int kw, int sh,
    int sw, int dh, int dw, int pt, int pl, FastDiv fOW, FastDiv fOH, FastDiv fC, DwBounds b,
    const float* __restrict__ residual, int act, float lo, float hi) {
  const int stride = gridDim.x * blockDim.x;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int t = fdiv(i, fOW);
    const int ox = i - t * OW;
    const int plane = fdiv(t, fOH);
    const int oy = t - plane * OH;
    const int c = plane - fdiv(plane, fC) * C;
    const float* xp = x + (int64_t)plane * H * W;
    const float* kp = w + c * kh * kw;
    float acc = bias ? bias[c] : 0.f;
    for (int ky = 0; ky < kh; ky++) {
      const int iy = oy * sh + ky * dh;
      if (iy < pt || iy >= H + pt) continue;
      const float* row = xp + (iy - pt) * W + ox * sw - pl;
#pragma unroll 8
      for (int kx = 0; kx < kw; kx++) {
        if (ox < b.omin[kx] || ox >= b.omax[kx]) continue;
        acc = __fadd_rn(acc, __fmul_rn(row[kx * dw], kp[ky * kw + kx]));
      }
    }
    if (residual) acc = __fadd_rn(acc, residual[i]);
    if (act == RTENHIP_ACT_RELU) acc = rust_max(acc, 0.f);
    else if (act == RTENHIP_ACT_CLIP) acc = rust_clamp(acc, lo, hi);
    y[i] = acc;
  }
}

// LDS-tiled depthwise conv.  A block owns PB consecutive planes (n*C + c) and
// TH output rows of each; thread t is column ox = t % OW of plane t / OW and
// walks the TH rows, so index math happens once per thread.  The input rows
// those outputs need are staged in LDS first (each plane's rows are one
// contiguous span: coalesced, no per-element division); weights and bias live
// in registers.  Tap order, skipping rules and rounding are those of
// depthwise32_kernel (conv_2d_depthwise_block, depthwise.rs).
template <int KH, int KW>  // 0 = runtime kernel size (weights read from memory)
__global__ __launch_bounds__(256) void depthwise_lds_kernel(
    const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
    float* __restrict__ y, int planes, int C, int H, int W, int OH, int OW, int kh_, int kw_,
    int sh, int sw, int dh, int dw, int pt, int pl, int TH, int PB, int rows_in, DwBounds b,
    const float* __restrict__ residual, int act, float lo, float hi, int flat) {
  extern __shared__ float tile[];
  const int plane0 = blockIdx.y * PB;
  const int oy0 = blockIdx.x * TH;
  const int iy_lo = oy0 * sh - pt;  // first input row the block's outputs read
  const int np = min(PB, planes - plane0);
  const int r0 = max(iy_lo, 0), r1 = min(iy_lo + rows_in, H);
  // Tile layout: plane pp's input row iy at tile + pp * pst + (iy - ibase) * W.
  // flat (whole planes per block, PB * H * W % 4 == 0, 16-byte aligned x):
  // the block's planes are one contiguous range of x, copied as is with
  // 16-byte loads -- the small planes of MobileNetV2's last stages (rows of
  // 14 or 7 floats) need no per-row split.
  const int pst = flat ? H * W : rows_in * W;
  const int ibase = flat ? 0 : iy_lo;
  if (flat) {
    const int n = np * H * W, n4 = n >> 2;
    const float4* src = reinterpret_cast<const float4*>(x + (int64_t)plane0 * H * W);
    stage_batched<4, float4>(n4, [&](int e) { return src[e]; },
                             [&](int e, const float4& v) { reinterpret_cast<float4*>(tile)[e] = v; });
    for (int t = 4 * n4 + (int)threadIdx.x; t < n; t += blockDim.x) tile[t] = x[(int64_t)plane0 * H * W + t];
  } else if (r1 > r0) {
    const int span = (r1 - r0) * W;
    if ((W & 3) == 0 && ((uintptr_t)x & 15) == 0) {
      // 16-byte copies, several in flight per thread (loads are batched
      // ahead of the LDS stores: the two address spaces cannot alias).
      const int n4 = span >> 2, total4 = np * n4;
      stage_batched<4, float4>(
          total4,
          [&](int t) {
            const int pp = t / n4, q4 = t - pp * n4;
            return *(const float4*)(x + (int64_t)(plane0 + pp) * H * W + (int64_t)r0 * W + 4 * q4);
          },
          [&](int t, const float4& v) {
            const int pp = t / n4, q4 = t - pp * n4;
            *(float4*)(tile + (pp * rows_in + (r0 - iy_lo)) * W + 4 * q4) = v;
          });
    } else {
      // Rows of 14 or 7 floats (MobileNetV2's last stages): one flat loop over
      // every plane's span, so a block of 36 small planes issues its loads
      // together instead of one plane (49 active lanes) per round trip.
      const int total = np * span;
      stage_batched<8, float>(
          total,
          [&](int t) {
            const int pp = t / span, q = t - pp * span;
            return x[(int64_t)(plane0 + pp) * H * W + (int64_t)r0 * W + q];
          },
          [&](int t, float v) {
            const int pp = t / span, q = t - pp * span;
            tile[(pp * rows_in + (r0 - iy_lo)) * W + q] = v;
          });
    }
  }
  __syncthreads();
  const int pp = threadIdx.x / OW;
  const int ox = threadIdx.x - pp * OW;
  if (pp >= np) return;
  const int plane = plane0 + pp;
  const int c = plane % C;
  const int kh = KH ? KH : kh_, kw = KW ? KW : kw_;
  constexpr int NT = KH * KW > 0 ? KH * KW : 1;
  float wr[NT];  // compile-time kernel: weights in registers
  if constexpr (KH * KW > 0) {
#pragma unroll
    for (int t = 0; t < NT; t++) wr[t] = w[c * NT + t];
  }
  const float* kp = w + c * kh * kw;
  const float b0 = bias ? bias[c] : 0.f;
  const int oh_blk = min(TH, OH - oy0);
  auto epilogue = [&](int oy, float acc) __attribute__((always_inline)) {
    const int64_t oi = (int64_t)plane * OH * OW + oy * OW + ox;
    if (residual) acc = __fadd_rn(acc, residual[oi]);
    if (act == RTENHIP_ACT_RELU) acc = rust_max(acc, 0.f);
    else if (act == RTENHIP_ACT_CLIP) acc = rust_clamp(acc, lo, hi);
    y[oi] = acc;
  };
  if constexpr (KH == 3 && KW == 3) {
    if (dh == 1 && dw == 1) {
      // 3x3 window in registers: consecutive output rows share 3 - sh input
      // rows, so each row loads only sh new rows of three taps from LDS;
      // column validity is fixed per thread.  Taps, skips and rounding order
      // as in the generic loop below.
      bool colok[3];
#pragma unroll
      for (int kx = 0; kx < 3; kx++) colok[kx] = ox >= b.omin[kx] && ox < b.omax[kx];
      const int cbase = ox * sw - pl;
      float win[3][3];
      auto load_row = [&](int slot, int iy) __attribute__((always_inline)) {
        const bool ok = iy >= 0 && iy < H;
        const float* row = tile + pp * pst + (ok ? iy - ibase : 0) * W + cbase;
#pragma unroll
        for (int kx = 0; kx < 3; kx++) win[slot][kx] = (ok && colok[kx]) ? row[kx] : 0.f;
      };
      int top = oy0 * sh - pt;  // input row of window row 0
      load_row(0, top);
      load_row(1, top + 1);
      load_row(2, top + 2);
      for (int oyl = 0; oyl < oh_blk; oyl++) {
        const int oy = oy0 + oyl;
        if (oyl > 0) {
          top = oy * sh - pt;
          if (sh == 1) {
#pragma unroll
            for (int kx = 0; kx < 3; kx++) {
              win[0][kx] = win[1][kx];
              win[1][kx] = win[2][kx];
            }
            load_row(2, top + 2);
          } else if (sh == 2) {
#pragma unroll
            for (int kx = 0; kx < 3; kx++) win[0][kx] = win[2][kx];
            load_row(1, top + 1);
            load_row(2, top + 2);
          } else {
            load_row(0, top);
            load_row(1, top + 1);
            load_row(2, top + 2);
          }
        }
        float acc = b0;
#pragma unroll
        for (int ky = 0; ky < 3; ky++) {
          const int iy = top + ky;
          if (iy < 0 || iy >= H) continue;
#pragma unroll
          for (int kx = 0; kx < 3; kx++)
            if (colok[kx]) acc = __fadd_rn(acc, __fmul_rn(win[ky][kx], wr[ky * 3 + kx]));
        }
        epilogue(oy, acc);
      }
      return;
    }
  }
  for (int oyl = 0; oyl < oh_blk; oyl++) {
    const int oy = oy0 + oyl;
    float acc = b0;
#pragma unroll
    for (int ky = 0; ky < (KH ? KH : kh); ky++) {
      const int iy = oy * sh + ky * dh;
      if (iy < pt || iy >= H + pt) continue;
      const float* row = tile + pp * pst + (iy - pt - ibase) * W + ox * sw - pl;
#pragma unroll
      for (int kx = 0; kx < (KW ? KW : kw); kx++) {
        if (ox < b.omin[kx] || ox >= b.omax[kx]) continue;
        const float wv = KH * KW > 0 ? wr[(ky * kw + kx) % NT] : kp[ky * kw + kx];
        acc = __fadd_rn(acc, __fmul_rn(row[kx * dw], wv));
      }
    }
    epilogue(oy, acc);
  }
}

// 3x3 depthwise, stride S in both axes, no dilation, OW % 4 == 0: a thread
// owns 4 adjacent output columns and TR consecutive output rows of one plane
// (16-byte output stores and residual loads, each staged input value read
// from LDS once per row instead of once per tap).  A block covers PB planes x
// RS row slices x OW/4 column groups; the input rows of its TH = RS * TR
// output rows are staged in LDS as in depthwise_lds_kernel, with a DW4_MARGIN
// float margin so edge reads stay inside the allocation (their values are
// never used: colok masks them).  Per output: bias, then + v * w over the taps
// in ky, kx order, skipped exactly as in depthwise32_kernel.
constexpr int DW4_MARGIN = 8;
constexpr int DW4_TR = 4;

template <int S>
__global__ __launch_bounds__(256) void depthwise_lds4_kernel(
    const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
    float* __restrict__ y, int planes, int C, int H, int W, int OH, int OW, int pt, int pl,
    int RS, int PB, int rows_in, DwBounds b, const float* __restrict__ residual, int act, float lo,
    float hi) {
  extern __shared__ float4 dw4_lds[];
  float* tile = reinterpret_cast<float*>(dw4_lds) + DW4_MARGIN;
  constexpr int NC = 3 * S + 3;  // input columns a thread's 4 outputs need (S=1: 6, S=2: 9)
  const int CG = OW >> 2;
  const int TH = RS * DW4_TR;
  const int plane0 = blockIdx.y * PB;
  const int oy0 = blockIdx.x * TH;
  const int iy_lo = oy0 * S - pt;  // input row held in tile row 0
  const int np = min(PB, planes - plane0);
  const int r0 = max(iy_lo, 0), r1 = min(iy_lo + rows_in, H);
  if (r1 > r0) {
    // W % 4 == 0 here (OW % 4 == 0 and W >= (OW - 1) * S + 1 ... checked on the host)
    const int n4 = ((r1 - r0) * W) >> 2, total4 = np * n4;
    stage_batched<4, float4>(
        total4,
        [&](int t) {
          const int pp = t / n4, q4 = t - pp * n4;
          return *(const float4*)(x + (int64_t)(plane0 + pp) * H * W + (int64_t)r0 * W + 4 * q4);
        },
        [&](int t, const float4& v) {
          const int pp = t / n4, q4 = t - pp * n4;
          *(float4*)(tile + (pp * rows_in + (r0 - iy_lo)) * W + 4 * q4) = v;
        });
  }
  __syncthreads();
  const int per_plane = RS * CG;
  const int pp = threadIdx.x / per_plane;
  const int rem = threadIdx.x - pp * per_plane;
  const int rs = rem / CG;
  const int ox0 = (rem - rs * CG) * 4;
  if (pp >= np) return;
  const int plane = plane0 + pp;
  const int c = plane % C;
  float wr[9];
#pragma unroll
  for (int t = 0; t < 9; t++) wr[t] = w[c * 9 + t];
  const float b0 = bias ? bias[c] : 0.f;
  bool colok[4][3];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int kx = 0; kx < 3; kx++) colok[i][kx] = ox0 + i >= b.omin[kx] && ox0 + i < b.omax[kx];
  const int cbase = ox0 * S - pl;
  const int oyb = oy0 + rs * DW4_TR;
  const int nrow = min(DW4_TR, OH - oyb);
  float win[3][NC];
  auto load_row = [&](int slot, int iy) __attribute__((always_inline)) {
    const bool ok = iy >= 0 && iy < H;
    const float* row = tile + (pp * rows_in + (ok ? iy - iy_lo : 0)) * W + cbase;
#pragma unroll
    for (int j = 0; j < NC; j++) win[slot][j] = ok ? row[j] : 0.f;
  };
  int top = oyb * S - pt;
  load_row(0, top);
  load_row(1, top + 1);
  load_row(2, top + 2);
  for (int r = 0; r < nrow; r++) {
    const int oy = oyb + r;
    if (r > 0) {
      top = oy * S - pt;
      if constexpr (S == 1) {
#pragma unroll
        for (int j = 0; j < NC; j++) {
          win[0][j] = win[1][j];
          win[1][j] = win[2][j];
        }
        load_row(2, top + 2);
      } else {
#pragma unroll
        for (int j = 0; j < NC; j++) win[0][j] = win[2][j];
        load_row(1, top + 1);
        load_row(2, top + 2);
      }
    }
    float acc[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      acc[i] = b0;
#pragma unroll
      for (int ky = 0; ky < 3; ky++) {
        const int iy = top + ky;
        if (iy < 0 || iy >= H) continue;
#pragma unroll
        for (int kx = 0; kx < 3; kx++)
          if (colok[i][kx]) acc[i] = __fadd_rn(acc[i], __fmul_rn(win[ky][i * S + kx], wr[ky * 3 + kx]));
      }
    }
    const int64_t oi = (int64_t)plane * OH * OW + (int64_t)oy * OW + ox0;
    if (residual) {
      const float4 rv = *(const float4*)(residual + oi);
      acc[0] = __fadd_rn(acc[0], rv.x);
      acc[1] = __fadd_rn(acc[1], rv.y);
      acc[2] = __fadd_rn(acc[2], rv.z);
      acc[3] = __fadd_rn(acc[3], rv.w);
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
      if (act == RTENHIP_ACT_RELU) acc[i] = rust_max(acc[i], 0.f);
      else if (act == RTENHIP_ACT_CLIP) acc[i] = rust_clamp(acc[i], lo, hi);
    }
    *(float4*)(y + oi) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  }
}

// Launch geometry of depthwise_lds4_kernel, or false when the shape is not
// one it handles.  Row slices per plane: the largest RS (TH = 4 RS output
// rows per block) whose staged rows fit the LDS budget, preferring a TH that
// divides OH; planes per block fill up to 256 threads.
struct Dw4Geom {
  int RS, PB, rows_in;
  size_t lds;
};
static bool dw4_geometry(int H, int W, int OH, int OW, int S, int pt, int pl, int pr, Dw4Geom& g) {
  if (OW % 4 != 0 || W % 4 != 0 || OW > 256 || pl > DW4_MARGIN / 2 || pr > DW4_MARGIN / 2) return false;
  const int CG = OW / 4;
  const int budget = 8192;  // floats of staged input per block (32 KB)
  auto rows_for = [&](int th) { return (th - 1) * S + 3; };
  int best = 0;
  for (int rs = std::max(1, std::min(256 / CG, (OH + DW4_TR - 1) / DW4_TR)); rs >= 1; rs--) {
    if (rows_for(rs * DW4_TR) * W > budget) continue;
    if (!best) best = rs;
    if (OH % (rs * DW4_TR) == 0) {
      if (2 * rs >= best) best = rs;  // an exact split unless it halves the block
      break;
    }
  }
  if (!best) return false;
  g.RS = best;
  g.rows_in = rows_for(best * DW4_TR);
  g.PB = std::max(1, 256 / (best * CG));
  while (g.PB > 1 && g.PB * g.rows_in * W > budget) g.PB--;
  g.lds = ((size_t)g.PB * g.rows_in * W + 2 * DW4_MARGIN) * sizeof(float);
  return true;
}

rtenhip_status launch_depthwise(const float* x, const float* w, const float* bias, float* y,
                                int N, int C, int H, int W, int OH, int OW, int kh, int kw,
                                int sh, int sw, int dh, int dw, int pt, int pl,
                                const float* residual, int act, float lo, float hi,
                                hipStream_t s) {
  const int64_t total = (int64_t)N * C * OH * OW;
  if (total == 0) return RTENHIP_OK;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  if (kw <= 8 && total + blocks * 256 < (int64_t(1) << 31) &&
      (int64_t)N * C * H * W < (int64_t(1) << 31)) {
    DwBounds b{};
    for (int kx = 0; kx < kw; kx++) {
      const int kxd = kx * dw;
      b.omin[kx] = pl - kxd > 0 ? pl - kxd : 0;
      const int t = W + pl - kxd > 0 ? W + pl - kxd : 0;
      int omax = (t + sw - 1) / sw;
      b.omax[kx] = omax > OW ? OW : omax;
    }
    const int planes = N * C;
    // Small square planes (28x28, 14x14, 7x7) without a residual: the streaming
    // kernel (dw_stream.hip), copies of later plane groups in flight while a
    // group computes.
    rtenhip_status dws_st = RTENHIP_OK;
    if (launch_depthwise_stream(x, w, bias, y, N, C, H, W, OH, OW, kh, kw, sh, sw, dh, dw, pt, pl, b.omin, b.omax,
                                residual, act, lo, hi, s, dws_st))
      return dws_st;
    // 4 output columns per thread (depthwise_lds4_kernel) where it applies:
    // stride 1 (3.1 -> 4.1 TB/s on MobileNetV2's s1 layers).  The stride-2
    // instance is bit-exact too but slower than depthwise_lds_kernel there
    // (4.3 -> 3.3 TB/s on 112x112 s2: one plane and 98 threads per block), so
    // it is not dispatched.
    static const bool dw4_on = [] {
      const char* e = getenv("RTENHIP_DW4");  // A/B experiments: 0 disables
      return !(e && atoi(e) == 0);
    }();
    const int pr = (OW - 1) * sw + (kw - 1) * dw + 1 - W - pl;  // right padding actually read
    const bool al16 = ((uintptr_t)x | (uintptr_t)y | (uintptr_t)residual) % 16 == 0;
    Dw4Geom g4;
    if (dw4_on && kh == 3 && kw == 3 && dh == 1 && dw == 1 && sh == 1 && sw == 1 && al16 &&
        dw4_geometry(H, W, OH, OW, sh, pt, pl, pr, g4)) {
      dim3 grid((unsigned)((OH + g4.RS * DW4_TR - 1) / (g4.RS * DW4_TR)), (unsigned)((planes + g4.PB - 1) / g4.PB));
      if (grid.y <= 65535) {
        const int threads = (g4.PB * g4.RS * (OW / 4) + 63) / 64 * 64;
        if (sh == 1)
          hipLaunchKernelGGL(depthwise_lds4_kernel<1>, grid, dim3(threads), g4.lds, s, x, w, bias, y, planes, C,
                             H, W, OH, OW, pt, pl, g4.RS, g4.PB, g4.rows_in, b, residual, act, lo, hi);
        else
          hipLaunchKernelGGL(depthwise_lds4_kernel<2>, grid, dim3(threads), g4.lds, s, x, w, bias, y, planes, C,
                             H, W, OH, OW, pt, pl, g4.RS, g4.PB, g4.rows_in, b, residual, act, lo, hi);
        RTENHIP_LAUNCH_CHECK();
        return RTENHIP_OK;
      }
    }
    // LDS tiling (depthwise_lds_kernel): PB planes x OW columns of threads,
    // TH output rows each, at most 16 KB of staged input per block.
    if (OW <= 256 && kh * kw <= 64) {
      const int PB = 256 / OW;
      auto rows_for = [&](int th) { return (th - 1) * sh + (kh - 1) * dh + 1; };
      int TH = OH;
      // 8192 floats: MobileNetV2's 14 -> 7 stride-2 layer then stages whole
      // planes (0.054 -> 0.022 ms); the other layers are unchanged and 16384
      // slows the 28 -> 14 one (profiles/r4_dw_budget.txt).
      static const int budget = [] {
        const char* e = getenv("RTENHIP_DW_LDS_FLOATS");  // tuning experiments
        return e ? atoi(e) : 8192;
      }();
      while (TH > 1 && PB * rows_for(TH) * W > budget) TH = (TH + 1) / 2;
      const int rows_in = rows_for(TH);
      static const bool flat_on = [] {
        const char* e = getenv("RTENHIP_DW_FLAT");  // A/B experiments: 0 disables
        return !(e && atoi(e) == 0);
      }();
      // Whole planes per block, rows not a multiple of 4 floats: stage the
      // block's contiguous planes with 16-byte copies (see the kernel).
      const int flat = flat_on && TH == OH && (W & 3) != 0 && ((int64_t)PB * H * W) % 4 == 0 &&
                       ((uintptr_t)x & 15) == 0;
      const size_t lds = (size_t)PB * (flat ? std::max(rows_in, H) : rows_in) * W * sizeof(float);
      dim3 grid((unsigned)((OH + TH - 1) / TH), (unsigned)((planes + PB - 1) / PB));
      if (lds <= 64 * 1024 && grid.y <= 65535) {
        const int threads = (PB * OW + 63) / 64 * 64;
        if (kh == 3 && kw == 3)
          hipLaunchKernelGGL((depthwise_lds_kernel<3, 3>), grid, dim3(threads), lds, s, x, w, bias,
                             y, planes, C, H, W, OH, OW, kh, kw, sh, sw, dh, dw, pt, pl, TH, PB,
                             rows_in, b, residual, act, lo, hi, flat);
        else
          hipLaunchKernelGGL((depthwise_lds_kernel<0, 0>), grid, dim3(threads), lds, s, x, w, bias,
                             y, planes, C, H, W, OH, OW, kh, kw, sh, sw, dh, dw, pt, pl, TH, PB,
                             rows_in, b, residual, act, lo, hi, flat);
        RTENHIP_LAUNCH_CHECK();
        return RTENHIP_OK;
      }
    }
    hipLaunchKernelGGL(depthwise32_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x, w, bias, y,
                       (int)total, C, H, W, OH, OW, kh, kw, sh, sw, dh, dw, pt, pl,
                       make_fastdiv((uint32_t)OW), make_fastdiv((uint32_t)OH),
                       make_fastdiv((uint32_t)C), b, residual, act, lo, hi);
    RTENHIP_LAUNCH_CHECK();
    return RTENHIP_OK;
  }
  hipLaunchKernelGGL(depthwise_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x, w, bias, y,
                     total, C, H, W, OH, OW, kh, kw, sh, sw, dh, dw, pt, pl, residual, act, lo,
                     hi);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

}  // namespace rtenhip
