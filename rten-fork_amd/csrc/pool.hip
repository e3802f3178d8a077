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
#include "vecmath.h"

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

rtenhip_status launch_pool(int is_max, const float* x, float* y, int64_t NC, int H, int W,
                           int OH, int OW, int kh, int kw, int sh, int sw, int pt, int pl,
                           int count_include_pad, hipStream_t s) {
  const int64_t total = NC * OH * OW;
  if (total == 0) return RTENHIP_OK;
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

rtenhip_status launch_gap(const float* x, float* y, int64_t NC, int64_t HW, hipStream_t s) {
  if (NC == 0) return RTENHIP_OK;
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

rtenhip_status launch_depthwise(const float* x, const float* w, const float* bias, float* y,
                                int N, int C, int H, int W, int OH, int OW, int kh, int kw,
                                int sh, int sw, int dh, int dw, int pt, int pl,
                                const float* residual, int act, float lo, float hi,
                                hipStream_t s) {
  const int64_t total = (int64_t)N * C * OH * OW;
  if (total == 0) return RTENHIP_OK;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(depthwise_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x, w, bias, y,
                     total, C, H, W, OH, OW, kh, kw, sh, sw, dh, dw, pt, pl, residual, act, lo,
                     hi);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

}  // namespace rtenhip
