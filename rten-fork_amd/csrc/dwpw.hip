// MobileNetV2 inverted-residual back half in one kernel: a 3x3 stride-1
// depthwise conv (+ bias, Clip / Relu) feeding the block's 1x1 project conv
// (+ bias, residual, activation), without writing the depthwise output to HBM
// and reading it back.  At batch 128 that output is 205 MB for features.1 and
// 231 MB for features.3.
//
// Arithmetic is exactly that of the two operators run apart, so the result is
// bit-identical to the unfused graph and to RTen:
//  - depthwise (conv_2d_depthwise_block, src/ops/conv/depthwise.rs:49-120):
//    bias, then + v * w over the taps in ky, kx order with separate roundings,
//    skipping rows outside the image and columns outside the reference's
//    min_max_out_x_coords range (depthwise.rs:24-38), then the activation --
//    the operations of depthwise_lds4_kernel (pool.hip) and mbconv.hip;
//  - project (conv_2d_pointwise, src/ops/conv.rs:24-68; K = C <= 256, one KC
//    block): the k-ordered fma chain from zero over the channels, + bias, the
//    residual, the activation -- conv_pw_valu_kernel's operations.
//
// Layout: a block owns one image and a band of TR output rows (all columns):
// thread (tr, t) owns output row oy0 + tr, columns 4t .. 4t + 3, and the
// MC <= 32 project outputs of those 4 pixels in registers (MC x 4 chains).
// The channels run in order: channel c's TR + 2 input rows are staged in LDS
// (double-buffered, loaded one channel ahead into registers, one barrier per
// channel); each thread forms its 4 depthwise values and fma's them into its
// project chains with the channel's weights as scalar operands.
//
// Measured slower than the two kernels apart (profiles/r3_dwpw_ab.txt): the
// channel loop is a serial chain of barrier + memory round trips per block
// (features.1: 0.19 ms vs 0.098 + 0.077; 192-channel 28x28 pairs 0.49 vs
// 0.064 ms), and loading channels 4 ahead or the weights as vector loads did
// not change that.  So the fusion is opt-in (RTENHIP_DWPW=1); bit-exact either way.
#include <algorithm>

#include "common.h"
#include "vecmath.h"

namespace rtenhip {

typedef float f32x2 __attribute__((ext_vector_type(2)));

struct DwPwDesc {
  const float* x;         // [N, C, H, W] depthwise input
  const float* wd;        // [C, 9]
  const float* bd;        // [C] or null
  const float* wt;        // [C][Mpad] project weights, transposed (pack_pw_weights)
  const float* bp;        // [M] or null
  const float* residual;  // [N, M, H, W] or null
  float* y;               // [N, M, H, W]
  int C, H, W, M, Mpad, pt, pl;
  int TR, rows_in, LW, tiles_y;
  int act_d, act_p;
  float lo_d, hi_d, lo_p, hi_p;
  int omin[3], omax[3];  // min_max_out_x_coords per kx
};

constexpr int kDpQ = 2;   // staged float4 per thread and channel (rows_in * W / 4 <= 512)

__device__ __forceinline__ float dp_act_d(float v, int act, float lo, float hi) {
  if (act == RTENHIP_ACT_RELU) return rust_max(v, 0.f);
  if (act == RTENHIP_ACT_CLIP) return rust_clamp(v, lo, hi);
  return v;
}

__device__ __forceinline__ float dp_act_p(float x, int act, float lo, float hi) {
  if (act == RTENHIP_ACT_RELU) return fmaxf(x, 0.f);
  if (act == RTENHIP_ACT_CLIP) return x < lo ? lo : (x > hi ? hi : x);
  return x;
}

template <int MC>
__global__ __launch_bounds__(256) void dw_pw_kernel(DwPwDesc d) {
  extern __shared__ float4 dp_lds4[];
  float* lds = reinterpret_cast<float*>(dp_lds4);
  const int plane = d.rows_in * d.LW;  // floats per staged channel
  const int tid = threadIdx.x;
  const int img = (int)blockIdx.x / d.tiles_y;
  const int oy0 = ((int)blockIdx.x - img * d.tiles_y) * d.TR;
  const int OW4 = d.W >> 2;
  const int tr = tid / OW4, t = tid - tr * OW4;
  const int oy = oy0 + tr;
  const bool active = tr < d.TR && oy < d.H;
  const int ox0 = 4 * t;

  // Which taps the reference takes for this thread's 4 outputs.
  bool rok[3], cok[4][3];
#pragma unroll
  for (int ky = 0; ky < 3; ky++) rok[ky] = oy - d.pt + ky >= 0 && oy - d.pt + ky < d.H;
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int kx = 0; kx < 3; kx++) cok[i][kx] = ox0 + i >= d.omin[kx] && ox0 + i < d.omax[kx];

  // Staging: slot s = (row r, float4 c4) of the channel's rows_in x W band;
  // LDS position j of a row holds input column j - 4 (16-byte aligned rows).
  const int W4 = d.W >> 2;
  const int nslots = d.rows_in * W4;
  const int iy_lo = oy0 - d.pt;
  const int64_t HW = (int64_t)d.H * d.W;
  const float* __restrict__ xi = d.x + (int64_t)img * d.C * HW;
  int soff[kDpQ], loff[kDpQ];
  bool sok[kDpQ];
#pragma unroll
  for (int q = 0; q < kDpQ; q++) {
    const int s = tid + 256 * q;
    const int r = s / W4, c4 = s - (s / W4) * W4;
    const int iy = iy_lo + r;
    sok[q] = s < nslots && iy >= 0 && iy < d.H;
    soff[q] = sok[q] ? iy * d.W + 4 * c4 : 0;
    loff[q] = s < nslots ? r * d.LW + 4 + 4 * c4 : -1;
  }
  float4 pre[kDpQ];
  auto load_c = [&](int c) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < kDpQ; q++)
      pre[q] = sok[q] ? *(const float4*)(xi + c * HW + soff[q]) : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  auto store_c = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < kDpQ; q++)
      if (loff[q] >= 0) *(float4*)(lds + buf * plane + loff[q]) = pre[q];
  };

  f32x2 acc[MC][2];
#pragma unroll
  for (int m = 0; m < MC; m++) acc[m][0] = acc[m][1] = (f32x2){0.f, 0.f};
  // This thread's window: row tr + ky, positions ox0 .. ox0 + 11 (three
  // 16-byte reads); output i, tap kx reads position ox0 + 3 + i + kx (input
  // column ox0 + i + kx - 1: pad 1).
  constexpr int o = 3;
  const int wbase = tr * d.LW + ox0;

  load_c(0);
  for (int c = 0; c < d.C; c++) {
    const int buf = c & 1;
    store_c(buf);
    if (c + 1 < d.C) load_c(c + 1);
    __syncthreads();
    if (active) {
      const float* __restrict__ wdc = d.wd + 9 * c;
      const float bdc = d.bd ? d.bd[c] : 0.f;
      float dv[4] = {bdc, bdc, bdc, bdc};
#pragma unroll
      for (int ky = 0; ky < 3; ky++) {
        const float4* rp = reinterpret_cast<const float4*>(lds + buf * plane + wbase + ky * d.LW);
        const float4 s0 = rp[0], s1 = rp[1], s2 = rp[2];
        const float win[12] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w, s2.x, s2.y, s2.z, s2.w};
#pragma unroll
        for (int kx = 0; kx < 3; kx++) {
          const float w = wdc[ky * 3 + kx];
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const float nv = __fadd_rn(dv[i], __fmul_rn(win[o + i + kx], w));
            dv[i] = rok[ky] && cok[i][kx] ? nv : dv[i];
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 4; i++) dv[i] = dp_act_d(dv[i], d.act_d, d.lo_d, d.hi_d);
      const f32x2 xa = {dv[0], dv[1]}, xb = {dv[2], dv[3]};
      const float* __restrict__ wr = d.wt + (int64_t)c * d.Mpad;
#pragma unroll
      for (int m = 0; m < MC; m++) {
        const f32x2 wv = {wr[m], wr[m]};
        acc[m][0] = __builtin_elementwise_fma(wv, xa, acc[m][0]);
        acc[m][1] = __builtin_elementwise_fma(wv, xb, acc[m][1]);
      }
    }
  }
  if (!active) return;
  const int64_t P = HW;
  const int64_t pix = (int64_t)oy * d.W + ox0;
#pragma unroll
  for (int m = 0; m < MC; m++) {
    if (m >= d.M) continue;
    float4 v = make_float4(acc[m][0].x, acc[m][0].y, acc[m][1].x, acc[m][1].y);
    if (d.bp) {
      const float b = d.bp[m];
      v.x = __fadd_rn(v.x, b);
      v.y = __fadd_rn(v.y, b);
      v.z = __fadd_rn(v.z, b);
      v.w = __fadd_rn(v.w, b);
    }
    const int64_t oi = ((int64_t)img * d.M + m) * P + pix;
    if (d.residual) {
      const float4 r = *(const float4*)(d.residual + oi);
      v.x = __fadd_rn(v.x, r.x);
      v.y = __fadd_rn(v.y, r.y);
      v.z = __fadd_rn(v.z, r.z);
      v.w = __fadd_rn(v.w, r.w);
    }
    v.x = dp_act_p(v.x, d.act_p, d.lo_p, d.hi_p);
    v.y = dp_act_p(v.y, d.act_p, d.lo_p, d.hi_p);
    v.z = dp_act_p(v.z, d.act_p, d.lo_p, d.hi_p);
    v.w = dp_act_p(v.w, d.act_p, d.lo_p, d.hi_p);
    *(float4*)(d.y + oi) = v;
  }
}

// Band height: rows of OW / 4 threads in a 256-thread block, the staged band
// (TR + 2 rows) within kDpQ float4 per thread; bands balanced over OH.
static int dw_pw_rows(int H, int W) {
  const int ow4 = W / 4;
  if (ow4 < 1 || ow4 > 256) return 0;
  // (at least 4 bands per image where H allows: enough blocks to fill the
  // chip at the 28x28 layers, whose rows are only 7 threads wide)
  int tr = std::min(std::max(1, H / 4), 256 / ow4);
  while (tr >= 1 && (tr + 2) * ow4 > 256 * kDpQ) tr--;
  if (tr < 1) return 0;
  const int bands = (H + tr - 1) / tr;
  return (H + bands - 1) / bands;
}

bool dw_pw_eligible(int C, int H, int W, int M, int pt, int pl, int pb, int pr) {
  // 3x3, stride 1, pad 1 on every side: the output has the input's size.
  return C >= 1 && C <= 1024 && M >= 1 && M <= 32 && W % 4 == 0 && pt == 1 && pb == 1 && pl == 1 && pr == 1 &&
         dw_pw_rows(H, W) > 0 && (int64_t)C * H * W < (1ll << 31);
}

rtenhip_status launch_dw_pw(const float* x, const float* wd, const float* bd, const float* wt, const float* bp,
                            const float* residual, float* y, int N, int C, int H, int W, int M, int pt, int pl,
                            int act_d, float lo_d, float hi_d, int act_p, float lo_p, float hi_p, hipStream_t s) {
  if (!dw_pw_eligible(C, H, W, M, pt, pl, pt, pl) || ((uintptr_t)x | (uintptr_t)y) % 16 ||
      (residual && (uintptr_t)residual % 16))
    return fail(RTENHIP_INVALID_VALUE, "depthwise+pointwise: unsupported shape");
  DwPwDesc d{};
  d.x = x;
  d.wd = wd;
  d.bd = bd;
  d.wt = wt;
  d.bp = bp;
  d.residual = residual;
  d.y = y;
  d.C = C;
  d.H = H;
  d.W = W;
  d.M = M;
  d.Mpad = (M + 31) / 32 * 32;
  d.pt = pt;
  d.pl = pl;
  d.TR = dw_pw_rows(H, W);
  d.rows_in = d.TR + 2;
  d.LW = W + 12;
  d.tiles_y = (H + d.TR - 1) / d.TR;
  d.act_d = act_d;
  d.lo_d = lo_d;
  d.hi_d = hi_d;
  d.act_p = act_p;
  d.lo_p = lo_p;
  d.hi_p = hi_p;
  // min_max_out_x_coords (depthwise.rs:24-38) for stride 1, dilation 1 and
  // OW = W, the bounds launch_depthwise passes its kernels.
  for (int kx = 0; kx < 3; kx++) {
    d.omin[kx] = pl - kx > 0 ? pl - kx : 0;
    d.omax[kx] = std::min(W, W + pl - kx);
  }
  const size_t bytes = (size_t)2 * d.rows_in * d.LW * 4;
  const unsigned blocks = (unsigned)((int64_t)N * d.tiles_y);
  if (blocks == 0) return RTENHIP_OK;
  if (M <= 16)
    dw_pw_kernel<16><<<blocks, 256, bytes, s>>>(d);
  else if (M <= 24)
    dw_pw_kernel<24><<<blocks, 256, bytes, s>>>(d);
  else
    dw_pw_kernel<32><<<blocks, 256, bytes, s>>>(d);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

}  // namespace rtenhip
