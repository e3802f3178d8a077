// MobileNetV2 inverted-residual front half in one kernel: the 1x1 expand
// conv (+ bias, Clip) feeding a 3x3 depthwise conv (+ bias, Clip), without
// writing the expand output to HBM and reading it back.  At batch 128 the
// expand outputs are 13 MB per image (616 MB for features.2 alone); here
// they live only in LDS, one channel at a time.
//
// Arithmetic is exactly that of the two operators run apart (so the result is
// bit-identical to the unfused graph and to RTen):
//  - expand (conv_2d_pointwise, src/ops/conv.rs:24-68; K = C_in <= 256, one
//    KC block): the k-ordered fma chain from zero (kernels.rs:206-316), then
//    + bias (gemm.rs:1034-1047), then the graph's Clip / Relu (the same
//    operations as conv_pw_valu_kernel and the DMA GEMM epilogue);
//  - depthwise (conv_2d_depthwise_block, src/ops/conv/depthwise.rs:49-120):
//    bias, then + v * w over the taps in ky, kx order with separate roundings,
//    skipping rows outside the image and columns outside the reference's
//    min_max_out_x_coords range, then Clip / Relu.
//
// Layout: a block owns one image, a band of TR output rows and a chunk of
// channels.  Its input rows (C_in x rows_in x W, rows_in = (TR-1)*S + 3) are
// loaded once into VGPRs -- thread t holds 4 consecutive pixels of one input
// row for all C_in channels -- so the x band is read from HBM once per block.
// Per channel: every thread forms its 4 expand values (C_in packed FMAs with
// the channel's weights as scalar operands) and stores them to an LDS plane
// (double-buffered, one barrier per channel); then the band's depthwise
// outputs are computed from LDS and stored (coalesced rows).
#include "common.h"
#include "vecmath.h"

namespace rtenhip {

typedef float f32x2 __attribute__((ext_vector_type(2)));

struct ExpandDwDesc {
  const float* x;   // [N, CIN, H, W]
  const float* we;  // [hidden, CIN] expand weights
  const float* be;  // [hidden] or null
  const float* wd;  // [hidden, 9] depthwise weights
  const float* bd;  // [hidden] or null
  float* y;         // [N, hidden, OH, OW]
  int hidden, H, W, OH, OW, pt, pl;
  int TR, rows_in, cpb;  // output rows per band, staged input rows, channels per block
  int act_e, act_d;
  float lo_e, hi_e, lo_d, hi_d;
  int omin[3], omax[3];  // min_max_out_x_coords per kx (depthwise.rs:24-38)
};

__device__ __forceinline__ float ed_act(float v, int act, float lo, float hi) {
  if (act == RTENHIP_ACT_RELU) return rust_max(v, 0.f);
  if (act == RTENHIP_ACT_CLIP) return rust_clamp(v, lo, hi);
  return v;
}

constexpr int kEdMargin = 4;  // floats before each LDS plane (never read: colok)

template <int CIN, int S>
__global__ __launch_bounds__(256) void expand_dw_kernel(ExpandDwDesc d) {
  extern __shared__ float4 ed_lds4[];
  float* lds = reinterpret_cast<float*>(ed_lds4);
  const int plane = d.rows_in * d.W + 2 * kEdMargin;  // one buffer of the double buffer
  const int n = blockIdx.y;
  const int oy0 = blockIdx.x * d.TR;
  const int iy_lo = oy0 * S - d.pt;  // input row of LDS row 0
  const int c_begin = blockIdx.z * d.cpb;
  const int c_end = min(d.hidden, c_begin + d.cpb);
  const int W4 = d.W >> 2;
  const int t = threadIdx.x;
  const int er = t / W4, ec = (t - er * W4) * 4;  // this thread's expand pixels: LDS row er, cols ec..ec+3
  const int iy = iy_lo + er;
  const bool e_on = er < d.rows_in && iy >= 0 && iy < d.H;
  const int64_t HW = (int64_t)d.H * d.W;
  float4 xr[CIN];
  if (e_on) {
    const float* xp = d.x + ((int64_t)n * CIN) * HW + (int64_t)iy * d.W + ec;
#pragma unroll
    for (int k = 0; k < CIN; k++) xr[k] = *(const float4*)(xp + k * HW);
  }
  const int oh_blk = min(d.TR, d.OH - oy0);
  const int n_out = oh_blk * d.OW;
  for (int c = c_begin; c < c_end; c++) {
    float* eb = lds + (c & 1) * plane + kEdMargin;
    if (e_on) {
      const float* __restrict__ wc = d.we + (int64_t)c * CIN;
      f32x2 a0 = {0.f, 0.f}, a1 = {0.f, 0.f};
#pragma unroll
      for (int k = 0; k < CIN; k++) {
        const f32x2 wv = {wc[k], wc[k]};
        a0 = __builtin_elementwise_fma(wv, (f32x2){xr[k].x, xr[k].y}, a0);
        a1 = __builtin_elementwise_fma(wv, (f32x2){xr[k].z, xr[k].w}, a1);
      }
      float4 v = make_float4(a0.x, a0.y, a1.x, a1.y);
      if (d.be) {
        const float b = d.be[c];
        v.x = __fadd_rn(v.x, b);
        v.y = __fadd_rn(v.y, b);
        v.z = __fadd_rn(v.z, b);
        v.w = __fadd_rn(v.w, b);
      }
      v.x = ed_act(v.x, d.act_e, d.lo_e, d.hi_e);
      v.y = ed_act(v.y, d.act_e, d.lo_e, d.hi_e);
      v.z = ed_act(v.z, d.act_e, d.lo_e, d.hi_e);
      v.w = ed_act(v.w, d.act_e, d.lo_e, d.hi_e);
      *(float4*)(eb + er * d.W + ec) = v;
    }
    // One barrier per channel: the plane written next iteration is the other
    // buffer, and the one after that is only written once every thread has
    // passed the next barrier, i.e. finished reading this one.
    __syncthreads();
    const float* __restrict__ wk = d.wd + (int64_t)c * 9;
    const float b0 = d.bd ? d.bd[c] : 0.f;
    float* yc = d.y + ((int64_t)n * d.hidden + c) * d.OH * d.OW;
    for (int o = t; o < n_out; o += 256) {
      const int ol = o / d.OW, ox = o - ol * d.OW;
      const int oy = oy0 + ol;
      float acc = b0;
#pragma unroll
      for (int ky = 0; ky < 3; ky++) {
        const int r = oy * S + ky - d.pt;  // input row
        if (r < 0 || r >= d.H) continue;
        const float* row = eb + (r - iy_lo) * d.W + ox * S - d.pl;
#pragma unroll
        for (int kx = 0; kx < 3; kx++) {
          if (ox < d.omin[kx] || ox >= d.omax[kx]) continue;
          acc = __fadd_rn(acc, __fmul_rn(row[kx], wk[ky * 3 + kx]));
        }
      }
      yc[(int64_t)oy * d.OW + ox] = ed_act(acc, d.act_d, d.lo_d, d.hi_d);
    }
  }
}

// Whether the fused kernel takes this pair: C_in in {16, 24, 32} (the x band
// in VGPRs), 3x3 depthwise with stride 1 or 2, no dilation, pads <= 1, W a
// multiple of 4 with a band of rows that fits one pass of 256 threads.
bool expand_dw_eligible(int cin, int W, int S, int pt, int pl, int pb, int pr) {
  if (cin != 16 && cin != 24 && cin != 32) return false;
  if (S != 1 && S != 2) return false;
  if (W % 4 != 0 || W / 4 > 256 / 3 || pt > 1 || pl > 1 || pb > 1 || pr > 1) return false;
  return (256 / (W / 4)) >= 3;  // at least one output row per band
}

rtenhip_status launch_expand_dw(const float* x, const float* we, const float* be, const float* wd, const float* bd,
                                float* y, int N, int cin, int hidden, int H, int W, int OH, int OW, int S, int pt,
                                int pl, int act_e, float lo_e, float hi_e, int act_d, float lo_d, float hi_d,
                                hipStream_t s) {
  if ((int64_t)N * hidden * OH * OW == 0) return RTENHIP_OK;
  ExpandDwDesc d{};
  d.x = x;
  d.we = we;
  d.be = be;
  d.wd = wd;
  d.bd = bd;
  d.y = y;
  d.hidden = hidden;
  d.H = H;
  d.W = W;
  d.OH = OH;
  d.OW = OW;
  d.pt = pt;
  d.pl = pl;
  d.act_e = act_e;
  d.lo_e = lo_e;
  d.hi_e = hi_e;
  d.act_d = act_d;
  d.lo_d = lo_d;
  d.hi_d = hi_d;
  for (int kx = 0; kx < 3; kx++) {
    d.omin[kx] = pl - kx > 0 ? pl - kx : 0;
    const int t = W + pl - kx > 0 ? W + pl - kx : 0;
    const int omax = (t + S - 1) / S;
    d.omax[kx] = omax > OW ? OW : omax;
  }
  // Band: the most output rows whose input rows fit one pass of 256 threads.
  const int W4 = W / 4;
  const int max_rows = 256 / W4;
  d.TR = std::max(1, std::min(OH, (max_rows - 3) / S + 1));
  d.rows_in = (d.TR - 1) * S + 3;
  const int bands = (OH + d.TR - 1) / d.TR;
  // Channel chunks: enough blocks to fill the chip a few times over, at least
  // 16 channels per chunk (each chunk re-reads the x band).
  int chunks = 1;
  while ((int64_t)bands * N * chunks < 1024 && hidden / (chunks * 2) >= 16) chunks *= 2;
  d.cpb = (hidden + chunks - 1) / chunks;
  const size_t lds = 2 * ((size_t)d.rows_in * W + 2 * kEdMargin) * sizeof(float);
  if (lds > 64 * 1024 || N > 65535 || chunks > 65535) return fail(RTENHIP_UNSUPPORTED_VALUE, "expand+depthwise tile too large");
  dim3 grid((unsigned)bands, (unsigned)N, (unsigned)chunks);
#define ED_CASE(C, SS) \
  if (cin == C && S == SS) { \
    hipLaunchKernelGGL((expand_dw_kernel<C, SS>), grid, dim3(256), lds, s, d); \
    RTENHIP_LAUNCH_CHECK(); \
    return RTENHIP_OK; \
  }
  ED_CASE(16, 1)
  ED_CASE(16, 2)
  ED_CASE(24, 1)
  ED_CASE(24, 2)
  ED_CASE(32, 1)
  ED_CASE(32, 2)
#undef ED_CASE
  return fail(RTENHIP_UNSUPPORTED_VALUE, "expand+depthwise: unsupported channel count");
}

}  // namespace rtenhip
