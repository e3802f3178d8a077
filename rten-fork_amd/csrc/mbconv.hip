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
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "common.h"
#include "vecmath.h"
#include "stage.h"

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

constexpr int kEdMaxQ = 4;   // depthwise outputs per thread and channel (TR * OW <= 1024)
constexpr int kEdZs = 16;    // floats before a plane's interior: the 9 zero slots (+ pad)

// Expand plane size in floats (zero slots, rows_in rows of W, a tail margin).
__host__ __device__ inline int ed_plane(int rows_in, int W) { return kEdZs + rows_in * W + 4; }

// Position of input column ix within an expand plane row.  At stride 2 a row
// is stored de-interleaved -- the even columns, then the odd ones -- so the
// taps of consecutive outputs (columns 2 ox - 1, 2 ox, 2 ox + 1) are
// consecutive LDS words instead of every other one (2-way bank conflicts).
template <int S>
__device__ __forceinline__ int ed_col(int ix, int W) {
  if constexpr (S == 2) return (ix & 1) * (W >> 1) + (ix >> 1);
  return ix;
}

// CP channels per pass (one barrier per pass); PLANE = ed_plane(...) when
// compile-time (every LDS offset an immediate), 0 = runtime.  The block's
// expand and depthwise weights and biases are staged in LDS once; each
// thread's depthwise outputs have their 9 tap addresses fixed before the
// channel loop.  A tap the reference skips (a row outside the image, a column
// outside min_max_out_x_coords) is pointed at a per-channel "zero slot"
// holding copysign(0, -w): its product is exactly -0, and x + (-0) == x for
// every x (+-0, inf and NaN included), so adding it is the skip -- for finite
// w.  A channel with a non-finite tap weight takes the select path instead.
// CLIPS: both activations are Clip (MobileNetV2's ReLU6), compiled in rather
// than selected per value at run time.
// MX (CP == 4): the expand on v_mfma_f32_4x4x1_16b_f32 (a chain of them is
// bitwise the k-ordered fmaf chain, tools/probes/mfma4x4_probe.hip): the
// block's 4 rows are the pass's 4 channels (lane l supplies the weight of
// channel c0 + l % 4), its columns 4 lanes' pixels, one MFMA chain per pixel
// of the lane's float4; lane l then holds channel c0 + r of its 4 pixels in
// register r of the 4 chains.  Every lane of the wave takes part (lanes
// outside the band run on zeros and store nothing).
template <int CIN, int S, int CP, int PLANE, int NQ, bool CLIPS, bool MX = false>
__global__ __launch_bounds__(256) void expand_dw_kernel(ExpandDwDesc d) {
  static_assert(!MX || CP == 4, "MFMA expand passes are 4 channels");
  extern __shared__ float4 ed_lds4[];
  float* lds = reinterpret_cast<float*>(ed_lds4);
  const int plane = PLANE > 0 ? PLANE : ed_plane(d.rows_in, d.W);
  const int n = blockIdx.y;
  const int oy0 = blockIdx.x * d.TR;
  const int iy_lo = oy0 * S - d.pt;  // input row of LDS row 0
  const int c_begin = blockIdx.z * d.cpb;
  const int c_end = min(d.hidden, c_begin + d.cpb);
  const int cnt = c_end - c_begin;
  float* w_e = lds + 2 * CP * plane;  // [cnt][CIN]
  float* w_d = w_e + d.cpb * CIN;     // [cnt][9]
  float* b_e = w_d + d.cpb * 9;       // [cnt]
  float* b_d = b_e + d.cpb;           // [cnt]
  int* fin = reinterpret_cast<int*>(b_d + d.cpb);  // [cnt]: every tap weight finite
  const int t = threadIdx.x;
  stage_batched<4, float>(cnt * CIN, [&](int e) { return d.we[(int64_t)c_begin * CIN + e]; },
                          [&](int e, float v) { w_e[e] = v; });
  stage_batched<4, float>(cnt * 9, [&](int e) { return d.wd[(int64_t)c_begin * 9 + e]; },
                          [&](int e, float v) { w_d[e] = v; });
  for (int i = t; i < cnt; i += 256) {
    b_e[i] = d.be ? d.be[c_begin + i] : 0.f;
    b_d[i] = d.bd ? d.bd[c_begin + i] : 0.f;
    bool f = true;
    for (int k = 0; k < 9; k++) f = f && __builtin_isfinite(d.wd[(int64_t)(c_begin + i) * 9 + k]);
    fin[i] = f;
  }
  const int W4 = d.W >> 2;
  const int er = t / W4, ec = (t - er * W4) * 4;  // this thread's expand pixels: LDS row er, cols ec..ec+3
  const int iy = iy_lo + er;
  const bool e_on = er < d.rows_in && iy >= 0 && iy < d.H;
  const int64_t HW = (int64_t)d.H * d.W;
  float4 xr[CIN];
  if (MX && !e_on) {
#pragma unroll
    for (int k = 0; k < CIN; k++) xr[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (e_on) {
    const float* xp = d.x + ((int64_t)n * CIN) * HW + (int64_t)iy * d.W + ec;
#pragma unroll
    for (int k = 0; k < CIN; k++) xr[k] = *(const float4*)(xp + k * HW);
  }
  // Depthwise outputs o = t + 256 q of the band: tap addresses (floats from
  // the plane start; a skipped tap -> its zero slot) and the skip mask.
  const int n_out = min(d.TR, d.OH - oy0) * d.OW;
  int taddr[NQ][9];
  uint32_t tmask[NQ];
#pragma unroll
  for (int q = 0; q < NQ; q++) {
    const int o = t + 256 * q;
    const int ol = o / d.OW, ox = o - ol * d.OW;
    const int oy = oy0 + ol;
    const int rbase = kEdZs + ol * S * d.W;  // LDS row ol * S
    uint32_t m = o < n_out ? 1u << 9 : 0u;  // bit 9: an output of this band
#pragma unroll
    for (int ky = 0; ky < 3; ky++) {
      const int r = oy * S + ky - d.pt;
      const bool row_ok = r >= 0 && r < d.H;
#pragma unroll
      for (int kx = 0; kx < 3; kx++) {
        const bool on = o < n_out && row_ok && ox >= d.omin[kx] && ox < d.omax[kx];
        m |= on ? 1u << (ky * 3 + kx) : 0u;
        taddr[q][ky * 3 + kx] = on ? rbase + ky * d.W + ed_col<S>(ox * S + kx - d.pl, d.W) : ky * 3 + kx;
      }
    }
    tmask[q] = m;
  }
  const bool e_act_relu = d.act_e == RTENHIP_ACT_RELU, e_act_clip = d.act_e == RTENHIP_ACT_CLIP;
  const bool d_act_relu = d.act_d == RTENHIP_ACT_RELU, d_act_clip = d.act_d == RTENHIP_ACT_CLIP;
  auto act = [](float v, bool relu, bool clip, float lo, float hi) __attribute__((always_inline)) {
    if constexpr (CLIPS) return rust_clamp(v, lo, hi);
    const float r = rust_max(v, 0.f);
    const float c = rust_clamp(v, lo, hi);
    return relu ? r : (clip ? c : v);
  };
  __syncthreads();  // weights staged

  // One pass: CP channels from c0 into buffer B (compile-time, so with a
  // compile-time PLANE the buffer / channel offsets are LDS immediates).
  auto pass = [&](const int c0, auto Bc) __attribute__((always_inline)) {
    constexpr int B = decltype(Bc)::value;
    float* ebuf = lds + B * CP * plane;
    if constexpr (MX) {
      typedef float ed_f32x4 __attribute__((ext_vector_type(4)));
      const int lane = t & 63;
      const float* __restrict__ wl = w_e + (min(c0 + (lane & 3), c_end - 1) - c_begin) * CIN;
      ed_f32x4 acc[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int k = 0; k < CIN; k++) {
        const float w = wl[k];
        acc[0] = __builtin_amdgcn_mfma_f32_4x4x1f32(w, xr[k].x, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_4x4x1f32(w, xr[k].y, acc[1], 0, 0, 0);
        acc[2] = __builtin_amdgcn_mfma_f32_4x4x1f32(w, xr[k].z, acc[2], 0, 0, 0);
        acc[3] = __builtin_amdgcn_mfma_f32_4x4x1f32(w, xr[k].w, acc[3], 0, 0, 0);
      }
      if (e_on) {
#pragma unroll
        for (int j = 0; j < CP; j++) {
          const int cl = min(c0 + j, c_end - 1) - c_begin;
          float4 v = make_float4(acc[0][j], acc[1][j], acc[2][j], acc[3][j]);
          if (d.be) {
            const float b = b_e[cl];
            v.x = __fadd_rn(v.x, b);
            v.y = __fadd_rn(v.y, b);
            v.z = __fadd_rn(v.z, b);
            v.w = __fadd_rn(v.w, b);
          }
          v.x = act(v.x, e_act_relu, e_act_clip, d.lo_e, d.hi_e);
          v.y = act(v.y, e_act_relu, e_act_clip, d.lo_e, d.hi_e);
          v.z = act(v.z, e_act_relu, e_act_clip, d.lo_e, d.hi_e);
          v.w = act(v.w, e_act_relu, e_act_clip, d.lo_e, d.hi_e);
          float* erow = ebuf + j * plane + kEdZs + er * d.W;
          if constexpr (S == 2) {
            *(float2*)(erow + (ec >> 1)) = make_float2(v.x, v.z);
            *(float2*)(erow + (d.W >> 1) + (ec >> 1)) = make_float2(v.y, v.w);
          } else {
            *(float4*)(erow + ec) = v;
          }
        }
      }
    } else if (e_on) {
#pragma unroll
      for (int j = 0; j < CP; j++) {
        const int cl = min(c0 + j, c_end - 1) - c_begin;  // a pass past c_end recomputes the last channel (unused)
        const float* __restrict__ wc = w_e + cl * CIN;
        f32x2 a0 = {0.f, 0.f}, a1 = {0.f, 0.f};
#pragma unroll
        for (int k = 0; k < CIN; k++) {
          const f32x2 wv = {wc[k], wc[k]};
          a0 = __builtin_elementwise_fma(wv, (f32x2){xr[k].x, xr[k].y}, a0);
          a1 = __builtin_elementwise_fma(wv, (f32x2){xr[k].z, xr[k].w}, a1);
        }
        float4 v = make_float4(a0.x, a0.y, a1.x, a1.y);
        if (d.be) {
          const float b = b_e[cl];
          v.x = __fadd_rn(v.x, b);
          v.y = __fadd_rn(v.y, b);
          v.z = __fadd_rn(v.z, b);
          v.w = __fadd_rn(v.w, b);
        }
        v.x = act(v.x, e_act_relu, e_act_clip, d.lo_e, d.hi_e);
        v.y = act(v.y, e_act_relu, e_act_clip, d.lo_e, d.hi_e);
        v.z = act(v.z, e_act_relu, e_act_clip, d.lo_e, d.hi_e);
        v.w = act(v.w, e_act_relu, e_act_clip, d.lo_e, d.hi_e);
        float* erow = ebuf + j * plane + kEdZs + er * d.W;
        if constexpr (S == 2) {  // de-interleaved row: even columns, then odd ones (see ed_col)
          *(float2*)(erow + (ec >> 1)) = make_float2(v.x, v.z);
          *(float2*)(erow + (d.W >> 1) + (ec >> 1)) = make_float2(v.y, v.w);
        } else {
          *(float4*)(erow + ec) = v;
        }
      }
    }
    if (t < 9 * CP) {  // zero slots: copysign(0, -w) per tap
      const int j = t / 9, k = t - 9 * j;
      const int cl = min(c0 + j, c_end - 1) - c_begin;
      ebuf[j * plane + k] = copysignf(0.f, -w_d[cl * 9 + k]);
    }
    // One barrier per pass: the planes written next pass are the other
    // buffer, and the ones after that are only written once every thread has
    // passed the next barrier, i.e. finished reading these.
    __syncthreads();
    // Depthwise products and sums as packed pairs (v_pk_mul / v_pk_add: each
    // component rounds exactly as the scalar op): two outputs of a channel
    // when a thread has several (stride 1), else the pass's two channels.
    if constexpr (NQ == 1 && (CP == 2 || CP == 4)) {
      const int cl0 = c0 - c_begin;
      bool all = c0 + CP - 1 < c_end;
#pragma unroll
      for (int j = 0; j < CP; j++) all = all && fin[min(cl0 + j, c_end - 1 - c_begin)];
      if (all) {
        if (tmask[0] >> 9) {
#pragma unroll
          for (int jp = 0; jp < CP; jp += 2) {
            const int cl = cl0 + jp;
            vm_f32x2 acc = {b_d[cl], b_d[cl + 1]};
#pragma unroll
            for (int i = 0; i < 9; i++) {
              const vm_f32x2 v = {ebuf[jp * plane + taddr[0][i]], ebuf[(jp + 1) * plane + taddr[0][i]]};
              const vm_f32x2 w = {w_d[cl * 9 + i], w_d[cl * 9 + 9 + i]};
              acc = acc + v * w;
            }
            float* y0 = d.y + ((int64_t)n * d.hidden + c0 + jp) * d.OH * d.OW + (int64_t)oy0 * d.OW + t;
            y0[0] = act(acc.x, d_act_relu, d_act_clip, d.lo_d, d.hi_d);
            y0[(int64_t)d.OH * d.OW] = act(acc.y, d_act_relu, d_act_clip, d.lo_d, d.hi_d);
          }
        }
        return;
      }
    }
#pragma unroll
    for (int j = 0; j < CP; j++) {
      const int c = c0 + j;
      if (c >= c_end) break;
      const int cl = c - c_begin;
      const float* eb = ebuf + j * plane;
      float wk[9];
#pragma unroll
      for (int i = 0; i < 9; i++) wk[i] = w_d[cl * 9 + i];
      const float b0 = b_d[cl];
      float* yc = d.y + ((int64_t)n * d.hidden + c) * d.OH * d.OW + (int64_t)oy0 * d.OW;
      if (fin[cl]) {
#pragma unroll
        for (int q = 0; q + 1 < NQ; q += 2) {
          if (!((tmask[q] | tmask[q + 1]) >> 9)) continue;  // neither is an output of this band
          // (a non-output's taps all point at zero slots: harmless reads)
          vm_f32x2 acc = {b0, b0};
#pragma unroll
          for (int i = 0; i < 9; i++) {
            const vm_f32x2 v = {eb[taddr[q][i]], eb[taddr[q + 1][i]]};
            acc = acc + v * (vm_f32x2){wk[i], wk[i]};
          }
          if (tmask[q] >> 9) yc[t + 256 * q] = act(acc.x, d_act_relu, d_act_clip, d.lo_d, d.hi_d);
          if (tmask[q + 1] >> 9) yc[t + 256 * (q + 1)] = act(acc.y, d_act_relu, d_act_clip, d.lo_d, d.hi_d);
        }
        if constexpr (NQ % 2 == 1) {
          constexpr int q = NQ - 1;
          if (tmask[q] >> 9) {
            float acc = b0;
#pragma unroll
            for (int i = 0; i < 9; i++) acc = __fadd_rn(acc, __fmul_rn(eb[taddr[q][i]], wk[i]));
            yc[t + 256 * q] = act(acc, d_act_relu, d_act_clip, d.lo_d, d.hi_d);
          }
        }
      } else {
#pragma unroll
        for (int q = 0; q < NQ; q++) {
          const uint32_t m = tmask[q];
          if (!(m >> 9)) continue;
          float acc = b0;
#pragma unroll
          for (int i = 0; i < 9; i++) {
            const float pr = __fmul_rn(eb[taddr[q][i]], wk[i]);
            acc = (m >> i) & 1u ? __fadd_rn(acc, pr) : acc;
          }
          yc[t + 256 * q] = act(acc, d_act_relu, d_act_clip, d.lo_d, d.hi_d);
        }
      }
    }
  };
  for (int c0 = c_begin; c0 < c_end; c0 += 2 * CP) {
    pass(c0, std::integral_constant<int, 0>{});
    if (c0 + CP < c_end) pass(c0 + CP, std::integral_constant<int, 1>{});
  }
}

// Small planes (MobileNetV2's 14x14 and 7x7 stages, C_in 64..160): a block
// owns one image and a chunk of channels; the image's whole x plane set
// (C_in x H*W) is staged in LDS once.  Each wave works on one channel
// sub-group (planes of at most 64 pixels: four sub-groups, a lane per pixel;
// larger planes: one sub-group, a thread per pixel), MC channels at a time:
// each x value read from LDS feeds MC fma chains, and the sub-group's weight
// rows are wave-uniform (scalar loads).  The G = sub-groups x MC expand
// planes of a pass go to LDS, then the pass's depthwise outputs.  Same
// arithmetic as expand_dw_kernel.
template <int S, int MC>
__global__ __launch_bounds__(256) void expand_dw_flat_kernel(ExpandDwDesc d, int cin) {
  extern __shared__ float4 edf_lds4[];
  const int P = d.H * d.W, OP = d.OH * d.OW;
  const bool small = P <= 64;
  const int subs = small ? 4 : 1;
  const int G = subs * MC;  // channels per pass
  float* xs = reinterpret_cast<float*>(edf_lds4);   // [cin][P]
  float* es = xs + cin * P;                          // [G][P + margins]
  const int estride = P + 2 * kEdMargin;
  const int n = blockIdx.y;
  const int c_begin = blockIdx.z * d.cpb;
  const int c_end = min(d.hidden, c_begin + d.cpb);
  const int t = threadIdx.x;
  {
    const float* xp = d.x + (int64_t)n * cin * P;
    const int total = cin * P;
    if ((total & 3) == 0 && ((uintptr_t)xp & 15) == 0) {
      stage_batched<8, float4>(total / 4, [&](int e) { return reinterpret_cast<const float4*>(xp)[e]; },
                               [&](int e, const float4& v) { reinterpret_cast<float4*>(xs)[e] = v; });
    } else {
      stage_batched<8, float>(total, [&](int e) { return xp[e]; }, [&](int e, float v) { xs[e] = v; });
    }
  }
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int px = small ? (t & 63) : t;
  const int sub = small ? wave : 0;
  const bool e_on = px < P;
  for (int c0 = c_begin; c0 < c_end; c0 += G) {
    const int cs = __builtin_amdgcn_readfirstlane(c0 + sub * MC);  // this wave's first channel
    if (e_on) {
      float acc[MC];
#pragma unroll
      for (int o = 0; o < MC; o++) acc[o] = 0.f;
      // Channels past c_end read weight row c_end - 1 (their values are unused).
      const float* __restrict__ wrow[MC];
#pragma unroll
      for (int o = 0; o < MC; o++) wrow[o] = d.we + (int64_t)min(cs + o, c_end - 1) * cin;
#pragma unroll 4
      for (int k = 0; k < cin; k++) {
        const float xv = xs[k * P + px];
#pragma unroll
        for (int o = 0; o < MC; o++) acc[o] = __fmaf_rn(wrow[o][k], xv, acc[o]);
      }
#pragma unroll
      for (int o = 0; o < MC; o++) {
        float v = acc[o];
        if (d.be) v = __fadd_rn(v, d.be[min(cs + o, c_end - 1)]);
        es[(sub * MC + o) * estride + kEdMargin + px] = ed_act(v, d.act_e, d.lo_e, d.hi_e);
      }
    }
    __syncthreads();
    const int ng = min(G, c_end - c0);
    for (int o = t; o < ng * OP; o += 256) {
      const int g = o / OP, q = o - g * OP;
      const int oy = q / d.OW, ox = q - oy * d.OW;
      const int c = c0 + g;
      const float* eb = es + g * estride + kEdMargin;
      const float* __restrict__ wk = d.wd + (int64_t)c * 9;
      float acc = d.bd ? d.bd[c] : 0.f;
#pragma unroll
      for (int ky = 0; ky < 3; ky++) {
        const int r = oy * S + ky - d.pt;
        if (r < 0 || r >= d.H) continue;
        const float* row = eb + r * d.W + ox * S - d.pl;
#pragma unroll
        for (int kx = 0; kx < 3; kx++) {
          if (ox < d.omin[kx] || ox >= d.omax[kx]) continue;
          acc = __fadd_rn(acc, __fmul_rn(row[kx], wk[ky * 3 + kx]));
        }
      }
      d.y[(((int64_t)n * d.hidden + c) * d.OH + oy) * d.OW + ox] = ed_act(acc, d.act_d, d.lo_d, d.hi_d);
    }
    // The next pass overwrites the expand planes.
    __syncthreads();
  }
}

static int flat_mc(int P) { return P <= 64 ? 8 : 16; }
static int flat_g(int P) { return (P <= 64 ? 4 : 1) * flat_mc(P); }

static bool flat_ok(int cin, int H, int W) {
  const int P = H * W;
  if (P > 256 || P < 1) return false;
  const size_t lds = ((size_t)cin * P + (size_t)flat_g(P) * (P + 2 * kEdMargin)) * sizeof(float);
  return lds <= 100 * 1024;
}

// Whether a fused kernel takes this pair: 3x3 depthwise, stride 1 or 2, no
// dilation, pads <= 1, and either C_in in {16, 24, 32} with W a multiple of 4
// (banded kernel, the x band in VGPRs) or a plane of at most 256 pixels whose
// channels fit LDS (flat kernel).
//
// Fused by default where the saved HBM round trip outweighs the kernel's VALU
// cost (measured at MobileNetV2 batch 128): the banded kernel for C_in = 16 / 24
// (features.2-4) and C_in = 32 at stride 2 (features.7).  RTENHIP_EXPAND_DW =
// "all" takes every eligible pair (tests), "0" none.
bool expand_dw_eligible(int cin, int H, int W, int S, int pt, int pl, int pb, int pr) {
  if (S != 1 && S != 2) return false;
  if (pt > 1 || pl > 1 || pb > 1 || pr > 1) return false;
  const char* e = getenv("RTENHIP_EXPAND_DW");
  const bool all = e && strcmp(e, "all") == 0;
  if (e && strcmp(e, "0") == 0) return false;
  const bool banded = (cin == 16 || cin == 24 || cin == 32) && W % 4 == 0 && W / 4 <= 256 / 3;
  // Default: the banded kernel for C_in = 16 / 24 (features.2-4: 0.197 / 0.173 / 0.122 ms fused vs
  // 0.21+ / 0.206 / 0.156 ms apart) and C_in = 32 at stride 2 (features.7: 0.052 vs 0.063 ms);
  // C_in = 32 at stride 1 is even or slower, the whole-plane kernel much slower
  // (profiles/r4_expand_dw_policy.txt).
  if (!all) return banded && (cin == 16 || cin == 24 || (cin == 32 && S == 2));
  return banded || flat_ok(cin, H, W);
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
  const bool banded = (cin == 16 || cin == 24 || cin == 32) && W % 4 == 0 && W / 4 <= 256 / 3;
  if (!banded) {
    if (!flat_ok(cin, H, W)) return fail(RTENHIP_UNSUPPORTED_VALUE, "expand+depthwise: plane too large");
    const int P = H * W, G = flat_g(P);
    int chunks = 1;
    while ((int64_t)N * chunks < 512 && hidden / (chunks * 2) >= G) chunks *= 2;
    d.cpb = (hidden + chunks - 1) / chunks;
    d.cpb = (d.cpb + G - 1) / G * G;
    chunks = (hidden + d.cpb - 1) / d.cpb;
    const size_t lds = ((size_t)cin * P + (size_t)G * (P + 2 * kEdMargin)) * sizeof(float);
    dim3 grid(1u, (unsigned)N, (unsigned)chunks);
    if (flat_mc(P) == 8) {
      if (S == 1)
        hipLaunchKernelGGL((expand_dw_flat_kernel<1, 8>), grid, dim3(256), lds, s, d, cin);
      else
        hipLaunchKernelGGL((expand_dw_flat_kernel<2, 8>), grid, dim3(256), lds, s, d, cin);
    } else {
      if (S == 1)
        hipLaunchKernelGGL((expand_dw_flat_kernel<1, 16>), grid, dim3(256), lds, s, d, cin);
      else
        hipLaunchKernelGGL((expand_dw_flat_kernel<2, 16>), grid, dim3(256), lds, s, d, cin);
    }
    RTENHIP_LAUNCH_CHECK();
    return RTENHIP_OK;
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
  constexpr int CP = 2;
  const int plane = ed_plane(d.rows_in, W);
  const size_t lds = (2 * CP * (size_t)plane + (size_t)d.cpb * (cin + 9 + 3)) * sizeof(float);
  // The expand on MFMA (MX, 4-channel passes) for the compile-time planes with
  // one depthwise output per thread and C_in >= 24 (MobileNetV2 b128 replayed:
  // features.4 103.6 vs 107.8 us, features.7 45.2 vs 46.3; features.2, C_in =
  // 16, 170.4 vs 165.9 keeps the VALU expand); RTENHIP_EDW_MX=0: the VALU
  // expand everywhere (A/B runs).
  static const bool mx_off = getenv("RTENHIP_EDW_MX") && getenv("RTENHIP_EDW_MX")[0] == '0';
  const size_t lds_mx = (2 * 4 * (size_t)plane + (size_t)d.cpb * (cin + 9 + 3)) * sizeof(float);
  if (lds > 64 * 1024 || N > 65535 || chunks > 65535 || (int64_t)d.TR * OW > 256 * kEdMaxQ)
    return fail(RTENHIP_UNSUPPORTED_VALUE, "expand+depthwise tile too large");
  dim3 grid((unsigned)bands, (unsigned)N, (unsigned)chunks);
  // Compile-time planes for MobileNetV2's pairs (features.2 / .3 / .4 / .5-6 / .7).
  const int nq = (int)((d.TR * OW + 255) / 256);  // depthwise outputs per thread and channel
  const bool clips = act_e == RTENHIP_ACT_CLIP && act_d == RTENHIP_ACT_CLIP;
#define ED_PL(C, SS, PL, Q)                                                                       \
  if (cin == C && S == SS && plane == PL && nq <= Q) {                                           \
    if (!mx_off && Q == 1 && C >= 24 && lds_mx <= 64 * 1024) {                                   \
      if (clips)                                                                                 \
        hipLaunchKernelGGL((expand_dw_kernel<C, SS, 4, PL, Q, true, true>), grid, dim3(256), lds_mx, s, d); \
      else                                                                                       \
        hipLaunchKernelGGL((expand_dw_kernel<C, SS, 4, PL, Q, false, true>), grid, dim3(256), lds_mx, s, d); \
      RTENHIP_LAUNCH_CHECK();                                                                    \
      return RTENHIP_OK;                                                                         \
    }                                                                                            \
    if (clips)                                                                                   \
      hipLaunchKernelGGL((expand_dw_kernel<C, SS, CP, PL, Q, true>), grid, dim3(256), lds, s, d);  \
    else                                                                                         \
      hipLaunchKernelGGL((expand_dw_kernel<C, SS, CP, PL, Q, false>), grid, dim3(256), lds, s, d); \
    RTENHIP_LAUNCH_CHECK();                                                                      \
    return RTENHIP_OK;                                                                           \
  }
  ED_PL(16, 2, 1028, 1)
  ED_PL(24, 1, 1028, 4)
  ED_PL(24, 2, 972, 1)
  ED_PL(32, 1, 860, 4)
  ED_PL(32, 2, 832, 1)
#undef ED_PL
#define ED_CASE(C, SS) \
  if (cin == C && S == SS) { \
    hipLaunchKernelGGL((expand_dw_kernel<C, SS, CP, 0, kEdMaxQ, false>), grid, dim3(256), lds, s, d); \
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
