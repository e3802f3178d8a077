// Depthwise 3x3 (+bias, act) -> pointwise 1x1 projection (+bias, residual,
// act) as one kernel: MobileNetV2's first bottleneck (features.1: 32 channels,
// 112 x 112, projected to 16), whose depthwise output otherwise makes a round
// trip through HBM (written by the depthwise kernel, read back by the
// projection: 2 x 205 MB at batch 128).
//
// A workgroup (8 waves) owns one image and 8 output rows, one per wave.  The
// projection is a v_mfma_f32_16x16x4_f32 chain over the channels, k-steps of 4
// channels; lane l = 16 kq + j supplies channel 4 g + kq of pixel group j in
// k-step g.  Its B operands are the depthwise outputs themselves: the lane
// computes channel 4 g + kq of pixels PX j .. PX j + PX - 1 (PX = W / 16) from
// a 3 x (PX + 2) window in LDS, and feeds them to PX MFMAs (tile p holds
// pixels PX j + p, so each tile is 16 pixels x 16 channels).  The input rows
// of k-step g + 2's four channels are loaded while k-step g computes, and
// g + 1's stored to LDS after it (two LDS buffers of 4 channels x ROWS + 2
// rows).
//
// Arithmetic (bit-identical to the two operators apart):
// - depthwise (conv_2d_depthwise_block, src/ops/conv/depthwise.rs:49-203, as
//   depthwise_lds_kernel states it): per output the bias, then + v * w over
//   the taps in (ky, kx) order, each product and sum rounded, taps outside the
//   image skipped (not added as zeros), then the activation;
// - projection (conv_2d_pointwise, src/ops/conv.rs:24-68; the GEMM's
//   summation, src/gemm.rs:733-1050): K = C <= 256 is one KC block, a fused
//   multiply-add chain over k in order from +0 (v_mfma_f32_16x16x4_f32 being
//   bitwise that chain), then + bias, then + the residual (a fused Add), then
//   the activation.
#include <algorithm>

#include "common.h"
#include "ctx.h"
#include "vecmath.h"

namespace rtenhip {

namespace {

typedef float dp_f32x4 __attribute__((ext_vector_type(4)));

struct DwProjDesc {
  const float* x;     // [N, C, H, W]
  const float* wd;    // [C, 1, 3, 3]
  const float* bd;    // [C] or null
  const float* wp;    // [M, C]
  const float* bp;    // [M] or null
  const float* res;   // [N, M, H, W] or null
  float* y;           // [N, M, H, W]
  int C, M, H, W;
  int bands;          // ceil(H / rows per workgroup)
  int act_d, act_p;
  float lo_d, hi_d, lo_p, hi_p;
};

// Output rows per workgroup (one per wave): 8 measured 1-2% faster than 4
// (profiles/r5_dw_project.txt).
constexpr int kDpRowsHost = 8;

template <int G, int MT, int PX, int ROWS>  // ROWS output rows per workgroup, one per wave
__global__ __launch_bounds__(64 * ROWS) void dw_project_kernel(DwProjDesc d) {
  constexpr int kDpRows = ROWS, kDpIn = ROWS + 2, NTH = 64 * ROWS;
  constexpr int W = 16 * PX;
  constexpr int RS = W + 8;           // staged row: 4 floats of margin either side
  constexpr int NQ = W / 4;           // float4s per row
  constexpr int NV = 4 * kDpIn * NQ;  // float4s per k-step's staged rows
  constexpr int NIT = (NV + NTH - 1) / NTH;
  constexpr int BUF = 4 * kDpIn * RS;
  constexpr int C = 4 * G;
  extern __shared__ float4 dp_lds4[];
  float* xb = reinterpret_cast<float*>(dp_lds4);  // [2][4][kDpIn][RS]
  float* wdl = xb + 2 * BUF;                      // [C][9]
  float* bdl = wdl + C * 9;                       // [C]
  float* dummy = bdl + C;                         // one float4 (16-byte aligned: C % 4 == 0)
  const int t = threadIdx.x;
  const int wave = t >> 6, lane = t & 63;
  const int j = lane & 15, kq = lane >> 4;
  const int img = (int)blockIdx.x / d.bands;
  const int oy0 = ((int)blockIdx.x - img * d.bands) * kDpRows;
  const int H = d.H;
  const float* ximg = d.x + (int64_t)img * C * H * W;

  // k-step g's four channels, input rows oy0 - 1 .. oy0 + 4 (clamped: rows
  // outside the image are never used, their taps are skipped).  The staging
  // array is an array of clang vectors passed by reference: one of HIP's
  // float4 class, or one captured by the lambda, stayed in scratch.
  auto load_step = [&](int g, dp_f32x4 (&pre)[NIT]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NIT; u++) {
      const int e = min(t + NTH * u, NV - 1);
      const int cc = e / (kDpIn * NQ), rem = e - cc * (kDpIn * NQ);
      const int r = rem / NQ, q = rem - r * NQ;
      const int iy = min(max(oy0 - 1 + r, 0), H - 1);
      pre[u] = *reinterpret_cast<const dp_f32x4*>(ximg + ((int64_t)(4 * g + cc) * H + iy) * W + 4 * q);
    }
  };
  // Unconditional stores, the slots past NV into a dummy float4.
  auto store_step = [&](int buf, const dp_f32x4 (&pre)[NIT]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NIT; u++) {
      const int e = t + NTH * u;
      const int cc = e / (kDpIn * NQ), rem = e - cc * (kDpIn * NQ);
      const int r = rem / NQ, q = rem - r * NQ;
      float* dst = e < NV ? xb + buf * BUF + (cc * kDpIn + r) * RS + 4 + 4 * q : dummy;
      *reinterpret_cast<dp_f32x4*>(dst) = pre[u];
    }
  };

  // Two k-steps in flight: step g + 2's rows are loaded while step g
  // computes, step g + 1's (loaded a step earlier) stored after it.
  dp_f32x4 pre[2][NIT];
  load_step(0, pre[0]);
  if (G > 1) load_step(1, pre[1]);
  for (int i = t; i < C * 9; i += NTH) wdl[i] = d.wd[i];
  for (int i = t; i < C; i += NTH) bdl[i] = d.bd ? d.bd[i] : 0.f;
  // The projection's A operands: W[16 mt + j][4 g + kq] (0 past M).
  float wa[G][MT];
#pragma unroll
  for (int g = 0; g < G; g++)
#pragma unroll
    for (int mt = 0; mt < MT; mt++) {
      const int m = 16 * mt + j;
      wa[g][mt] = m < d.M ? d.wp[(int64_t)m * C + 4 * g + kq] : 0.f;
    }
  store_step(0, pre[0]);
  __syncthreads();

  const int oy = oy0 + wave;
  // Rows of the window (oy - 1 + ky) inside the image: wave-uniform.
  const bool row_ok0 = oy - 1 >= 0 && oy - 1 < H, row_ok1 = oy < H, row_ok2 = oy + 1 < H;
  dp_f32x4 acc[PX][MT];
#pragma unroll
  for (int p = 0; p < PX; p++)
#pragma unroll
    for (int mt = 0; mt < MT; mt++) acc[p][mt] = (dp_f32x4){0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int g = 0; g < G; g++) {
    if (g + 2 < G) load_step(g + 2, pre[g & 1]);
    const int c = 4 * g + kq;
    const float* wk = wdl + c * 9;
    float wv[9];
#pragma unroll
    for (int i = 0; i < 9; i++) wv[i] = wk[i];
    const float b0 = bdl[c];
    // Window: staged rows wave .. wave + 2 of channel kq, columns
    // PX j - 1 .. PX j + PX (LDS offset 4 + column).
    const float* base = xb + (g & 1) * BUF + (kq * kDpIn + wave) * RS + 3 + PX * j;
    float win[3][PX + 2];
#pragma unroll
    for (int ky = 0; ky < 3; ky++)
#pragma unroll
      for (int x = 0; x < PX + 2; x++) win[ky][x] = base[ky * RS + x];
    float v[PX];
#pragma unroll
    for (int p = 0; p < PX; p++) {
      float a = b0;
#pragma unroll
      for (int ky = 0; ky < 3; ky++) {
        if (!(ky == 0 ? row_ok0 : (ky == 1 ? row_ok1 : row_ok2))) continue;
#pragma unroll
        for (int kx = 0; kx < 3; kx++) {
          // column PX j + p - 1 + kx outside [0, W): only the row's ends
          const bool col_ok = !((p == 0 && kx == 0 && j == 0) || (p == PX - 1 && kx == 2 && j == 15));
          if (col_ok) a = __fadd_rn(a, __fmul_rn(win[ky][p + kx], wv[ky * 3 + kx]));
        }
      }
      if (d.act_d == RTENHIP_ACT_RELU) a = rust_max(a, 0.f);
      else if (d.act_d == RTENHIP_ACT_CLIP) a = rust_clamp(a, d.lo_d, d.hi_d);
      v[p] = a;
    }
#pragma unroll
    for (int p = 0; p < PX; p++)
#pragma unroll
      for (int mt = 0; mt < MT; mt++)
        acc[p][mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[g][mt], v[p], acc[p][mt], 0, 0, 0);
    if (g + 1 < G) store_step((g + 1) & 1, pre[(g + 1) & 1]);
    __syncthreads();
  }

  // Epilogue: acc[p][mt][r] is channel 16 mt + 4 kq + r, pixel PX j + p of row
  // oy.  Residual loads are issued before the stores (vmcnt is in order).
  if (oy >= H) return;
  const int64_t plane = (int64_t)H * W;
  const int64_t obase = (int64_t)img * d.M * plane + (int64_t)oy * W + PX * j;
  float rv[MT][4][PX];
#pragma unroll
  for (int mt = 0; mt < MT; mt++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int m = min(16 * mt + 4 * kq + r, d.M - 1);
#pragma unroll
      for (int p = 0; p < PX; p++) rv[mt][r][p] = d.res ? d.res[obase + m * plane + p] : 0.f;
    }
#pragma unroll
  for (int mt = 0; mt < MT; mt++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int m = 16 * mt + 4 * kq + r;
      if (m >= d.M) continue;
      const float bb = d.bp ? d.bp[m] : 0.f;
#pragma unroll
      for (int p = 0; p < PX; p++) {
        float o = acc[p][mt][r];
        if (d.bp) o = __fadd_rn(o, bb);
        if (d.res) o = __fadd_rn(o, rv[mt][r][p]);
        if (d.act_p == RTENHIP_ACT_RELU) o = rust_max(o, 0.f);
        else if (d.act_p == RTENHIP_ACT_CLIP) o = rust_clamp(o, d.lo_p, d.hi_p);
        d.y[obase + m * plane + p] = o;
      }
    }
}

}  // namespace

bool dw_project_eligible(int C, int H, int W, int M, int S, int pt, int pl, int pb, int pr) {
  return C == 32 && W == 112 && H >= 1 && M >= 1 && M <= 32 && S == 1 && pt == 1 && pl == 1 && pb == 1 && pr == 1;
}

rtenhip_status launch_dw_project(const float* x, const float* wd, const float* bd, int act_d, float lo_d,
                                 float hi_d, const float* wp, const float* bp, const float* res, int act_p,
                                 float lo_p, float hi_p, float* y, int N, int C, int H, int W, int M,
                                 hipStream_t s) {
  if (!dw_project_eligible(C, H, W, M, 1, 1, 1, 1, 1) || ((uintptr_t)x % 16))
    return fail(RTENHIP_UNSUPPORTED_VALUE, "depthwise+projection: unsupported shape");
  if (N == 0) return RTENHIP_OK;
  DwProjDesc d{};
  d.x = x;
  d.wd = wd;
  d.bd = bd;
  d.wp = wp;
  d.bp = bp;
  d.res = res;
  d.y = y;
  d.C = C;
  d.M = M;
  d.H = H;
  d.W = W;
  constexpr int R = kDpRowsHost;
  d.bands = (H + R - 1) / R;
  d.act_d = act_d;
  d.act_p = act_p;
  d.lo_d = lo_d;
  d.hi_d = hi_d;
  d.lo_p = lo_p;
  d.hi_p = hi_p;
  constexpr int PX = 7, G = 8;
  const size_t lds = (size_t)(2 * 4 * (R + 2) * (16 * PX + 8) + C * 9 + C + 4) * sizeof(float);
  const int64_t blocks = (int64_t)N * d.bands;
  if (blocks > 0x7fffffff) return fail(RTENHIP_UNSUPPORTED_VALUE, "depthwise+projection: grid too large");
  const dim3 grid((unsigned)blocks), blk(64 * R);
  if (M <= 16) hipLaunchKernelGGL((dw_project_kernel<G, 1, PX, R>), grid, blk, lds, s, d);
  else hipLaunchKernelGGL((dw_project_kernel<G, 2, PX, R>), grid, blk, lds, s, d);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

}  // namespace rtenhip
