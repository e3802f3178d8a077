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

typedef float dp_f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// One k-step of the depthwise -> projection chain for one lane: the depthwise
// outputs of channel c (taps wk[9], bias b0, then the activation) at pixels
// PX j .. PX j + PX - 1 of one row, from the 3 x (PX + 2) window at base
// (stride RS between the window's rows; rows whose ok flag is false and the
// columns outside [0, 16 PX) are skipped), each fed to MT MFMAs as the B
// operand of k-step rows 4 g + kq.
template <int PX, int MT>
__device__ __forceinline__ void dp_dw_mfma(const float* base, int RS, const float* wk, float b0, bool row_ok0,
                                           bool row_ok1, bool row_ok2, int j, int act_d, float lo_d, float hi_d,
                                           const float (&wa)[MT], dp_f32x4 (&acc)[PX][MT]) {
  // Window rows one at a time (ky outer, pixels inner: each output's taps are
  // still added in (ky, kx) order), 9 + PX values live instead of 3 (PX + 2).
  float v[PX];
#pragma unroll
  for (int p = 0; p < PX; p++) v[p] = b0;
#pragma unroll
  for (int ky = 0; ky < 3; ky++) {
    if (!(ky == 0 ? row_ok0 : (ky == 1 ? row_ok1 : row_ok2))) continue;
    float win[PX + 2];
#pragma unroll
    for (int x = 0; x < PX + 2; x++) win[x] = base[ky * RS + x];
    const float w0 = wk[3 * ky], w1 = wk[3 * ky + 1], w2 = wk[3 * ky + 2];
#pragma unroll
    for (int p = 0; p < PX; p++) {
      // column PX j + p - 1 + kx outside [0, W): only the row's ends
      if (!(p == 0 && j == 0)) v[p] = __fadd_rn(v[p], __fmul_rn(win[p], w0));
      v[p] = __fadd_rn(v[p], __fmul_rn(win[p + 1], w1));
      if (!(p == PX - 1 && j == 15)) v[p] = __fadd_rn(v[p], __fmul_rn(win[p + 2], w2));
    }
  }
#pragma unroll
  for (int p = 0; p < PX; p++) {
    if (act_d == RTENHIP_ACT_RELU) v[p] = rust_max(v[p], 0.f);
    else if (act_d == RTENHIP_ACT_CLIP) v[p] = rust_clamp(v[p], lo_d, hi_d);
  }
#pragma unroll
  for (int p = 0; p < PX; p++)
#pragma unroll
    for (int mt = 0; mt < MT; mt++)
      acc[p][mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[mt], v[p], acc[p][mt], 0, 0, 0);
}

// Projection epilogue of one row: acc[p][mt][r] is channel 16 mt + 4 kq + r,
// pixel PX j + p of the row at obase (+ channel * plane).  Residual loads are
// issued before the stores (vmcnt is in order).
template <int PX, int MT>
__device__ __forceinline__ void dp_store_row(const DwProjDesc& d, int64_t obase, int64_t plane, int kq,
                                             const dp_f32x4 (&acc)[PX][MT]) {
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

// dp_store_row through LDS: the row's 16 MT channels go out as whole 448-byte
// channel rows of 16-byte stores (dp_store_row's per-element stores scatter
// every instruction over four channel planes at a 28-byte lane stride).  Per
// chunk (mt, r) the lanes write channel 16 mt + 4 kq + r, pixels PX j .. into
// ex[kq][W] (this wave's 4 W floats of LDS), then read it back as float4s:
// float4 i = (slot i / (W / 4), pixel quad i % (W / 4)).  Same bias, residual
// and activation order as dp_store_row.  The bias comes from LDS (bpl[M]): a
// global load here would wait (vmcnt is in order) for the previous chunks'
// stores.
template <int PX, int MT>
__device__ __forceinline__ void dp_store_row_lds(const DwProjDesc& d, float* yrow, const float* rrow, int plane,
                                                 int j, int kq, int lane, float* ex, const float* bpl,
                                                 const dp_f32x4 (&acc)[PX][MT]) {
  constexpr int W = 16 * PX, NQ = W / 4, NU = (4 * NQ + 63) / 64;
  // All chunks through LDS into registers first, then every store: nothing
  // that waits on vmcnt (a residual load, a scratch reload) sits between
  // this row's stores.
  float4 ov[MT * 4][NU];
#pragma unroll
  for (int mt = 0; mt < MT; mt++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
#pragma unroll
      for (int p = 0; p < PX; p++) ex[kq * W + PX * j + p] = acc[p][mt][r];
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's writes before its reads
#pragma unroll
      for (int u = 0; u < NU; u++) {
        const int i = min(lane + 64 * u, 4 * NQ - 1);
        const int slot = i / NQ, q = i - slot * NQ;
        const int m = min(16 * mt + 4 * slot + r, 31);
        float4 o = *reinterpret_cast<const float4*>(ex + slot * W + 4 * q);
        if (d.bp) {
          const float bb = bpl[m];
          o.x = __fadd_rn(o.x, bb);
          o.y = __fadd_rn(o.y, bb);
          o.z = __fadd_rn(o.z, bb);
          o.w = __fadd_rn(o.w, bb);
        }
        if (rrow && 16 * mt + 4 * slot + r < d.M) {
          const float4 rv = *reinterpret_cast<const float4*>(rrow + (uint32_t)(m * plane + 4 * q));
          o.x = __fadd_rn(o.x, rv.x);
          o.y = __fadd_rn(o.y, rv.y);
          o.z = __fadd_rn(o.z, rv.z);
          o.w = __fadd_rn(o.w, rv.w);
        }
        if (d.act_p == RTENHIP_ACT_RELU) {
          o.x = rust_max(o.x, 0.f);
          o.y = rust_max(o.y, 0.f);
          o.z = rust_max(o.z, 0.f);
          o.w = rust_max(o.w, 0.f);
        } else if (d.act_p == RTENHIP_ACT_CLIP) {
          o.x = rust_clamp(o.x, d.lo_p, d.hi_p);
          o.y = rust_clamp(o.y, d.lo_p, d.hi_p);
          o.z = rust_clamp(o.z, d.lo_p, d.hi_p);
          o.w = rust_clamp(o.w, d.lo_p, d.hi_p);
        }
        ov[mt * 4 + r][u] = o;
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // reads done before the next chunk's writes
    }
#pragma unroll
  for (int mt = 0; mt < MT; mt++)
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
      for (int u = 0; u < NU; u++) {
        const int i = lane + 64 * u;
        const int slot = i / NQ, q = i - slot * NQ;
        const int m = 16 * mt + 4 * slot + r;
        if (i < 4 * NQ && m < d.M)
          *reinterpret_cast<float4*>(yrow + (uint32_t)(m * plane + 4 * q)) = ov[mt * 4 + r][u];
      }
}

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
    // Window: staged rows wave .. wave + 2 of channel kq, columns
    // PX j - 1 .. PX j + PX (LDS offset 4 + column).
    dp_dw_mfma<PX, MT>(xb + (g & 1) * BUF + (kq * kDpIn + wave) * RS + 3 + PX * j, RS, wdl + c * 9, bdl[c], row_ok0,
                       row_ok1, row_ok2, j, d.act_d, d.lo_d, d.hi_d, wa[g], acc);
    if (g + 1 < G) store_step((g + 1) & 1, pre[(g + 1) & 1]);
    __syncthreads();
  }

  if (oy >= H) return;
  const int64_t plane = (int64_t)H * W;
  dp_store_row<PX, MT>(d, (int64_t)img * d.M * plane + (int64_t)oy * W + PX * j, plane, kq, acc);
}


// ---------------------------------------------------------------------------
// MobileNetV2's stem (features.0: 3 -> 32 channels, 3x3 / 2, pads 1, + bias,
// act) feeding features.1 (the depthwise -> projection above) in one kernel:
// the stem's output (205 MB at batch 128, written by one kernel and read back
// by the next with a band halo) never leaves the CU.
//
// A persistent workgroup of 14 waves walks bands of 14 output rows (one per
// wave, as dw_project_kernel).  A band's 33 input rows (all 3 channels) are
// staged in LDS once, each row split into its odd and even columns so that a
// stride-2 output quad reads its window as conflict-free 16-byte words: for
// outputs 4q .. 4q + 3, tap kx = 1 is even[4q .. 4q + 3], kx = 2 odd[4q ..
// 4q + 3], kx = 0 (odd[4q - 1], odd[4q .. 4q + 2]); odd[-1] is a zero margin.
// Per k-step g (4 channels) waves 0..6 compute the stem outputs of channels
// 4g .. 4g + 3 on the band's 16 rows (14 + a halo row either side; 448 items
// of 4 pixels x 4 channels, weights as scalar operands) into one of two LDS
// tiles laid out as dw_project_kernel's staged rows, while every wave runs
// k-step g - 1's depthwise + projection from the other tile; one barrier per
// k-step.  The next band's input rows are loaded at k-step 6, right after the
// last stem step, and staged at k-step 7.
//
// Arithmetic: the stem is RTen's im2col GEMM (conv.rs:24-68 via
// VirtualIm2Col, gemm.rs:733-1050: K = 27 is one KC block) -- per output a
// fused multiply-add chain over k = (c, ky, kx) from +0 including the
// zero-padding positions, then + bias, then the activation -- exactly as
// conv_direct_lds_kernel computes it; the depthwise and the projection are
// dp_dw_mfma / dp_store_row, so the bits are the three operators'.
struct StemDwProjDesc {
  DwProjDesc p;      // the depthwise -> projection (p.x unused; C = 32, W = 112, H = stem rows)
  const float* img;  // [N, 3, H0, 224]
  const float* ws;   // [32, 3, 3, 3]
  const float* bs;   // [32] or null
  int H0, nbands;    // input rows; N * p.bands
  int act_s;
  float lo_s, hi_s;
  int dbg;  // timing experiments only (RTENHIP_SD_DBG): 1 skips the stem steps, 2 the depthwise steps,
            // 4 the output stores, 8 the next bands' input loads
};

constexpr int kSdRows = 14;              // output rows per band, one per wave
constexpr int kSdStem = kSdRows + 2;     // stem rows per band
constexpr int kSdIn = 2 * kSdStem + 1;   // input rows per band
constexpr int kSdLrow = 228;             // staged input row: [4 margin + 112 odd columns][112 even columns]
constexpr int kSdEven = 116;
constexpr int kSdRS = 120;               // stem-output row, as dw_project_kernel's staged rows
// Channel planes of a stem-output tile 48 floats apart mod 64 banks (16 rows
// x 120 would be 0 mod 64: the depthwise reads of lanes kq = 0..3 collide).
constexpr int kSdCS = kSdStem * kSdRS + 48;
constexpr int kSdBuf = 4 * kSdCS;
constexpr int kSdNT = 64 * kSdRows;
constexpr int kSdIn4 = 3 * kSdIn * 56;   // float4s of a band's input rows
constexpr int kSdPre = (kSdIn4 + kSdNT - 1) / kSdNT;
constexpr size_t kSdLdsBytes =
    (size_t)(3 * kSdIn * kSdLrow + 2 * kSdBuf + 32 * 9 + 32 + 8 * 2 * 64 + 32 * 36 + 32 + 32) * sizeof(float);
static_assert(kSdLdsBytes <= 160 * 1024, "one workgroup per CU");  // (163,504 bytes)
static_assert(kSdRows * 4 * 112 <= kSdBuf, "epilogue exchange fits one stem tile");
static_assert(kSdStem * 28 == 2 * 16 * kSdRows, "two 16-quad MFMA stem items per wave");

// The stem's activation (as the conv epilogues: Relu = max(x, 0), Clip = clamp).
__device__ __forceinline__ float sd_act(float x, int act, float lo, float hi) {
  if (act == RTENHIP_ACT_RELU) return rust_max(x, 0.f);
  if (act == RTENHIP_ACT_CLIP) return rust_clamp(x, lo, hi);
  return x;
}

template <int MT>
__global__ __launch_bounds__(kSdNT) void stem_dw_project_kernel(StemDwProjDesc s) {
  constexpr int G = 8, PX = 7, W = 112, C = 32;
  extern __shared__ float4 sd_lds4[];
  float* xin = reinterpret_cast<float*>(sd_lds4);  // [3][kSdIn][kSdLrow]
  float* sout = xin + 3 * kSdIn * kSdLrow;          // [2][4][kSdCS: kSdStem rows of kSdRS]
  float* wdl = sout + 2 * kSdBuf;                   // [C][9]
  float* bdl = wdl + C * 9;                         // [C]
  float* wpl = bdl + C;                             // [G][MT][64]
  float* wsl = wpl + G * 2 * 64;                    // stem weights [4g + ch][c][12]
  float* bsl = wsl + C * 36;                        // stem bias [C]
  float* bpl = bsl + C;                             // projection bias [32]
  const DwProjDesc& d = s.p;
  const int t = threadIdx.x;
  const int wave = t >> 6, lane = t & 63;
  const int j = lane & 15, kq = lane >> 4;
  const int H = d.H, H0 = s.H0;
  // The thread id as the lambdas' index math sees it: made opaque once per band
  // so that their per-thread offsets are formed in the band loop, not hoisted
  // out of it (and spilled) by the compiler.
  int tv = t;

  // A band's input rows 2 oy0 - 3 .. 2 oy0 + 29 (zero outside the image).
  auto load_in = [&](int band, dp_f32x4 (&pre)[kSdPre]) __attribute__((always_inline)) {
    const int img = band / d.bands, r0 = 2 * (band - img * d.bands) * kSdRows - 3;
    const float* base = s.img + (int64_t)img * 3 * H0 * (2 * W);
#pragma unroll
    for (int u = 0; u < kSdPre; u++) {
      const int e = tv + kSdNT * u;
      const int c = e / (kSdIn * 56), rem = e - c * (kSdIn * 56);
      const int r = rem / 56, q = rem - r * 56;
      const int iy = r0 + r;
      pre[u] = (dp_f32x4){0.f, 0.f, 0.f, 0.f};
      if (e < kSdIn4 && iy >= 0 && iy < H0)
        pre[u] = *reinterpret_cast<const dp_f32x4*>(base + ((int64_t)c * H0 + iy) * (2 * W) + 4 * q);
    }
  };
  // Input columns 4q .. 4q + 3: even columns 4q, 4q + 2 -> even[2q, 2q + 1],
  // odd columns 4q + 1, 4q + 3 -> odd[2q, 2q + 1].
  auto store_in = [&](const dp_f32x4 (&pre)[kSdPre]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < kSdPre; u++) {
      const int e = tv + kSdNT * u;
      if (e >= kSdIn4) continue;
      const int c = e / (kSdIn * 56), rem = e - c * (kSdIn * 56);
      const int r = rem / 56, q = rem - r * 56;
      float* row = xin + (c * kSdIn + r) * kSdLrow;
      *reinterpret_cast<float2*>(row + 4 + 2 * q) = make_float2(pre[u].y, pre[u].w);
      *reinterpret_cast<float2*>(row + kSdEven + 2 * q) = make_float2(pre[u].x, pre[u].z);
    }
  };
  // Stem outputs of channels 4g .. 4g + 3 on the band's rows oy0 - 1 ..
  // oy0 + 14 -> dst [4][kSdCS] (rows of kSdRS, column offset 4), on MFMA:
  // v_mfma_f32_4x4x1_16b_f32 (16 blocks of 4 x 4 x 1; a chain of them is
  // bitwise the k-ordered fmaf chain, tools/probes/mfma4x4_probe.hip) with the
  // block's rows the 4 channels and its columns the 4 pixels of a quad: lane l
  // supplies A = W[4g + l % 4][k] and B = x(k) at pixel 4 q + l % 4 of quad
  // (row, q) = block l / 4 of the item, and holds D for channel r in register
  // r.  The band's 16 x 28 quads are 28 items of 16 quads, two per wave.  Rows
  // outside the image are computed from the zero rows (the depthwise skips
  // them).
  auto stem_step = [&](int g, int oy0, float* dst) __attribute__((always_inline)) {
    if (s.dbg & 1) return;
    (void)oy0;
    const int l = tv & 63, w = tv >> 6;
    const int ch = l & 3;
    int px[2], rowoff[2], sro[2];
#pragma unroll
    for (int it = 0; it < 2; it++) {
      const int f = 16 * (w + kSdRows * it) + (l >> 2);
      const int sr = f / 28, q = f - 28 * sr;
      px[it] = 4 * q + (l & 3);
      rowoff[it] = 2 * sr * kSdLrow;
      sro[it] = sr * kSdRS;
    }
    dp_f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    // (c not unrolled: the scheduler would hoist every window's LDS reads)
#pragma unroll 1
    for (int c = 0; c < 3; c++) {
      float wk[12];  // W[4g + ch][9c .. 9c + 8] (+3 pad)
#pragma unroll
      for (int i = 0; i < 3; i++) {
        const float4 q4 = *reinterpret_cast<const float4*>(wsl + ((g * 4 + ch) * 3 + c) * 12 + 4 * i);
        wk[4 * i] = q4.x;
        wk[4 * i + 1] = q4.y;
        wk[4 * i + 2] = q4.z;
        wk[4 * i + 3] = q4.w;
      }
#pragma unroll
      for (int ky = 0; ky < 3; ky++) {
        float x[2][3];
#pragma unroll
        for (int it = 0; it < 2; it++) {
          const float* row = xin + (c * kSdIn + ky) * kSdLrow + rowoff[it];
          x[it][0] = row[3 + px[it]];          // input column 2 px - 1: odd[px - 1]
          x[it][1] = row[kSdEven + px[it]];    // 2 px: even[px]
          x[it][2] = row[4 + px[it]];          // 2 px + 1: odd[px]
        }
#pragma unroll
        for (int kx = 0; kx < 3; kx++)
#pragma unroll
          for (int it = 0; it < 2; it++)
            acc[it] = __builtin_amdgcn_mfma_f32_4x4x1f32(wk[3 * ky + kx], x[it][kx], acc[it], 0, 0, 0);
      }
    }
#pragma unroll
    for (int it = 0; it < 2; it++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        float v = acc[it][r];
        if (s.bs) v = __fadd_rn(v, bsl[4 * g + r]);
        dst[r * kSdCS + sro[it] + 4 + px[it]] = sd_act(v, s.act_s, s.lo_s, s.hi_s);
      }
  };

  // Prologue: the stem / depthwise / projection weights and biases into LDS
  // (the stem's and the biases there because a global load inside the band
  // loop would wait -- vmcnt is in order -- for every store and prefetch load
  // issued before it; the projection's A operands W[16 mt + j][4 g + kq], 0
  // past M, as wpl[g][mt][lane]) and the first band's input rows: every load
  // issued before any LDS store, one memory round trip for all of them.
  constexpr int NWS = C * 36, NWD = C * 9, NWP = G * MT * 64;
  constexpr int NST = NWS + NWD + 3 * C + NWP;
  constexpr int NSU = (NST + kSdNT - 1) / kSdNT;
  float sv[NSU];
  float* sdst[NSU];
#pragma unroll
  for (int u = 0; u < NSU; u++) {
    int e = t + kSdNT * u;
    sv[u] = 0.f;
    sdst[u] = nullptr;
    if (e < NWS) {  // [4g + ch][c][12]: k = 9c + i12 for i12 < 9
      const int i12 = e % 12, c = (e / 12) % 3, oc = e / 36;
      if (i12 < 9) sv[u] = s.ws[oc * 27 + c * 9 + i12];
      sdst[u] = wsl + e;
    } else if ((e -= NWS) < NWD) {
      sv[u] = d.wd[e];
      sdst[u] = wdl + e;
    } else if ((e -= NWD) < C) {
      if (d.bd) sv[u] = d.bd[e];
      sdst[u] = bdl + e;
    } else if ((e -= C) < C) {
      if (s.bs) sv[u] = s.bs[e];
      sdst[u] = bsl + e;
    } else if ((e -= C) < C) {
      if (d.bp && e < d.M) sv[u] = d.bp[e];
      sdst[u] = bpl + e;
    } else if ((e -= C) < NWP) {
      const int l = e & 63, mt = (e >> 6) % MT, g = (e >> 6) / MT;
      const int m = 16 * mt + (l & 15);
      if (m < d.M) sv[u] = d.wp[(int64_t)m * C + 4 * g + (l >> 4)];
      sdst[u] = wpl + e;
    }
  }
  dp_f32x4 pre[kSdPre];
  int band = blockIdx.x;
  if (band < s.nbands) load_in(band, pre);
#pragma unroll
  for (int u = 0; u < NSU; u++)
    if (sdst[u]) *sdst[u] = sv[u];
  for (int i = t; i < 3 * kSdIn; i += kSdNT) *reinterpret_cast<float4*>(xin + i * kSdLrow) = make_float4(0.f, 0.f, 0.f, 0.f);
  if (band < s.nbands) store_in(pre);
  __syncthreads();
  const int64_t plane = (int64_t)H * W;
  for (; band < s.nbands; band += gridDim.x) {
    asm volatile("" : "+v"(tv));
    const int img = band / d.bands, oy0 = (band - img * d.bands) * kSdRows;
    const int next = band + (int)gridDim.x;
    const int oy = oy0 + wave;
    const bool row_ok0 = oy - 1 >= 0 && oy - 1 < H, row_ok1 = oy < H, row_ok2 = oy + 1 < H;
    stem_step(0, oy0, sout);
    __syncthreads();
    dp_f32x4 acc[PX][MT];
#pragma unroll
    for (int p = 0; p < PX; p++)
#pragma unroll
      for (int mt = 0; mt < MT; mt++) acc[p][mt] = (dp_f32x4){0.f, 0.f, 0.f, 0.f};
    // (two k-steps per unrolled body: the tile parity stays static)
#pragma unroll 2
    for (int g = 0; g < G; g++) {
      if (g + 1 < G) stem_step(g + 1, oy0, sout + ((g + 1) & 1) * kSdBuf);
      // (after the last stem step: the prefetch registers are never live across one)
      if (g == G - 2 && next < s.nbands && !(s.dbg & 8)) load_in(next, pre);
      const int c = 4 * g + kq;
      float wa[MT];
#pragma unroll
      for (int mt = 0; mt < MT; mt++) wa[mt] = wpl[(g * MT + mt) * 64 + lane];
      if (!(s.dbg & 2))
      dp_dw_mfma<PX, MT>(sout + (g & 1) * kSdBuf + kq * kSdCS + wave * kSdRS + 3 + PX * j, kSdRS, wdl + c * 9,
                         bdl[c], row_ok0, row_ok1, row_ok2, j, d.act_d, d.lo_d, d.hi_d, wa, acc);
      if (g == G - 1 && next < s.nbands && !(s.dbg & 8)) store_in(pre);
      __syncthreads();
    }
    // (through this wave's 4 W floats of the second stem tile: free until the
    // next band's first barrier, which every wave passes after its stores)
    if (oy < H && !(s.dbg & 4)) {
      // (the lane id made opaque here: the epilogue's per-lane addresses are
      // formed here instead of being hoisted out of the band loop and spilled
      // -- a scratch reload between the chunks' stores waits for all of them)
      int le = lane;
      asm volatile("" : "+v"(le));
      const int64_t rb = (int64_t)img * d.M * plane + (int64_t)oy * W;  // wave-uniform
      dp_store_row_lds<PX, MT>(d, d.y + rb, d.res ? d.res + rb : nullptr, (int)plane, le & 15, le >> 4, le,
                               sout + kSdBuf + wave * 4 * W, bpl, acc);
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

bool stem_dw_project_eligible(int C0, int H0, int W0, int kh, int kw, int sh, int sw, int pt, int pl, int O, int OH,
                              int OW) {
  return C0 == 3 && W0 == 224 && H0 >= 1 && kh == 3 && kw == 3 && sh == 2 && sw == 2 && pt == 1 && pl == 1 && O == 32 &&
         OW == 112 && OH == (H0 - 1) / 2 + 1;
}

rtenhip_status launch_stem_dw_project(const float* img, const float* ws, const float* bs, int act_s, float lo_s,
                                      float hi_s, int H0, const float* wd, const float* bd, int act_d, float lo_d,
                                      float hi_d, const float* wp, const float* bp, const float* res, int act_p,
                                      float lo_p, float hi_p, float* y, int N, int H, int M, hipStream_t s) {
  if (!stem_dw_project_eligible(3, H0, 224, 3, 3, 2, 2, 1, 1, 32, H, 112) || M < 1 || M > 32 ||
      ((uintptr_t)img % 16))
    return fail(RTENHIP_UNSUPPORTED_VALUE, "stem+depthwise+projection: unsupported shape");
  if (N == 0) return RTENHIP_OK;
  StemDwProjDesc d{};
  d.p.wd = wd;
  d.p.bd = bd;
  d.p.wp = wp;
  d.p.bp = bp;
  d.p.res = res;
  d.p.y = y;
  d.p.C = 32;
  d.p.M = M;
  d.p.H = H;
  d.p.W = 112;
  d.p.bands = (H + kSdRows - 1) / kSdRows;
  d.p.act_d = act_d;
  d.p.act_p = act_p;
  d.p.lo_d = lo_d;
  d.p.hi_d = hi_d;
  d.p.lo_p = lo_p;
  d.p.hi_p = hi_p;
  d.img = img;
  d.ws = ws;
  d.bs = bs;
  d.H0 = H0;
  d.act_s = act_s;
  static const int sd_dbg = getenv("RTENHIP_SD_DBG") ? atoi(getenv("RTENHIP_SD_DBG")) : 0;
  d.dbg = sd_dbg;
  d.lo_s = lo_s;
  d.hi_s = hi_s;
  const int64_t nb = (int64_t)N * d.p.bands;
  if (nb > 0x7fffffff) return fail(RTENHIP_UNSUPPORTED_VALUE, "stem+depthwise+projection: grid too large");
  d.nbands = (int)nb;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  const dim3 grid((unsigned)std::min<int64_t>(nb, cus)), blk(kSdNT);
#define SD_LAUNCH(MT)                                                                                           \
  {                                                                                                             \
    static const bool attr = hipFuncSetAttribute((const void*)stem_dw_project_kernel<MT>,                       \
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSdLdsBytes) == \
                             hipSuccess;                                                                        \
    (void)attr;                                                                                                 \
    hipLaunchKernelGGL((stem_dw_project_kernel<MT>), grid, blk, kSdLdsBytes, s, d);                           \
  }
  if (M <= 16) SD_LAUNCH(1) else SD_LAUNCH(2)
#undef SD_LAUNCH
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

}  // namespace rtenhip
