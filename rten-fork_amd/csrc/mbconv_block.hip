// MobileNetV2 inverted residual block in one kernel: 1x1 expand (+ bias,
// Clip) -> 3x3 depthwise (+ bias, Clip) -> 1x1 project (+ bias) [+ the
// block's residual Add], with neither the expanded nor the depthwise
// activation ever written to HBM.  At batch 128 those two intermediates are
// ~5.5 GB of the ~5.8 GB a MobileNetV2 step moves when the three convs run
// apart.
//
// Arithmetic is exactly that of the three operators run apart (bit-identical
// to the unfused graph and to RTen):
//  - expand, conv_2d_pointwise (src/ops/conv.rs:24-68, K = C_in < 256: one
//    KC block): the k-ordered fma chain from +0 (kernels.rs:206-316) as
//    v_mfma_f32_16x16x4f32 steps (bitwise that chain), then + bias
//    (gemm.rs:1034-1047), then the fused Clip / Relu;
//  - depthwise, conv_2d_depthwise_block (src/ops/conv/depthwise.rs:49-120):
//    bias, then + v * w per tap in ky, kx order with separate roundings,
//    skipping rows outside the image and columns outside the reference's
//    min_max_out_x_coords range, then Clip / Relu;
//  - project, conv_2d_pointwise with K = hidden: one fma chain per KC = 256
//    block from +0 (MFMA steps again), block 0 + bias, later blocks added in
//    K order (gemm.rs:733-1050), then the residual Add and the activation.
//
// Mapping: a workgroup owns one image and a band of TR output rows, all
// output channels.  The band's input rows (clipped to the image) are staged
// in LDS once as X[c][pixel].  The hidden channels are walked in chunks of
// 16 (one MFMA tile of rows):
//  1. expand: the chunk's 16 channels at every band input pixel, 16x16
//     MFMA tiles (16 channels x 16 pixels) split over the waves, into the
//     LDS plane set E[chunk % 2][16][pixel] (double-buffered: one barrier per
//     chunk);
//  2. depthwise + project: wave w owns output pixel tiles w, w + NW, ...;
//     lane (c, h) forms the depthwise outputs of channels h, h + 4, h + 8,
//     h + 12 at pixel c of the tile -- exactly the project MFMA's B operand
//     for k = 4s + h, s = 0..3 -- and feeds them straight into the project
//     accumulators (all output channels of that tile).  The depthwise values
//     never leave registers.
// Weights are repacked once per plan (pack_mbconv_block) into the lanes'
// operand order: one float4 load per lane per MFMA group.
#include <cstdlib>
#include <cstring>
#include <vector>

#include "common.h"
#include "stage.h"
#include "vecmath.h"

// Timing experiments only (never set in a product build): 1 = no depthwise /
// project phase, 2 = no expand MFMAs, 3 = no weight prefetch loads, 4 = no
// project MFMAs.
#ifndef RTENHIP_MB_EXPERIMENT
#define RTENHIP_MB_EXPERIMENT 0
#endif

namespace rtenhip {

typedef float mb_f32x4 __attribute__((ext_vector_type(4)));

struct MbBlockDesc {
  const float* x;    // [N, CIN, H, W]
  const float* pk;   // packed weights (mbconv_block_pack_floats)
  const float* res;  // residual [N, COUT, OH, OW] (null: none); res_lds: it is x (read from the staged band)
  float* y;          // [N, COUT, OH, OW]
  int hid, cout, H, W, OH, OW, pt, pl;
  int TR;            // output rows per band
  int RX, RE;        // LDS row strides (floats) of X and E
  int res_lds;
  int act_e, act_d, act_p;
  float lo_e, hi_e, lo_d, hi_d, lo_p, hi_p;
  int omin[3], omax[3];  // min_max_out_x_coords per kx (depthwise.rs:24-38)
  int has_be, has_bd, has_bp;
};

// Packed record sizes (floats).  Per 16-channel chunk: expand A operand
// [GE][64 lanes][4], expand bias [4 h][4], depthwise [4 h][9 taps][4],
// depthwise bias [4 h][4], project A operand [MT][64][4]; then the project
// bias [MT][4 h][4].
__host__ __device__ inline int mb_ge(int cin) { return (cin + 15) / 16; }
// Every LDS plane row (X and E) starts with MB_ZS floats: slots 0..8 hold
// copysign(0, -w) of the row channel's 9 depthwise taps, so a tap the
// reference skips reads its slot and adds w * slot = -0 (x + (-0) == x for
// every x): no select per tap.  Needs finite depthwise weights (checked when
// the plan fuses the block).  Pixel p of a row is at MB_ZS + p.
constexpr int MB_ZS = 16;
__host__ __device__ inline int mb_chunk_floats(int cin, int mt) { return mb_ge(cin) * 256 + 16 + 144 + 16 + mt * 256; }

__device__ __forceinline__ float mb_act(float v, int act, float lo, float hi) {
  if (act == RTENHIP_ACT_RELU) return rust_max(v, 0.f);
  if (act == RTENHIP_ACT_CLIP) return rust_clamp(v, lo, hi);
  return v;
}

// NT threads; S stride; CIN input channels; MT = ceil(COUT / 16) project
// row tiles; MAXT = output pixel tiles per wave (host-checked).  EXP false:
// a block without the expand conv (MobileNetV2's features.1, depthwise ->
// project): the depthwise reads the staged band itself (hidden = CIN), no
// per-chunk planes or barriers.
template <int NT, int S, int CIN, int MT, int MAXT, bool EXP = true>
__global__ __launch_bounds__(NT, 2) void mbconv_block_kernel(MbBlockDesc d) {
  constexpr int NW = NT / 64;
  constexpr int KS = CIN / 4;  // expand MFMA steps
  constexpr int GE = EXP ? (CIN + 15) / 16 : 0;
  extern __shared__ float4 mb_lds4[];
  float* X = reinterpret_cast<float*>(mb_lds4);  // [CIN][RX]
  float* E = X + CIN * d.RX;                      // [2][16][RE] (EXP)
  // Weight records of three chunks (ch % 3): the record of chunk ch + 2 is
  // loaded while chunk ch runs and stored after its barrier, so no chunk
  // waits on a global load for its operands.
  float4* Wr = reinterpret_cast<float4*>(EXP ? E + 2 * 16 * d.RE : E);
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int c = lane & 15, h = lane >> 4;
  const int n = blockIdx.y;
  const int oy0 = blockIdx.x * d.TR;
  const int orows = min(d.TR, d.OH - oy0);
  const int ia = max(0, oy0 * S - d.pt);
  const int ib = min(d.H, (oy0 + orows - 1) * S - d.pt + 3);  // input rows [ia, ib) of the band
  const int W = d.W, OW = d.OW;
  const int pin = (ib - ia) * W, pout = orows * OW;
  const int tin = (pin + 15) >> 4, tout = (pout + 15) >> 4;
  const int64_t HW = (int64_t)d.H * W;

  // Stage the band: X[ci][(iy - ia) * W + ix] = x[n][ci][iy][ix].
  {
    const float* xb = d.x + (int64_t)n * CIN * HW + (int64_t)ia * W;
    const int total = CIN * pin;
    if ((pin & 3) == 0 && (HW & 3) == 0 && ((uintptr_t)xb & 15) == 0 && (d.RX & 3) == 0) {
      const int q = pin >> 2;
      stage_batched<8, float4>(
          total >> 2, [&](int e) { const int ci = e / q; return *reinterpret_cast<const float4*>(xb + ci * HW + 4 * (e - ci * q)); },
          [&](int e, const float4& v) { const int ci = e / q; *reinterpret_cast<float4*>(X + ci * d.RX + MB_ZS + 4 * (e - ci * q)) = v; });
    } else {
      stage_batched<8, float>(
          total, [&](int e) { const int ci = e / pin; return xb[ci * HW + (e - ci * pin)]; },
          [&](int e, float v) { const int ci = e / pin; X[ci * d.RX + MB_ZS + (e - ci * pin)] = v; });
    }
  }

  // This lane's output pixels (column c of each owned tile): the depthwise
  // tap base (E offset of tap (0, 0)) and the 9-bit tap mask.
  int tidx[MAXT][9];  // plane-row offset read for tap k: the pixel, or slot k when skipped
#pragma unroll
  for (int u = 0; u < MAXT; u++) {
    const int tile = wave + u * NW;
    const int o = tile * 16 + c;
    const int ol = min(o, pout - 1) / OW, ox = min(o, pout - 1) - (min(o, pout - 1) / OW) * OW;
    const int oy = oy0 + ol;
    const int base = MB_ZS + (oy * S - d.pt - ia) * W + ox * S - d.pl;
#pragma unroll
    for (int ky = 0; ky < 3; ky++) {
      const int r = oy * S + ky - d.pt;
      const bool row_ok = r >= 0 && r < d.H;
#pragma unroll
      for (int kx = 0; kx < 3; kx++) {
        const bool on = tile < tout && o < pout && row_ok && ox >= d.omin[kx] && ox < d.omax[kx];
        tidx[u][ky * 3 + kx] = on ? base + ky * W + kx : ky * 3 + kx;
      }
    }
  }

  const int nchunks = d.hid >> 4;
  const int cf = mb_chunk_floats(EXP ? CIN : 0, MT);
  const int cf4 = cf >> 2;  // float4s per record (<= 2 * NT, host-checked)
  const float4* pk4 = reinterpret_cast<const float4*>(d.pk);
  // Records 0 and 1 staged with the band.
  for (int i = t; i < min(2, nchunks) * cf4; i += NT) Wr[i] = pk4[i];
  // Project accumulators (current KC block) and the folded sum.
  mb_f32x4 acc[MAXT][MT], sum[MAXT][MT];
#pragma unroll
  for (int u = 0; u < MAXT; u++)
#pragma unroll
    for (int m = 0; m < MT; m++) acc[u][m] = sum[u][m] = (mb_f32x4){0.f, 0.f, 0.f, 0.f};
  bool folded = false;  // block 0 folded into sum (with the project bias)
  const float4* bp4 = pk4 + (int64_t)nchunks * (cf >> 2);  // [MT][4][4]

  __syncthreads();  // X staged

  // Record prefetch: chunk ch loads record ch + 2 into registers and stores
  // the one it loaded a chunk earlier (record ch + 1) into its slot during
  // its expand phase, so a load has a whole chunk of work to land.  Slot
  // (ch + 1) % 3 last held record ch - 2, read before barrier ch - 1; the
  // stores are visible to expand ch + 1 after barrier ch.
  float4 held[2] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
  bool held_ok = false;  // record 1 was staged with the band
  for (int ch = 0; ch < nchunks; ch++) {
    const float4* rec = Wr + (ch % 3) * cf4;
    float4 nxt[2];
    const bool pf = ch + 2 < nchunks && RTENHIP_MB_EXPERIMENT != 3;
    {
      const float4* src = pk4 + (int64_t)(ch + 2) * cf4;
#pragma unroll
      for (int u = 0; u < 2; u++) nxt[u] = pf ? src[min(t + u * NT, cf4 - 1)] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (held_ok) {
      float4* dst = Wr + ((ch + 1) % 3) * cf4;
#pragma unroll
      for (int u = 0; u < 2; u++)
        if (t + u * NT < cf4) dst[t + u * NT] = held[u];
    }
    // The chunk's 16 depthwise input planes: expand planes, or the band.
    float* Eb = EXP ? E + (ch & 1) * 16 * d.RE : X + ch * 16 * d.RX;
    const int re = EXP ? d.RE : d.RX;
    // 1. Expand: tiles of 16 channels x 16 band pixels, wave-strided.
    if constexpr (EXP) {
      float4 wa[GE];
#pragma unroll
      for (int g = 0; g < GE; g++) wa[g] = rec[g * 64 + lane];
      const float4 be = rec[GE * 64 + h];
      for (int tile = wave; tile < tin; tile += NW) {
        mb_f32x4 e = {0.f, 0.f, 0.f, 0.f};
        const float* xc = X + h * d.RX + MB_ZS + tile * 16 + c;
#pragma unroll
        for (int s = 0; s < (RTENHIP_MB_EXPERIMENT == 2 ? 0 : KS); s++) {
          const float a = s % 4 == 0 ? wa[s / 4].x : s % 4 == 1 ? wa[s / 4].y : s % 4 == 2 ? wa[s / 4].z : wa[s / 4].w;
          e = __builtin_amdgcn_mfma_f32_16x16x4f32(a, xc[4 * s * d.RX], e, 0, 0, 0);
        }
        // Lane (c, h) holds channels 4h + r of pixel tile * 16 + c.
        float v[4] = {e[0], e[1], e[2], e[3]};
        const float bb[4] = {be.x, be.y, be.z, be.w};
#pragma unroll
        for (int r = 0; r < 4; r++) {
          if (d.has_be) v[r] = __fadd_rn(v[r], bb[r]);
          Eb[(4 * h + r) * d.RE + MB_ZS + tile * 16 + c] = mb_act(v[r], d.act_e, d.lo_e, d.hi_e);
        }
      }
    }
    // The chunk's 16 x 9 skip slots, copysign(0, -w) (see MB_ZS).
    if (t < 144) {
      const int cl = t / 9, k = t - cl * 9;  // channel cl = hh + 4 j of the chunk
      const float w = reinterpret_cast<const float*>(rec + GE * 64 + 4)[((cl & 3) * 9 + k) * 4 + (cl >> 2)];
      Eb[cl * re + k] = copysignf(0.f, -w);
    }
    // Chunk ch's expand planes, slots (and record ch + 1) complete; every
    // wave is past chunk ch - 1, so its plane buffer is free.
    __syncthreads();
    held[0] = nxt[0];
    held[1] = nxt[1];
    held_ok = pf;
    // 2. Depthwise (channels h + 4j of this lane's pixel) -> project MFMAs.
    {
      const float4* dwr = rec + GE * 64 + 4;
      float4 wd[9];
#pragma unroll
      for (int k = 0; k < 9; k++) wd[k] = dwr[h * 9 + k];
      const float4 bd = dwr[36 + h];
      float4 wp[MT];
#pragma unroll
      for (int m = 0; m < MT; m++) wp[m] = dwr[40 + m * 64 + lane];
#pragma unroll
      for (int u = 0; u < MAXT; u++) {
        if (wave + u * NW >= tout || RTENHIP_MB_EXPERIMENT == 1) break;
        // Two channels per packed f32 operation (v_pk_mul / v_pk_add: one
        // IEEE rounding per component, the same ops as apart).
        float dv[4];
#pragma unroll
        for (int jp = 0; jp < 2; jp++) {
          const float* ep0 = Eb + (h + 8 * jp) * re;
          const float* ep1 = ep0 + 4 * re;
          vm_f32x2 a = d.has_bd ? (jp == 0 ? (vm_f32x2){bd.x, bd.y} : (vm_f32x2){bd.z, bd.w}) : (vm_f32x2){0.f, 0.f};
#pragma unroll
          for (int k = 0; k < 9; k++) {
            const int idx = tidx[u][k];
            const vm_f32x2 ev = {ep0[idx], ep1[idx]};
            const vm_f32x2 w = jp == 0 ? (vm_f32x2){wd[k].x, wd[k].y} : (vm_f32x2){wd[k].z, wd[k].w};
            a = a + ev * w;  // a skipped tap adds -0
          }
          dv[2 * jp] = mb_act(a[0], d.act_d, d.lo_d, d.hi_d);
          dv[2 * jp + 1] = mb_act(a[1], d.act_d, d.lo_d, d.hi_d);
        }
        if constexpr (RTENHIP_MB_EXPERIMENT == 4) {
#pragma unroll
          for (int m = 0; m < MT; m++) acc[u][m][0] += dv[0] + dv[1] + dv[2] + dv[3];
          continue;
        }
#pragma unroll
        for (int m = 0; m < MT; m++) {
          acc[u][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(wp[m].x, dv[0], acc[u][m], 0, 0, 0);
          acc[u][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(wp[m].y, dv[1], acc[u][m], 0, 0, 0);
          acc[u][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(wp[m].z, dv[2], acc[u][m], 0, 0, 0);
          acc[u][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(wp[m].w, dv[3], acc[u][m], 0, 0, 0);
        }
      }
    }
    // End of a KC block of the project chain (every 16 chunks) or of K.
    if (((ch + 1) & 15) == 0 || ch + 1 == nchunks) {
#pragma unroll
      for (int u = 0; u < MAXT; u++)
#pragma unroll
        for (int m = 0; m < MT; m++) {
          const float4 bp = bp4[m * 4 + h];
          const float bb[4] = {bp.x, bp.y, bp.z, bp.w};
#pragma unroll
          for (int r = 0; r < 4; r++) {
            if (!folded)
              sum[u][m][r] = d.has_bp ? __fadd_rn(acc[u][m][r], bb[r]) : acc[u][m][r];
            else
              sum[u][m][r] = __fadd_rn(sum[u][m][r], acc[u][m][r]);
          }
          acc[u][m] = (mb_f32x4){0.f, 0.f, 0.f, 0.f};
        }
      folded = true;
    }
  }

  // Epilogue: residual, activation, store.  Lane (c, h) holds output
  // channels 16m + 4h + r of pixel tile * 16 + c.
#pragma unroll
  for (int u = 0; u < MAXT; u++) {
    const int tile = wave + u * NW;
    const int o = tile * 16 + c;
    if (tile >= tout) break;
    const bool ok = o < pout;
    const int ol = min(o, pout - 1) / OW, ox = min(o, pout - 1) - ol * OW;
    const int oy = oy0 + ol;
    const int64_t opix = (int64_t)oy * OW + ox;
#pragma unroll
    for (int m = 0; m < MT; m++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int co = 16 * m + 4 * h + r;
        if (co >= d.cout || !ok) continue;
        float v = sum[u][m][r];
        if (d.res_lds)
          v = __fadd_rn(v, X[co * d.RX + MB_ZS + (oy - ia) * W + ox]);
        else if (d.res)
          v = __fadd_rn(v, d.res[((int64_t)n * d.cout + co) * d.OH * OW + opix]);
        d.y[((int64_t)n * d.cout + co) * d.OH * OW + opix] = mb_act(v, d.act_p, d.lo_p, d.hi_p);
      }
  }
}

// Host side --------------------------------------------------------------

// cin = 0: a block without the expand conv (we, be unused).
int mbconv_block_pack_floats(int cin, int hid, int cout) {
  const int mt = (cout + 15) / 16;
  return (hid / 16) * mb_chunk_floats(cin, mt) + mt * 16;
}

// Repack the three convs' weights and biases into the lanes' operand order
// (see MbBlockDesc / the kernel): we [hid][cin], be [hid], wd [hid][9], bd
// [hid], wp [cout][hid], bp [cout] (biases may be null: zeros).
void mbconv_block_pack(const float* we, const float* be, const float* wd, const float* bd, const float* wp,
                       const float* bp, int cin, int hid, int cout, float* out) {
  const int mt = (cout + 15) / 16, ge = mb_ge(cin), cf = mb_chunk_floats(cin, mt);
  for (int ch = 0; ch < hid / 16; ch++) {
    float* r = out + (size_t)ch * cf;
    const int h0 = ch * 16;
    // Expand A: lane L: row h0 + L % 16, step s = 4g + i covers k = 4s + L / 16.
    for (int g = 0; g < ge; g++)
      for (int L = 0; L < 64; L++)
        for (int i = 0; i < 4; i++) {
          const int k = 4 * (4 * g + i) + L / 16;
          r[(g * 64 + L) * 4 + i] = k < cin ? we[(size_t)(h0 + L % 16) * cin + k] : 0.f;
        }
    r += ge * 256;
    // Expand bias: [h][r] = be[h0 + 4h + r].
    for (int i = 0; i < 16; i++) r[i] = be ? be[h0 + i] : 0.f;
    r += 16;
    // Depthwise: [h][tap][j] = wd[h0 + h + 4j][tap]; bias [h][j].
    for (int h = 0; h < 4; h++)
      for (int k = 0; k < 9; k++)
        for (int j = 0; j < 4; j++) r[(h * 9 + k) * 4 + j] = wd[(size_t)(h0 + h + 4 * j) * 9 + k];
    r += 144;
    for (int h = 0; h < 4; h++)
      for (int j = 0; j < 4; j++) r[h * 4 + j] = bd ? bd[h0 + h + 4 * j] : 0.f;
    r += 16;
    // Project A: tile m, lane L: row 16m + L % 16, step s covers k = h0 + 4s + L / 16.
    for (int m = 0; m < mt; m++)
      for (int L = 0; L < 64; L++)
        for (int s = 0; s < 4; s++) {
          const int o = 16 * m + L % 16;
          r[(m * 64 + L) * 4 + s] = o < cout ? wp[(size_t)o * hid + h0 + 4 * s + L / 16] : 0.f;
        }
  }
  float* b = out + (size_t)(hid / 16) * cf;
  for (int m = 0; m < mt; m++)
    for (int i = 0; i < 16; i++) b[m * 16 + i] = (bp && 16 * m + i < cout) ? bp[16 * m + i] : 0.f;
}

namespace {
// The instantiated shapes (MobileNetV2's blocks features.2 .. features.13):
// stride, C_in, project row tiles ceil(C_out / 16), threads per workgroup.
// 512 threads where the accumulators of 4 tiles per wave would not fit.
struct MbInst {
  int S, cin, mt, nt;
  bool exp;
};
constexpr MbInst kMbInsts[] = {{2, 16, 2, 256, true}, {1, 24, 2, 256, true}, {2, 24, 2, 256, true},
                               {1, 32, 2, 256, true}, {2, 32, 4, 512, true}, {1, 64, 4, 512, true},
                               {1, 64, 6, 512, true}, {1, 96, 6, 512, true}, {1, 32, 1, 256, false}};

const MbInst* mb_inst(int S, int cin, int mt, bool exp) {
  for (const MbInst& m : kMbInsts)
    if (m.S == S && m.cin == cin && m.mt == mt && m.exp == exp) return &m;
  return nullptr;
}

struct MbGeom {
  int TR, RX, RE, NT, MAXT;
  size_t lds;
};

// Band height and LDS layout: the most output rows whose staged input band,
// two expand plane sets and three weight records fit the budget, with at most
// 4 (256 threads) / 2 (512 threads) output pixel tiles per wave.  Row
// strides: X rows are read 16 consecutive floats per half-wave (2 rows per
// 32-lane group): stride = 16 (mod 32); E rows are read at pixel steps of S:
// stride 16 (mod 32) for S = 1, odd for S = 2.
// N > 0: then the band is also cut until the grid fills every CU once (two
// 256-thread or one 512-thread workgroup per CU), down to 2 output rows.
bool mb_geom(int cin, int cout, int H, int W, int OH, int OW, int S, bool exp, MbGeom& g, int N = 0) {
  const MbInst* in = mb_inst(S, cin, (cout + 15) / 16, exp);
  if (!in) return false;
  // 256 threads: two workgroups per CU; 512 (about 200 VGPRs): one.
  const int nt = in->nt, nw = nt / 64, maxt = nt == 256 ? 4 : 2;
  const size_t budget = nt == 256 ? 80 * 1024 : 156 * 1024;
  const int cf = mb_chunk_floats(exp ? cin : 0, in->mt);
  if (cf / 4 > 2 * nt) return false;  // a record is prefetched as two float4s per thread
  for (int tr = OH; tr >= 1; tr--) {
    const int rows = std::min(H, (tr - 1) * S + 3);  // input rows of the widest band
    const int tin16 = MB_ZS + (rows * W + 15) / 16 * 16;  // slots + pixels
    // (without the expand, the depthwise reads the band: its stride follows E's rule)
    int rx = tin16;
    if (exp || S == 1)
      while (rx % 32 != 16) rx++;
    else if (rx % 2 == 0)
      rx++;
    int re = tin16;
    if (S == 1)
      while (re % 32 != 16) re++;
    else if (re % 2 == 0)
      re++;
    const size_t lds = ((size_t)cin * rx + (exp ? 2 * 16 * (size_t)re : 0) + 3 * (size_t)cf) * sizeof(float);
    const int tout = (tr * OW + 15) / 16;
    if (lds > budget || (tout + nw - 1) / nw > maxt) continue;
    const int64_t wgs = (int64_t)N * ((OH + tr - 1) / tr);
    if (N > 0 && tr > 2 && wgs < (nt == 256 ? 512 : 256)) continue;
    g.TR = tr;
    g.RX = rx;
    g.RE = re;
    g.NT = nt;
    g.MAXT = maxt;
    g.lds = lds;
    return true;
  }
  return false;
}
}  // namespace

// Whether the fused kernel takes this block: an instantiated (stride, C_in,
// C_out) shape (kMbInsts), 3x3 depthwise with pads <= 1, hidden a multiple
// of 16, and a band that fits LDS.  RTENHIP_MBCONV=0 disables the fusion.
bool mbconv_block_eligible(int cin, int hid, int cout, int H, int W, int OH, int OW, int S, int pt, int pl, int pb,
                           int pr, bool expand) {
  // Opt-in (RTENHIP_MBCONV=all fuses every instantiated shape; unset or 0:
  // none).  Measured at MobileNetV2 batch 128 (profiles/r4_mbconv_block.txt,
  // kernel time per block run, fused vs the kernels apart): 1.0-1.8x slower
  // on every block (features.4 200 vs 195 us, features.3 291 vs 277 us), so
  // the plan keeps the convs apart by default.
  const char* e = getenv("RTENHIP_MBCONV");
  if (!e || strcmp(e, "all") != 0) return false;
  if (pt > 1 || pl > 1 || pb > 1 || pr > 1) return false;
  if (hid % 16 != 0 || hid <= 0 || cout <= 0 || (!expand && hid != cin)) return false;
  MbGeom g;
  return mb_geom(cin, cout, H, W, OH, OW, S, expand, g);
}

rtenhip_status launch_mbconv_block(const float* x, const float* pk, const float* res, bool res_is_x, float* y, int N,
                                   int cin, int hid, int cout, int H, int W, int OH, int OW, int S, int pt, int pl,
                                   int act_e, float lo_e, float hi_e, int act_d, float lo_d, float hi_d, int act_p,
                                   float lo_p, float hi_p, bool has_be, bool has_bd, bool has_bp, bool expand,
                                   hipStream_t s) {
  if ((int64_t)N * cout * OH * OW == 0) return RTENHIP_OK;
  MbGeom g;
  if (hid % 16 != 0 || (!expand && hid != cin) || !mb_geom(cin, cout, H, W, OH, OW, S, expand, g, N))
    return fail(RTENHIP_UNSUPPORTED_VALUE, "inverted residual block: unsupported shape");
  if (res_is_x && (S != 1 || cin != cout || OH != H || OW != W))
    return fail(RTENHIP_INVALID_VALUE, "inverted residual block: residual shape");
  if (N > 65535) return fail(RTENHIP_UNSUPPORTED_VALUE, "inverted residual block: batch too large");
  MbBlockDesc d{};
  d.x = x;
  d.pk = pk;
  d.res = res_is_x ? nullptr : res;
  d.res_lds = res_is_x ? 1 : 0;
  d.y = y;
  d.hid = hid;
  d.cout = cout;
  d.H = H;
  d.W = W;
  d.OH = OH;
  d.OW = OW;
  d.pt = pt;
  d.pl = pl;
  d.TR = g.TR;
  d.RX = g.RX;
  d.RE = g.RE;
  d.act_e = act_e;
  d.lo_e = lo_e;
  d.hi_e = hi_e;
  d.act_d = act_d;
  d.lo_d = lo_d;
  d.hi_d = hi_d;
  d.act_p = act_p;
  d.lo_p = lo_p;
  d.hi_p = hi_p;
  d.has_be = has_be;
  d.has_bd = has_bd;
  d.has_bp = has_bp;
  for (int kx = 0; kx < 3; kx++) {
    d.omin[kx] = pl - kx > 0 ? pl - kx : 0;
    const int t = W + pl - kx > 0 ? W + pl - kx : 0;
    const int omax = (t + S - 1) / S;
    d.omax[kx] = omax > OW ? OW : omax;
  }
  const int bands = (OH + g.TR - 1) / g.TR;
  const dim3 grid((unsigned)bands, (unsigned)N);
  const int mt = (cout + 15) / 16;
#define MB_LAUNCH(S_, CIN_, MT_, NT_, EXP_)                                                                   \
  if (S == S_ && cin == CIN_ && mt == MT_ && expand == EXP_) {                                             \
    hipLaunchKernelGGL((mbconv_block_kernel<NT_, S_, CIN_, MT_, NT_ == 256 ? 4 : 2, EXP_>), grid, dim3(NT_), g.lds, \
                       s, d);                                                                                 \
    RTENHIP_LAUNCH_CHECK();                                                                                   \
    return RTENHIP_OK;                                                                                        \
  }
  MB_LAUNCH(2, 16, 2, 256, true)
  MB_LAUNCH(1, 24, 2, 256, true)
  MB_LAUNCH(2, 24, 2, 256, true)
  MB_LAUNCH(1, 32, 2, 256, true)
  MB_LAUNCH(2, 32, 4, 512, true)
  MB_LAUNCH(1, 64, 4, 512, true)
  MB_LAUNCH(1, 64, 6, 512, true)
  MB_LAUNCH(1, 96, 6, 512, true)
  MB_LAUNCH(1, 32, 1, 256, false)
#undef MB_LAUNCH
  return fail(RTENHIP_UNSUPPORTED_VALUE, "inverted residual block: unsupported shape");
}

}  // namespace rtenhip
