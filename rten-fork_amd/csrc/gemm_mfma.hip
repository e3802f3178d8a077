// f32 implicit-GEMM engine for gfx950 (CDNA4) on v_mfma_f32_32x32x2_f32.
//
// Replaces RTen's BLIS GEMM (src/gemm.rs:733-1050), its packing
// (src/gemm/packing.rs) and the virtual im2col B operand
// (src/ops/conv/im2col.rs:44-367) with one kernel:
//
//   C[M, N] = epilogue( alpha * A[M, K] @ B[K, N] )
//
// where B is a dense strided matrix, the im2col matrix of an NCHW image batch
// (batch folded into N = images * OH * OW, unlike the reference's per-image
// GEMMs — conv.rs:243-270), or a pointwise-conv view.  Tiles are staged
// global -> VGPR -> LDS (double buffered, one barrier per K-tile) and consumed
// by 32x32x2 f32 MFMAs.
//
// Summation order = the reference's.  gemm_impl splits K into KC=256 blocks
// (depth_block_size, gemm.rs:546-548); the FmaKernel micro-kernel computes
// each block as an fma chain from +0 (kernels.rs:206-316) and blocks are
// combined in order as out = out + chain, with the bias added after block 0
// (gemm_block, gemm.rs:1034-1047).  v_mfma_f32_32x32x2_f32 is bit-for-bit a
// k-ordered fmaf chain (lane-half 0's k first), so each wave keeps a fresh
// accumulator per 256-deep block and folds it into a running sum at every
// block boundary: results are bit-identical to RTen's CPU GEMM.
#include "common.h"
#include "vecmath.h"

#include <algorithm>

namespace rtenhip {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int KC = 256;      // reference depth block (gemm.rs:546-548)
constexpr int PAD = 4;       // LDS row pad (floats): 2-way at worst on writes

// NT threads (NT/64 waves in a WAVES_M x WAVES_N grid), BM x BN output tile,
// BK-deep K tiles (BK divides KC), MINW = min waves per SIMD for the
// register allocator.
// BMODE 0: dense B, dense output out[m*out_m + n] (GEMM / MatMul).
// BMODE 1: im2col B, NCHW output.  BMODE 2: pointwise-conv B, NCHW output.
// All offsets inside one operand are 32-bit (the host checks sizes).
template <int NT, int BM, int BN, int BK, int WAVES_M, int WAVES_N, int MINW, int BMODE,
          bool MULTI_KB>
__global__ __launch_bounds__(NT, MINW) void gemm_mfma_kernel(GemmDesc d, int tiles_m, int tiles_n) {
  static_assert(KC % BK == 0, "BK divides KC");
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int MI = WM / 32, NI = WN / 32;
  constexpr int APT = BM * BK / NT;  // A elements staged per thread
  constexpr int BPT = BN * BK / NT;  // B elements staged per thread
  constexpr int KSTEP = NT / BN;
  static_assert(WAVES_M * WAVES_N == NT / 64, "wave grid");
  static_assert(MI >= 1 && NI >= 1, "wave tile >= 32x32");
  static_assert(NT % BN == 0 && NT % BM == 0, "tile widths divide the block");
  static_assert(APT >= 1 && BPT >= 1, "staging");

  if (BMODE == 0 && d.nbatch > 1) {
    // Batched MatMul: offset the operands by this batch's prefix index.
    int64_t rem = blockIdx.y, oa = 0, ob = 0, oo = 0;
    for (int i = d.nbp - 1; i >= 0; i--) {
      const int64_t idx = rem % d.pshape[i];
      rem /= d.pshape[i];
      oa += idx * d.pa[i];
      ob += idx * d.pb[i];
      oo += idx * d.po[i];
    }
    d.a += oa;
    d.b += ob;
    d.out += oo;
    if (d.residual) d.residual += oo;
  }

  __shared__ float As[2][BK][BM + PAD];
  __shared__ float Bs[2][BK][BN + PAD];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = (wave / WAVES_N) * WM;
  const int wn = (wave % WAVES_N) * WN;

  // XCD-aware, bijective block remap: blocks b and b+8 share an XCD, so give
  // each XCD a contiguous run of tiles (neighbouring tiles share A/B panels
  // in that XCD's L2).  Speed only; correctness never depends on placement.
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tm = (wg % tiles_m) * BM;
  const int tn = (wg / tiles_m) * BN;

  const int M = d.M, N = d.N, K = d.K;
  const int m_lim = M - 1 - tm;  // largest valid local row
  const int n_lim = N - 1 - tn;  // largest valid local column

  // ---- A staging: element e = tid + NT*i of the BK x BM tile ----
  // m-contiguous A: (kk, mm) = (e / BM, e % BM); k-contiguous: (e % BK, e / BK).
  const bool a_mcontig = d.a_m == 1 && d.a_k != 1;
  const int a_mm0 = a_mcontig ? tid % BM : tid / BK;
  const int a_kk0 = a_mcontig ? tid / BM : tid % BK;
  const int a_dm = a_mcontig ? 0 : NT / BK;
  const int a_dk = a_mcontig ? NT / BM : 0;
  const int am = (int)d.a_m, ak = (int)d.a_k;
  const float* a_tile = d.a + (int64_t)tm * d.a_m;

  // ---- B staging ----
  const int n_local = tid % BN;
  const int kr0 = __builtin_amdgcn_readfirstlane(tid / BN);
  const bool n_valid = n_local <= n_lim;
  const bool b_ncontig = !(d.b_k == 1 && d.b_n != 1);
  const int b_nn0 = b_ncontig ? n_local : tid / BK;
  const int b_kk0 = b_ncontig ? kr0 : tid % BK;
  const int b_dn = b_ncontig ? 0 : NT / BK;
  const int b_dk = b_ncontig ? KSTEP : 0;
  const int bk_ = (int)d.b_k, bn_ = (int)d.b_n;
  const float* b_tile = d.b + (BMODE == 0 ? (int64_t)tn * d.b_n : 0);
  int iy0 = 0, ix0 = 0, colbase = 0;
  if constexpr (BMODE != 0) {
    const int ncl = n_valid ? tn + n_local : 0;
    const int img = ncl / d.P;
    const int p = ncl - img * d.P;
    if constexpr (BMODE == 1) {
      const int oy = p / d.OW;
      const int ox = p - oy * d.OW;
      iy0 = oy * d.sh - d.pt;
      ix0 = ox * d.sw - d.pl;
      colbase = img * (int)d.x_img + iy0 * d.W + ix0;
    } else {
      colbase = img * (int)d.x_img + p;
    }
  }

  float ra[APT], rb[BPT];

  // Loads are never skipped: out-of-range elements read a clamped, valid
  // address and are replaced by 0 (no divergent branches in the K loop).
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < APT; i++) {
      const int mm = a_mm0 + a_dm * i, kk = k0 + a_kk0 + a_dk * i;
      const bool ok = mm <= m_lim && kk < K;
      const float v = a_tile[min(mm, m_lim) * am + min(kk, K - 1) * ak];
      ra[i] = ok ? v : 0.f;
    }
#pragma unroll
    for (int i = 0; i < BPT; i++) {
      float v;
      bool ok;
      if constexpr (BMODE == 0) {
        const int nn = b_nn0 + b_dn * i, kk = k0 + b_kk0 + b_dk * i;
        ok = nn <= n_lim && kk < K;
        v = b_tile[min(kk, K - 1) * bk_ + min(nn, n_lim) * bn_];
      } else if constexpr (BMODE == 1) {
        const int k = k0 + kr0 + KSTEP * i;  // wave-uniform -> scalar table load
        const int2 t = d.ktab[min(k, K - 1)];
        const int y = iy0 + (t.y >> 16);
        const int x = ix0 + (t.y & 0xffff);
        ok = k < K && n_valid && (unsigned)y < (unsigned)d.H && (unsigned)x < (unsigned)d.W;
        v = d.b[ok ? colbase + t.x : 0];
      } else {
        const int k = k0 + kr0 + KSTEP * i;
        ok = k < K && n_valid;
        v = d.b[ok ? colbase + k * d.P : 0];
      }
      rb[i] = ok ? v : 0.f;
    }
  };

  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < APT; i++) As[buf][a_kk0 + a_dk * i][a_mm0 + a_dm * i] = ra[i];
#pragma unroll
    for (int i = 0; i < BPT; i++) {
      if constexpr (BMODE == 0)
        Bs[buf][b_kk0 + b_dk * i][b_nn0 + b_dn * i] = rb[i];
      else
        Bs[buf][kr0 + KSTEP * i][n_local] = rb[i];
    }
  };

  f32x16 acc[MI][NI];
  f32x16 sum[MULTI_KB ? MI : 1][MULTI_KB ? NI : 1];
#pragma unroll
  for (int mi = 0; mi < MI; mi++)
#pragma unroll
    for (int ni = 0; ni < NI; ni++) acc[mi][ni] = (f32x16){0};

  const int half = lane >> 5;
  const int l32 = lane & 31;

  // Local row of accumulator register j: C/D map of the 32x32 MFMA family on
  // gfx950, col = lane&31, row = (j&3) + 8*(j>>2) + 4*(lane>>5).
  auto lrow = [&](int mi, int j) { return wm + mi * 32 + (j & 3) + 8 * (j >> 2) + 4 * half; };

  // First K-block: v = alpha*acc (beta == 0: out not read) or
  // fma(acc, alpha, beta*cin) (simd_gemm store variants, kernels.rs:268-315),
  // then + bias[m] (gemm_block, gemm.rs:1034-1047).
  auto first_block = [&](f32x16& v, const f32x16& a, int mi, int ni) {
    const int nl = min(wn + ni * 32 + l32, n_lim);
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const int ml = min(lrow(mi, j), m_lim);
      float x;
      if (BMODE == 0 && d.cin) {
        const float c = d.cin[(int64_t)(tm + ml) * d.out_m + tn + nl];
        x = __fmaf_rn(a[j], d.alpha, __fmul_rn(c, d.beta));
      } else {
        x = __fmul_rn(a[j], d.alpha);
      }
      if (d.bias) x = __fadd_rn(x, d.bias[tm + ml]);
      v[j] = x;
    }
  };

  int buf = 0;
  const int ntiles = (K + BK - 1) / BK;
  load_tile(0);
  store_tile(0);
  __syncthreads();

  for (int t = 0; t < ntiles; t++) {
    const bool more = t + 1 < ntiles;
    if (more) load_tile((t + 1) * BK);

#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      float av[MI], bv[NI];
#pragma unroll
      for (int mi = 0; mi < MI; mi++) av[mi] = As[buf][kk + half][wm + mi * 32 + l32];
#pragma unroll
      for (int ni = 0; ni < NI; ni++) bv[ni] = Bs[buf][kk + half][wn + ni * 32 + l32];
#pragma unroll
      for (int mi = 0; mi < MI; mi++)
#pragma unroll
        for (int ni = 0; ni < NI; ni++)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[mi], bv[ni], acc[mi][ni], 0, 0, 0);
    }

    if constexpr (MULTI_KB) {
      // KC-block boundary: fold this block's chain into the running sum.
      if (((t + 1) * BK) % KC == 0 || !more) {
        if (t * BK < KC) {
#pragma unroll
          for (int mi = 0; mi < MI; mi++)
#pragma unroll
            for (int ni = 0; ni < NI; ni++) first_block(sum[mi][ni], acc[mi][ni], mi, ni);
        } else {
#pragma unroll
          for (int mi = 0; mi < MI; mi++)
#pragma unroll
            for (int ni = 0; ni < NI; ni++)
#pragma unroll
              for (int j = 0; j < 16; j++)
                sum[mi][ni][j] = __fmaf_rn(acc[mi][ni][j], d.alpha, sum[mi][ni][j]);
        }
#pragma unroll
        for (int mi = 0; mi < MI; mi++)
#pragma unroll
          for (int ni = 0; ni < NI; ni++) acc[mi][ni] = (f32x16){0};
      }
    }

    if (more) store_tile(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }

  // ---- epilogue: (+ residual) -> activation -> store ----
  const bool full_tile = m_lim >= BM - 1 && n_lim >= BN - 1;
#pragma unroll
  for (int ni = 0; ni < NI; ni++) {
    const int nl = wn + ni * 32 + l32;
    const bool ncol_ok = nl <= n_lim;
    int nbase;       // element offset of (row 0, this column) in out
    int mstride;     // element stride between rows
    if constexpr (BMODE == 0) {
      nbase = tn + min(nl, n_lim);
      mstride = (int)d.out_m;
    } else {
      const int n = tn + min(nl, n_lim);
      const int img = n / d.P;
      nbase = img * (int)d.out_img + (n - img * d.P);
      mstride = d.P;
    }
#pragma unroll
    for (int mi = 0; mi < MI; mi++) {
      f32x16 v;
      if constexpr (MULTI_KB) {
        v = sum[mi][ni];
      } else {
        first_block(v, acc[mi][ni], mi, ni);
      }
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const int ml = lrow(mi, j);
        const int idx = nbase + (tm + ml) * mstride;
        float x = v[j];
        if (d.residual) x = __fadd_rn(x, d.residual[full_tile || (ncol_ok && ml <= m_lim) ? idx : 0]);
        if (d.act == RTENHIP_ACT_RELU) {
          x = fmaxf(x, 0.f);
        } else if (d.act == RTENHIP_ACT_CLIP) {
          x = rust_clamp(x, d.act_lo, d.act_hi);
        }
        if (full_tile || (ncol_ok && ml <= m_lim)) d.out[idx] = x;
      }
    }
  }
}

template <int NT, int BM, int BN, int BK, int WM_, int WN_, int MINW, int BMODE>
static void launch_cfg(const GemmDesc& d, hipStream_t s) {
  int tiles_m = (d.M + BM - 1) / BM, tiles_n = (d.N + BN - 1) / BN;
  dim3 grid(tiles_m * tiles_n, d.nbatch > 1 ? d.nbatch : 1), block(NT);
  if (d.K > KC)
    hipLaunchKernelGGL((gemm_mfma_kernel<NT, BM, BN, BK, WM_, WN_, MINW, BMODE, true>), grid,
                       block, 0, s, d, tiles_m, tiles_n);
  else
    hipLaunchKernelGGL((gemm_mfma_kernel<NT, BM, BN, BK, WM_, WN_, MINW, BMODE, false>), grid,
                       block, 0, s, d, tiles_m, tiles_n);
}

// Tile configurations (id -> template); RTENHIP_GEMM_CFG forces one (tuning).
static int g_forced_cfg = -2;
static int forced_cfg() {
  if (g_forced_cfg == -2) {
    const char* s = getenv("RTENHIP_GEMM_CFG");
    g_forced_cfg = s ? atoi(s) : -1;
  }
  return g_forced_cfg;
}
int gemm_forced_cfg() { return forced_cfg(); }

}  // namespace rtenhip

extern "C" void rtenhip_debug_set_gemm_config(int cfg) { rtenhip::g_forced_cfg = cfg; }

namespace rtenhip {

template <int BMODE>
static void launch_mode(const GemmDesc& d, hipStream_t s) {
  int cfg = forced_cfg();
  if (cfg < 0) cfg = d.M <= 64 ? 1 : 0;
  switch (cfg) {
    case 1: launch_cfg<512, 64, 128, 16, 2, 4, 2, BMODE>(d, s); break;
    case 2: launch_cfg<256, 128, 128, 16, 2, 2, 2, BMODE>(d, s); break;
    case 3: launch_cfg<256, 128, 128, 32, 2, 2, 2, BMODE>(d, s); break;
    case 4: launch_cfg<512, 128, 256, 16, 2, 4, 1, BMODE>(d, s); break;
    case 5: launch_cfg<256, 64, 128, 16, 2, 2, 2, BMODE>(d, s); break;
    case 6: launch_cfg<256, 128, 64, 16, 2, 2, 2, BMODE>(d, s); break;
    case 7: launch_cfg<512, 128, 128, 32, 4, 2, 2, BMODE>(d, s); break;
    default: launch_cfg<512, 128, 128, 16, 4, 2, 2, BMODE>(d, s); break;
  }
}

// K == 0 (gemm.rs:757-765): out = beta * (beta == 0 ? 0 : out); no bias.
__global__ void gemm_k0_kernel(float* out, int64_t out_m, int M, int N, float beta) {
  const int64_t total = (int64_t)M * N;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    float* p = out + (i / N) * out_m + (i % N);
    const float t = beta == 0.f ? 0.f : *p;
    *p = __fmul_rn(beta, t);
  }
}

// Small-M dense GEMM (the FC layer: M = batch <= 256, N = 1000, K = 2048).
// MFMA tiles would leave most CUs idle at this size, so the K blocks are
// split across workgroups instead -- exactly at the reference's KC = 256
// boundaries, which keeps the arithmetic identical: kernel 1 computes each
// block's fma chain from +0 in k order (one lane per row m, four columns per
// wave, B read as wave-uniform scalar loads) into a workspace; kernel 2 folds
// the block chains in order: fma(c0, alpha, beta*cin) or alpha*c0, + bias[m],
// then fma(c_b, alpha, sum) (gemm.rs:1004-1050).
typedef __attribute__((address_space(4))) const float const_float_t;

template <bool UNIT>  // a_k == 1 and b_k == 1 (row-major A, B = W^T view)
__global__ __launch_bounds__(256) void gemm_kblock_kernel(GemmDesc d, float* __restrict__ ws) {
  constexpr int COLS = 4;  // columns per wave
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int kb = blockIdx.y;
  const int n0 = blockIdx.x * (4 * COLS) + w * COLS;
  const int mrow = blockIdx.z * 64 + lane;  // 64 rows per z slice
  const int m = min(mrow, d.M - 1);
  const int k0 = kb * 256, k1 = min(d.K, k0 + 256);
  const float* ap = d.a + (int64_t)m * d.a_m;
  const_float_t* bp = (const_float_t*)d.b;
  const int64_t ak = UNIT ? 1 : d.a_k, bk = UNIT ? 1 : d.b_k;
  float c[COLS];
#pragma unroll
  for (int j = 0; j < COLS; j++) c[j] = 0.f;
  int nn[COLS];
#pragma unroll
  for (int j = 0; j < COLS; j++) nn[j] = min(n0 + j, d.N - 1);
  // Chunks of 16 k: all loads of a chunk are issued before its fma chain.
  int k = k0;
  for (; k + 16 <= k1; k += 16) {
    float av[16], bv[16][COLS];
#pragma unroll
    for (int t = 0; t < 16; t++) av[t] = ap[(int64_t)(k + t) * ak];
#pragma unroll
    for (int t = 0; t < 16; t++)
#pragma unroll
      for (int j = 0; j < COLS; j++) bv[t][j] = bp[(int64_t)(k + t) * bk + (int64_t)nn[j] * d.b_n];
#pragma unroll
    for (int t = 0; t < 16; t++)
#pragma unroll
      for (int j = 0; j < COLS; j++) c[j] = __fmaf_rn(av[t], bv[t][j], c[j]);
  }
  for (; k < k1; k++) {
    const float av = ap[(int64_t)k * d.a_k];
#pragma unroll
    for (int j = 0; j < COLS; j++)
      c[j] = __fmaf_rn(av, bp[(int64_t)k * d.b_k + (int64_t)nn[j] * d.b_n], c[j]);
  }
  if (mrow >= d.M) return;
#pragma unroll
  for (int j = 0; j < COLS; j++)
    if (n0 + j < d.N) ws[((int64_t)kb * d.M + mrow) * d.N + n0 + j] = c[j];
}

__global__ __launch_bounds__(256) void gemm_kfold_kernel(GemmDesc d, const float* __restrict__ ws,
                                                         int nkb) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t MN = (int64_t)d.M * d.N;
  if (i >= MN) return;
  const int m = (int)(i / d.N), n = (int)(i - (int64_t)m * d.N);
  const float c0 = ws[i];
  float x;
  if (d.cin) {
    x = __fmaf_rn(c0, d.alpha, __fmul_rn(d.cin[(int64_t)m * d.out_m + n], d.beta));
  } else {
    x = __fmul_rn(c0, d.alpha);
  }
  if (d.bias) x = __fadd_rn(x, d.bias[m]);
  for (int kb = 1; kb < nkb; kb++) x = __fmaf_rn(ws[kb * MN + i], d.alpha, x);
  if (d.act == RTENHIP_ACT_RELU) {
    x = fmaxf(x, 0.f);
  } else if (d.act == RTENHIP_ACT_CLIP) {
    x = rust_clamp(x, d.act_lo, d.act_hi);
  }
  d.out[(int64_t)m * d.out_m + n] = x;
}

bool gemm_smallm_eligible(const GemmDesc& d) {
  return d.K > 0 && d.bmode == 0 && d.nbatch <= 1 && !d.residual && d.M <= 256 && d.N >= 64 &&
         (int64_t)d.M * d.N <= (int64_t(1) << 20) && g_forced_cfg < 0;
}

int64_t gemm_smallm_ws_floats(const GemmDesc& d) {
  return (int64_t)((d.K + 255) / 256) * d.M * d.N;
}

rtenhip_status launch_gemm_smallm(const GemmDesc& d, float* ws, hipStream_t s) {
  const int nkb = (d.K + 255) / 256;
  dim3 grid((d.N + 15) / 16, nkb, (d.M + 63) / 64);
  if (d.a_k == 1 && d.b_k == 1)
    hipLaunchKernelGGL(gemm_kblock_kernel<true>, grid, dim3(256), 0, s, d, ws);
  else
    hipLaunchKernelGGL(gemm_kblock_kernel<false>, grid, dim3(256), 0, s, d, ws);
  RTENHIP_LAUNCH_CHECK();
  const int64_t MN = (int64_t)d.M * d.N;
  hipLaunchKernelGGL(gemm_kfold_kernel, dim3((unsigned)((MN + 255) / 256)), dim3(256), 0, s, d,
                     (const float*)ws, nkb);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

rtenhip_status launch_gemm(const GemmDesc& d, hipStream_t s) {
  if (d.M <= 0 || d.N <= 0) return RTENHIP_OK;

  if (d.K <= 0) {
    // The tiled kernel issues clamped loads and needs K >= 1.
    if (d.bmode != 0) return RTENHIP_OK;
    const int64_t total = (int64_t)d.M * d.N;
    const int blocks = (int)std::min<int64_t>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(gemm_k0_kernel, dim3(blocks), dim3(256), 0, s, d.out, d.out_m, d.M, d.N,
                       d.beta);
    RTENHIP_LAUNCH_CHECK();
    return RTENHIP_OK;
  }
  switch (d.bmode) {
    case 0:
      launch_mode<0>(d, s);
      break;
    case 1:
      launch_mode<1>(d, s);
      break;
    default:
      launch_mode<2>(d, s);
      break;
  }
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

// ---------------------------------------------------------------------------
// gemv (M == 1, unpacked A and B): gemm.rs:651-704 with simd_gemv*
// (kernels.rs:26-194) on the AVX2 kernel (S::LEN = 8).  One thread per output
// column reproduces the reference's exact order:
//  - column blocks of >= 128 are independent; K is split in blocks of 512
//    (B unit row stride, i.e. transposed) or 8 (otherwise), beta applies to
//    the first block and 1.0 after; bias added at the end.
//  - b_rs == 1 (simd_gemv_transposed): 8 lane partial chains over k = 8t+j,
//    __m256::sum tree, remainder k's chained, out = alpha*acc (+ beta*out).
//  - b_cs == 1: 32-column tiles are plain chains; remainder columns use a
//    non-fused acc += a*b and out = beta*out + acc*alpha.
//  - else (fallback): chain, acc *= alpha, out = acc (+ beta*out).
// ---------------------------------------------------------------------------
__global__ void gemv_kernel(int64_t N, int64_t K, const float* __restrict__ a,
                            const float* __restrict__ b, int64_t b_rs, int64_t b_cs,
                            float* __restrict__ out, float alpha, float beta,
                            const float* __restrict__ bias, int64_t bbs, const float* __restrict__ cin,
                            int64_t cin_stride) {
  int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= N) return;
  // Column chunk handled by one gemv_kernel call in the reference.
  const int64_t start = c / bbs * bbs;
  const int64_t width = min(bbs, N - start);
  const int64_t full8 = start + width / 8 * 8;
  const int64_t full32 = start + width / 32 * 32;
  const int64_t kbs = b_rs == 1 ? 512 : 8;
  float o = beta == 0.f ? 0.f : (cin ? cin[c * cin_stride] : out[c]);
  float eb = beta;
  for (int64_t k0 = 0; k0 < K; k0 += kbs) {
    const int64_t k1 = min(K, k0 + kbs);
    float res;
    if (b_rs == 1) {
      // Column tiles of 8 inside the call; the chunk's partial tile goes to
      // simd_gemv_fallback.
      if (c < full8) {
        float lanes[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const int64_t depth = k1 - k0, nfull = depth / 8 * 8;
        const float* col = b + c * b_cs;
        for (int64_t d0 = 0; d0 < nfull; d0 += 8)
#pragma unroll
          for (int j = 0; j < 8; j++) lanes[j] = __fmaf_rn(a[k0 + d0 + j], col[k0 + d0 + j], lanes[j]);
        float s4[4], s2[2];
#pragma unroll
        for (int i = 0; i < 4; i++) s4[i] = __fadd_rn(lanes[i], lanes[i + 4]);
#pragma unroll
        for (int i = 0; i < 2; i++) s2[i] = __fadd_rn(s4[i], s4[i + 2]);
        float acc = __fadd_rn(s2[0], s2[1]);
        for (int64_t k = k0 + nfull; k < k1; k++) acc = __fmaf_rn(a[k], col[k], acc);
        res = eb == 0.f ? __fmul_rn(alpha, acc) : __fadd_rn(__fmul_rn(alpha, acc), __fmul_rn(eb, o));
      } else {
        float acc = 0.f;
        for (int64_t k = k0; k < k1; k++) acc = __fmaf_rn(a[k], b[k * b_rs + c * b_cs], acc);
        acc = __fmul_rn(acc, alpha);
        res = eb == 0.f ? acc : __fadd_rn(acc, __fmul_rn(eb, o));
      }
    } else if (b_cs == 1) {
      if (c < full32) {
        float acc = 0.f;
        for (int64_t k = k0; k < k1; k++) acc = __fmaf_rn(a[k], b[k * b_rs + c], acc);
        if (alpha != 1.f) acc = __fmul_rn(acc, alpha);
        if (eb == 0.f)
          res = acc;
        else if (eb == 1.f)
          res = __fadd_rn(o, acc);
        else
          res = __fmaf_rn(o, eb, acc);
      } else {
        float acc = 0.f;
        for (int64_t k = k0; k < k1; k++) acc = __fadd_rn(acc, __fmul_rn(a[k], b[k * b_rs + c]));
        float t = eb == 0.f ? 0.f : o;
        res = __fadd_rn(__fmul_rn(eb, t), __fmul_rn(acc, alpha));
      }
    } else {
      float acc = 0.f;
      for (int64_t k = k0; k < k1; k++) acc = __fmaf_rn(a[k], b[k * b_rs + c * b_cs], acc);
      acc = __fmul_rn(acc, alpha);
      res = eb == 0.f ? acc : __fadd_rn(acc, __fmul_rn(eb, o));
    }
    o = res;
    eb = 1.f;
  }
  if (bias) o = __fadd_rn(o, bias[0]);
  out[c] = o;
}

// gemv with B in unit row stride (simd_gemv_transposed; the FC layer at batch
// 1, B = W^T): one wavefront per output column instead of one thread.  The
// reference's eight lane chains of a 512-deep K block are independent of the
// other blocks' (the lanes restart at zero per block), so lane kb*8+j of a
// pass runs chain j of block kb (8 blocks per pass, 64 FMAs each) and a wave
// reads a column as coalesced 32-byte runs.  The __m256::sum tree is three
// xor shuffles (each a single commutative add, as in the reference), the
// block's remainder k's are chained by the group's first lane, and lane 0
// folds the blocks in K order (alpha*acc + eb*out, eb = beta then 1).  Columns
// in a chunk's partial 8-wide tile take simd_gemv_fallback on lane 0.
// One output column c of the transposed gemv (the body of gemv_t_kernel).
__device__ __forceinline__ void gemv_t_column(const int64_t c, int64_t N, int64_t K, const float* a,
                                              const float* __restrict__ b, int64_t b_cs, float* __restrict__ out,
                                              float alpha, float beta, const float* __restrict__ bias, int64_t bbs,
                                              const float* __restrict__ cin, int64_t cin_stride) {
  const int lane = threadIdx.x & 63;
  const int64_t start = c / bbs * bbs;
  const int64_t width = min(bbs, N - start);
  const bool tiled = c < start + width / 8 * 8;
  const float* col = b + c * b_cs;
  float o = beta == 0.f ? 0.f : (cin ? cin[c * cin_stride] : out[c]);
  float eb = beta;
  constexpr int64_t KB = 512;
  const int64_t nkb = (K + KB - 1) / KB;
  if (!tiled) {
    if (lane == 0)
      for (int64_t k0 = 0; k0 < K; k0 += KB) {
        const int64_t k1 = min(K, k0 + KB);
        float acc = 0.f;
        for (int64_t k = k0; k < k1; k++) acc = __fmaf_rn(a[k], col[k], acc);
        acc = __fmul_rn(acc, alpha);
        o = eb == 0.f ? acc : __fadd_rn(acc, __fmul_rn(eb, o));
        eb = 1.f;
      }
  } else {
    const int j = lane & 7, g = lane >> 3;
    for (int64_t kb0 = 0; kb0 < nkb; kb0 += 8) {
      const int64_t kb = kb0 + g;
      const int64_t k0 = kb * KB;
      const int64_t k1 = kb < nkb ? min(K, k0 + KB) : k0;
      const int64_t nfull = (k1 - k0) / 8 * 8;
      float l = 0.f;
      int64_t d = 0;
      if (nfull == KB) {
        // A whole 512-deep block: all 64 of the lane's operand pairs are
        // loaded before its chain runs (one memory round trip instead of one
        // per 64 k); the same fma order as the loop below.
        float av[64], bv[64];
#pragma unroll
        for (int u = 0; u < 64; u++) {
          av[u] = a[k0 + 8 * u + j];
          bv[u] = col[k0 + 8 * u + j];
        }
#pragma unroll
        for (int u = 0; u < 64; u++) l = __fmaf_rn(av[u], bv[u], l);
        d = KB;
      }
      for (; d + 64 <= nfull; d += 64) {
        float av[8], bv[8];
#pragma unroll
        for (int t = 0; t < 8; t++) {
          av[t] = a[k0 + d + 8 * t + j];
          bv[t] = col[k0 + d + 8 * t + j];
        }
#pragma unroll
        for (int t = 0; t < 8; t++) l = __fmaf_rn(av[t], bv[t], l);
      }
      for (; d < nfull; d += 8) l = __fmaf_rn(a[k0 + d + j], col[k0 + d + j], l);
      l = __fadd_rn(l, __shfl_xor(l, 4));
      l = __fadd_rn(l, __shfl_xor(l, 2));
      float acc = __fadd_rn(l, __shfl_xor(l, 1));
      if (j == 0)
        for (int64_t k = k0 + nfull; k < k1; k++) acc = __fmaf_rn(a[k], col[k], acc);
      const int nb = (int)(nkb - kb0 < 8 ? nkb - kb0 : 8);
      for (int q = 0; q < nb; q++) {
        const float r = __shfl(acc, q * 8);
        o = eb == 0.f ? __fmul_rn(alpha, r) : __fadd_rn(__fmul_rn(alpha, r), __fmul_rn(eb, o));
        eb = 1.f;
      }
    }
  }
  if (lane == 0) {
    if (bias) o = __fadd_rn(o, bias[0]);
    out[c] = o;
  }
}

__global__ __launch_bounds__(256) void gemv_t_kernel(int64_t N, int64_t K,
                                                     const float* __restrict__ a,
                                                     const float* __restrict__ b, int64_t b_cs,
                                                     float* __restrict__ out, float alpha,
                                                     float beta, const float* __restrict__ bias,
                                                     int64_t bbs, const float* __restrict__ cin,
                                                     int64_t cin_stride) {
  const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= N) return;  // whole wave
  gemv_t_column(c, N, K, a, b, b_cs, out, alpha, beta, bias, bbs, cin, cin_stride);
}

rtenhip_status launch_gemv(int64_t N, int64_t K, const float* a, const float* b, int64_t b_rs,
                           int64_t b_cs, float* out, float alpha, float beta, const float* bias,
                           int64_t ref_threads, hipStream_t s, const float* cin, int64_t cin_stride) {
  // Column blocks (gemm.rs:673): b_block_size = max(ceil(N / threads), 128).
  // Which columns fall in a chunk's partial 8/32-wide tile depends on it,
  // so the reference's thread count (RTEN_NUM_THREADS semantics) is a
  // parameter of the numerics here, exactly as it is for RTen.
  int64_t t = ref_threads > 0 ? ref_threads : 1;
  int64_t bbs = (N + t - 1) / t;
  if (bbs < 128) bbs = 128;
  if (N <= 0) return RTENHIP_OK;
  if (b_rs == 1) {
    hipLaunchKernelGGL(gemv_t_kernel, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, s, N, K, a, b,
                       b_cs, out, alpha, beta, bias, bbs, cin, cin_stride);
    RTENHIP_LAUNCH_CHECK();
    return RTENHIP_OK;
  }
  hipLaunchKernelGGL(gemv_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, N, K, a, b,
                     b_rs, b_cs, out, alpha, beta, bias, bbs, cin, cin_stride);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

}  // namespace rtenhip
