#include <algorithm>
// Host side of the LDS-DMA GEMM (kernel template: gemm_dma_kernel.h; the
// tile configurations are instantiated in gemm_dma_p*.hip): configuration
// table, default choice, KC split plan, launch dispatch, and the A pack
// kernel.
#include "gemm_dma_kernel.h"

namespace rtenhip {

struct DmaCfgInfo {
  int nt, bm, bn, bk, waves_m, waves_n;
};
static const DmaCfgInfo kDmaCfgs[] = {
#define RTENHIP_DMA_INFO(id, NT, BM, BN, BK, WMW, WNW, MINW, ST, HD) {NT, BM, BN, BK, WMW, WNW},
    RTENHIP_DMA_CONFIGS(RTENHIP_DMA_INFO)
#undef RTENHIP_DMA_INFO
};
constexpr int kNumDmaCfgs = sizeof(kDmaCfgs) / sizeof(kDmaCfgs[0]);
static int g_dma_cfg = -1;
static int g_dma_dbg = 0;
static unsigned long long* g_dma_stamps = nullptr;
static int g_dma_persist = -1;  // debug override of DmaDesc::persist_k (-1: none)

int dma_num_cfgs() { return kNumDmaCfgs; }

bool dma_cfg_bvec(int cfg) {
  switch (cfg) {
#define RTENHIP_DMA_BV(id, NT, BM, BN, BK, WMW, WNW, MINW, ST, HD) \
  case id:                                                  \
    return dma_bvec_ok<NT, BM, BN, BK, WMW, WNW>();
    RTENHIP_DMA_CONFIGS(RTENHIP_DMA_BV)
#undef RTENHIP_DMA_BV
    default:
      return false;
  }
}

bool dma_cfg_dual(int cfg) {
  switch (cfg) {
#define RTENHIP_DMA_DU(id, NT, BM, BN, BK, WMW, WNW, MINW, ST, HD) \
  case id:                                                  \
    return dma_dual_ok<NT, BM, BN, BK, WMW, WNW>();
    RTENHIP_DMA_CONFIGS(RTENHIP_DMA_DU)
#undef RTENHIP_DMA_DU
    default:
      return false;
  }
}

bool dma_cfg_vec_epilogue(int cfg) {
  switch (cfg) {
#define RTENHIP_DMA_VE(id, NT, BM, BN, BK, WMW, WNW, MINW, ST, HD) \
  case id:                                                  \
    return (NT / 64) * 1024 <= ST * (BM + BN) * BK;
    RTENHIP_DMA_CONFIGS(RTENHIP_DMA_VE)
#undef RTENHIP_DMA_VE
    default:
      return false;
  }
}

int dma_cfg_info_bn(int cfg) { return cfg >= 0 && cfg < kNumDmaCfgs ? kDmaCfgs[cfg].bn : 64; }

DmaTile dma_cfg_tile(int cfg) {
  const DmaCfgInfo& c = kDmaCfgs[cfg];
  return DmaTile{c.bm, c.bk, 1};  // k-quad layout, independent of the wave tile
}

int dma_default_cfg(int M, int N, int K) {
  (void)K;
  if (g_dma_cfg >= 0 && g_dma_cfg < kNumDmaCfgs) return g_dma_cfg;
  // Largest tile that still gives every CU about two blocks.
  auto tiles = [&](int c) {
    return (int64_t)((M + kDmaCfgs[c].bm - 1) / kDmaCfgs[c].bm) *
           ((N + kDmaCfgs[c].bn - 1) / kDmaCfgs[c].bn);
  };
  if (M <= 64) return tiles(2) >= 512 ? 2 : (tiles(4) >= 512 ? 4 : 7);
  if (tiles(1) >= 512) return 1;
  if (tiles(3) >= 512) return 3;
  return 7;
}

DmaSplit dma_split_plan(int M, int N, int K, int cfg) {
  DmaSplit sp{0, 0, 0, 0};
  const DmaCfgInfo& c = kDmaCfgs[cfg];
  const int tiles = ((M + c.bm - 1) / c.bm) * ((N + c.bn - 1) / c.bn);
  const int nkb = (K + DKC - 1) / DKC;
  if (nkb < 2) return sp;
  // Whole tiles fill complete rounds of one tile per CU; the remainder would
  // run as a partial round, so it is split into KC blocks.
  constexpr int CUS = 256;
  const int rem = tiles % CUS;
  if (rem == 0) return sp;
  sp.split_tiles = rem;
  sp.nkb = nkb;
  sp.ws_floats = (int64_t)rem * nkb * c.bm * c.bn;
  sp.counters = rem;
  return sp;
}

// Tile order of dense MatMul DMA GEMMs (DmaDesc::swz): strips of g tile
// columns, n fastest within a strip, so a strip's B columns (g * BN * K
// floats) stay in the XCD's L2 while its tiles walk down the rows.
// RTENHIP_DMA_SWZ_MM=g fixes g for every GEMM; RTENHIP_DMA_SWZ_MM=-b sizes
// the strip per GEMM to at most b KiB of B (A/B experiments).  Default 8.
int dma_dense_swz(int64_t K, int BN) {
  static const int v = [] { const char* e = getenv("RTENHIP_DMA_SWZ_MM"); return e ? atoi(e) : 8; }();
  if (v >= 0) return v;
  const int64_t per_col = (int64_t)BN * K * 4;
  const int64_t g = ((int64_t)-v * 1024) / (per_col > 0 ? per_col : 1);
  return (int)std::max<int64_t>(1, std::min<int64_t>(16, g));
}

rtenhip_status launch_gemm_dma(const DmaDesc& d, int cfg, hipStream_t s, const DmaDesc* d2) {
  if (d.M <= 0 || d.N <= 0 || d.K <= 0) return fail(RTENHIP_INVALID_VALUE, "empty DMA GEMM");
  if (cfg < 0 || cfg >= kNumDmaCfgs) return fail(RTENHIP_INVALID_VALUE, "unknown DMA config");
  if (!(dma_cfg_tile(cfg) == d.tile))
    return fail(RTENHIP_INVALID_VALUE, "A packed for another tile shape");
  if (d.pk_out && (!d.vec4 || !dma_cfg_vec_epilogue(cfg) || d.P != d.N || d.pk_lbk < 3))
    return fail(RTENHIP_INVALID_VALUE, "packed-A output needs the vectorised epilogue of a dense GEMM");
  DmaDesc dd = d;
  dd.dbg = g_dma_dbg;
  dd.stamps = g_dma_stamps;
  if (g_dma_persist >= 0) dd.persist_k = g_dma_persist;
  {
    // Tile order (DmaDesc::swz).  Dense MatMuls run in strips of 8 tile
    // columns: BERT-base b32 +1.4% in an interleaved
    // A/B (4,925 / 4,916 -> 4,992 / 4,984 seq/s; strips of 4: +1%); the conv
    // GEMMs keep the m-fastest order (ResNet-50 b64 strips of 8: -0.3%)
    // (profiles/r4_tile_order_ab.txt).  Experiments: RTENHIP_DMA_SWZ=g for
    // every DMA GEMM, RTENHIP_DMA_SWZ_MM=g for the dense ones (0: m fastest).
    // (The dense-MatMul order is set by gemm_dense_dma, dma_dense_swz.)
    static const int swz_all = [] { const char* e = getenv("RTENHIP_DMA_SWZ"); return e ? atoi(e) : -1; }();
    if (swz_all >= 0) dd.swz = swz_all;
  }
  const DmaCfgInfo& ci = kDmaCfgs[cfg];
  const int tiles = ((d.M + ci.bm - 1) / ci.bm) * ((d.N + ci.bn - 1) / ci.bn);
  if (d.split_tiles > 0) {
    if (d.K <= DKC || !d.ws || !d.counters || d.split_tiles > tiles ||
        d.nkb != (d.K + DKC - 1) / DKC)
      return fail(RTENHIP_INVALID_VALUE, "bad DMA split");
    dd.n_full = tiles - d.split_tiles;
  } else {
    dd.n_full = tiles;
  }
  DmaDesc dd2{};
  if (d2) {
    // Dual GEMM: same output tiles, no KC split, both segments through the
    // multi-block fold with 4-byte B copies.
    if (d2->M != d.M || d2->N != d.N || d2->K <= 0 || !(d2->tile == d.tile) || d.split_tiles || d.residual ||
        d.cin || d2->cin || d.pk_out)
      return fail(RTENHIP_INVALID_VALUE, "bad dual DMA GEMM");
    dd2 = *d2;
    dd2.dbg = dd.dbg;
    dd2.n_full = dd.n_full;
    dd2.swz = dd.swz;  // both segments walk the same tiles
    // One K loop needs segment 1 to end on an even tile (register-set
    // parity) with no partial tile.  RTENHIP_DMA_DUAL1=0: two passes.
    // (read per launch, so tests can cover both forms in one process)
    const char* dual1_env = getenv("RTENHIP_DMA_DUAL1");
    const int dual1 = dual1_env ? atoi(dual1_env) : 1;
    dd.dual_one = dual1 && d2->K % (2 * ci.bk) == 0;
    // 16-byte B copies only when both segments allow them, in one K loop
    // (otherwise both take 4-byte copies, always valid).
    if (!(dd.bvec && dd2.bvec && dd.dual_one && dma_cfg_bvec(cfg))) dd.bvec = dd2.bvec = 0;
  }
  bool launched = false;
  const DmaDesc* p2 = d2 ? &dd2 : nullptr;
  switch (cfg % DMA_PARTS) {
    case 0: launched = dma_launch_part<0>(cfg, dd, s, p2); break;
    case 1: launched = dma_launch_part<1>(cfg, dd, s, p2); break;
    case 2: launched = dma_launch_part<2>(cfg, dd, s, p2); break;
    default: launched = dma_launch_part<3>(cfg, dd, s, p2); break;
  }
  if (!launched) return fail(RTENHIP_INVALID_VALUE, d2 ? "DMA config has no dual instance" : "unknown DMA config");
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

}  // namespace rtenhip

extern "C" void rtenhip_debug_set_dma_config(int cfg) { rtenhip::g_dma_cfg = cfg; }
extern "C" void rtenhip_debug_set_dma_mode(int mode) { rtenhip::g_dma_dbg = mode; }
// Placement experiment builds only: device buffer of 4 u64 per block.
extern "C" void rtenhip_debug_set_dma_persist(int k) { rtenhip::g_dma_persist = k; }
extern "C" void rtenhip_debug_set_dma_stamps(void* buf) {
  rtenhip::g_dma_stamps = static_cast<unsigned long long*>(buf);
}

namespace rtenhip {

// Pack A[M, K] (row stride lda, unit column stride) into
// [tiles_m][tiles_k][BK/4][BM][4] tiles, zero padded: within a tile, float
// (q * BM + r) * 4 + j holds row r, k = 8 * (q >> 1) + 2 * j + (q & 1), so
// the lane owning row r and k parity (q & 1) reads the A operands of 4
// consecutive 32x32x2 MFMA steps with one ds_read_b128.  One workgroup per
// (RB-row slice of an m tile, kcw-wide k chunk): the RB rows are read as
// kcw*4-byte segments (float4 per lane when aligned), transposed through LDS,
// and written as RB*16-byte runs (one per tile and q) with float4 stores.
// RB < BM lets kcw grow (longer row segments per read) at the same
// workgroup count.

__global__ __launch_bounds__(256) void pack_a_kernel(const float* __restrict__ a, int64_t lda,
                                                     int M, int K, int lbm, int lbk,
                                                     int tiles_k, int lkcw, int lrb, int vec,
                                                     float* __restrict__ out) {
  extern __shared__ float sh[];  // [kcw][RB + 1]
  const int BM = 1 << lbm, BK = 1 << lbk, kcw = 1 << lkcw, RB = 1 << lrb;
  const int ld = RB + 1;
  const int lsub = lbm - lrb;
  const int mt = blockIdx.x >> lsub, rs = blockIdx.x & ((1 << lsub) - 1);
  const int kc = blockIdx.y;
  const int k0 = kc * kcw;
  const int64_t m0 = (int64_t)mt * BM + (int64_t)rs * RB;
  // RB rows x kcw/4 float4s: 1..8 per thread (a multiple of 256 in total),
  // all loads issued before the LDS stores.
  const int lq4 = lkcw - 2;
  const int per = (RB << lq4) >> 8;
  float4 v[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (j < per) {
      const int idx = threadIdx.x + j * 256;
      const int r = idx >> lq4, c = (idx & ((1 << lq4) - 1)) * 4;
      const int64_t m = m0 + r;
      const int k = k0 + c;
      if (m < M) {
        const float* src = a + m * lda + k;
        if (vec && k + 3 < K) {
          v[j] = *(const float4*)src;
        } else {
          if (k < K) v[j].x = src[0];
          if (k + 1 < K) v[j].y = src[1];
          if (k + 2 < K) v[j].z = src[2];
          if (k + 3 < K) v[j].w = src[3];
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; j++)
    if (j < per) {
      const int idx = threadIdx.x + j * 256;
      const int r = idx >> lq4, c = (idx & ((1 << lq4) - 1)) * 4;
      sh[(c + 0) * ld + r] = v[j].x;
      sh[(c + 1) * ld + r] = v[j].y;
      sh[(c + 2) * ld + r] = v[j].z;
      sh[(c + 3) * ld + r] = v[j].w;
    }
  __syncthreads();
  const int kt0 = k0 / BK;
  const int nkt = min(kcw / BK, tiles_k - kt0);
  float* o = out + ((int64_t)mt * tiles_k + kt0) * (int64_t)(BK * BM) + (int64_t)rs * RB * 4;
  const int lq = lbk - 2;            // log2(BK / 4): q values per tile
  const int n4 = (nkt << lq) << lrb;  // float4 runs to write
  for (int i4 = threadIdx.x; i4 < n4; i4 += 256) {
    const int tq = i4 >> lrb, rl = i4 & (RB - 1);
    const int t = tq >> lq, q = tq & ((1 << lq) - 1);
    const int kb = t * BK + 8 * (q >> 1) + (q & 1);  // k of j = 0, within the chunk
    *(float4*)(o + (int64_t)t * (BK * BM) + ((int64_t)q * BM + rl) * 4) =
        make_float4(sh[kb * ld + rl], sh[(kb + 2) * ld + rl], sh[(kb + 4) * ld + rl],
                    sh[(kb + 6) * ld + rl]);
  }
}

int64_t packed_a_floats(int M, int K, const DmaTile& t) {
  const int64_t tm = (M + t.bm - 1) / t.bm, tk = (K + t.bk - 1) / t.bk;
  return tm * tk * t.bm * t.bk;
}

rtenhip_status launch_pack_a(const float* a, int64_t lda, int M, int K, const DmaTile& t,
                             float* out, hipStream_t s) {
  const int tiles_k = (K + t.bk - 1) / t.bk;
  const int tiles_m = (M + t.bm - 1) / t.bm;
  if ((int64_t)tiles_m * tiles_k == 0) return RTENHIP_OK;
  // Workgroups of RB rows x kcw columns, at least one float4 per thread
  // (RB * kcw / 4 >= 256): RB = min(BM, 32) with kcw widened towards 64 while
  // K allows, so each row is read as >= 128-byte segments; narrow chunks
  // give many workgroups, so reads and writes overlap across them.
  static const int env_rb = [] {
    const char* e = getenv("RTENHIP_PACK_RB");  // tuning experiments
    return e ? atoi(e) : 0;
  }();
  int rb = env_rb > 0 ? env_rb : std::min(t.bm, 32);
  if (rb > t.bm || (rb & (rb - 1)) != 0 || rb < 16) rb = t.bm;
  int kcw = t.bk;
  while (rb * kcw < 1024) kcw *= 2;
  while (kcw < 64 && kcw < K && rb * kcw * 2 <= 2048) kcw *= 2;
  auto pow2 = [](int v) { return v > 0 && (v & (v - 1)) == 0; };
  if (kcw % t.bk != 0 || kcw > 64 || !pow2(t.bm) || t.bm < 32 || t.bm > 256 || !pow2(t.bk) || t.bk % 8 != 0 ||
      tiles_m > 0x7fffffff)
    return fail(RTENHIP_UNSUPPORTED_VALUE, "unsupported A pack shape");
  // packed output chunks are 16-byte aligned (BK * BM % 4 == 0); float4 reads
  // need 16-byte aligned rows
  const int vec = ((uintptr_t)a % 16 == 0 && lda % 4 == 0) ? 1 : 0;
  const size_t lds = (size_t)kcw * (rb + 1) * sizeof(float);
  dim3 grid((unsigned)tiles_m * (unsigned)(t.bm / rb), (unsigned)((K + kcw - 1) / kcw));
  hipLaunchKernelGGL(pack_a_kernel, grid, dim3(256), lds, s, a, lda, M, K, __builtin_ctz(t.bm),
                     __builtin_ctz(t.bk), tiles_k, __builtin_ctz(kcw), __builtin_ctz(rb), vec, out);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

}  // namespace rtenhip
