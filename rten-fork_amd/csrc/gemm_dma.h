// LDS-DMA GEMM fast path (gemm_dma.hip).
#pragma once

#include "common.h"

namespace rtenhip {

// Buffer offset past num_records: the hardware returns 0 for such loads.
constexpr uint32_t DMA_OOB = 0x80000000u;
// K tables are padded with DMA_OOB entries to a multiple of this (>= any BK).
constexpr int DMA_KTAB_PAD = 64;

// Tile shape of a DMA launch.  A is packed per tile as [bk][bm] with the rows
// of each wave's 32*il-row slab interleaved (row mi*32+l -> position l*il+mi)
// so a lane reads its il A values with one LDS instruction.
struct DmaTile {
  int bm, bk, il;
  bool operator==(const DmaTile& o) const { return bm == o.bm && bk == o.bk && il == o.il; }
};

// C[M,N] = epilogue(alpha * A @ B) with
//   A: packed [tiles_m][tiles_k][bk][bm] (launch_pack_a, interleaved by il),
//   B[k][n] = x[colbase(n) + koff(k)] with no bounds checks, where for
//     n = img*P + oy*OW + ox:  colbase = img*x_img + oy*ystride + ox*xstride
//     and koff = ktab4[k] / 4 (ktab4 holds byte offsets, DMA_OOB past K,
//     padded to a multiple of DMA_KTAB_PAD entries),
//   out index  = img*out_img + m*out_c + oy*out_row + ox + out_off,
//   residual   = img*res_img + m*res_c + (oy*OW + ox).
struct DmaDesc {
  int M, N, K;
  DmaTile tile;             // tile shape A was packed for
  const float* apk;
  const float* x;
  uint32_t x_bytes;         // buffer size in bytes (num_records)
  int64_t x_img;
  int64_t ystride, xstride;
  int OW, P;
  FastDiv fdOW, fdP;        // divisors OW and P
  const int* ktab4;
  float* out;
  int64_t out_img, out_c, out_row, out_off;
  const float* residual;
  int64_t res_img, res_c;
  const float* bias;
  const float* colbias;     // per-column bias colbias[p] (p = oy*OW + ox), added after the
                            // K fold and before the residual (MatMul -> Add(bias[N]))
  const float* cin;         // beta != 0 (dense outputs only; out_c = row stride)
  // Conv -> BatchNormalization (Graph::optimize): per output row m, after the
  // K fold and the bias and before the residual, x = (x - bn[m]) * bn[bn_c + m]
  // + bn[2 * bn_c + m] -- mean, scale / sqrt(var + eps), beta
  // (batch_norm_in_place, src/ops/norm.rs:45-49); null otherwise.
  const float* bn;
  int bn_c;
  float alpha, beta;
  int act;
  float act_lo, act_hi;
  // KC split of the last split_tiles tiles (0 = none): nkb K blocks each,
  // chains in ws (split_tiles * nkb * BM*BN floats), arrival counters
  // (split_tiles ints, zero between launches; the kernel re-zeroes them).
  int split_tiles, nkb;
  float* ws;
  int* counters;
  int n_full;               // set by launch_gemm_dma
  // Persistent launch: persist_k resident blocks per CU (0: one block per work
  // item), enforced with LDS padding so that every CU holds exactly that many;
  // items are dealt out statically per XCD (see gemm_dma_kernel).
  int persist_k;
  // Tile order (0: m tile fastest).  swz > 0: strips of swz tile columns, the
  // tiles of a strip row by row (n fastest within the strip), so a run of
  // consecutive tiles -- what one XCD's resident blocks work on together --
  // is a compact block of A rows and B columns in that XCD's L2.
  int swz;
  // Dual GEMM (set by launch_gemm_dma): 1 = one continuous K loop over both
  // segments (segment 2's first tiles stream in while segment 1 finishes),
  // 0 = two passes with a drain between them.
  int dual_one;
  int bvec;                 // B copied 16 bytes per lane (dma_cfg_bvec(cfg) and pointwise:
                            // koff(k) = k * kstride, P % 4 == 0, K % BK == 0)
  int kstride;              // elements between consecutive k rows of B (bvec)
  int vec4;                 // outputs/residual row-contiguous with P % 4 == 0, unpadded:
                            // 16-byte epilogue accesses (no cin)
  // Dense MatMul whose output is the next MatMul's A: the vectorised
  // epilogue stores the values in that MatMul's packed-A layout
  // ([tiles_m][tiles_k][BK/4][BM][4] k-quads, see pack_a_kernel) at pk_out
  // instead of row-major at out (column n = that MatMul's k, row m its row).
  float* pk_out;
  int pk_lbm, pk_lbk, pk_tiles_k;  // log2 BM, log2 BK and tiles_k of the consumer's packing
  int k3x3;                 // latency GEMM: 3x3 window, koff(k) computed from k = 9c + 3ky + kx
  int kt_plane, kt_row, kt_col;  // ... as c * kt_plane + ky * kt_row + kx * kt_col (elements)
  int dbg;                  // tuning experiments only: 1 = no K-loop DMA, 2 = no MFMA
  unsigned long long* stamps;  // placement experiment builds only (RTENHIP_DMA_EXPERIMENT 5):
                               // per block {hw ids, start, end, block}; null otherwise
};

// KC split plan for one configuration (split_tiles == 0: not worth it).
struct DmaSplit {
  int split_tiles, nkb;
  int64_t ws_floats, counters;
};
DmaSplit dma_split_plan(int M, int N, int K, int cfg);

// Tile order of dense MatMul DMA GEMMs (DmaDesc::swz; gemm_dma.hip).
int dma_dense_swz(int64_t K, int BN);

// Kernel configurations (all bit-identical; see gemm_dma.hip).
int dma_num_cfgs();
bool dma_cfg_bvec(int cfg);
// Whether cfg's kernel has the vectorised (LDS-transposed, 16-byte) epilogue.
bool dma_cfg_vec_epilogue(int cfg);
int dma_default_cfg(int M, int N, int K);
DmaTile dma_cfg_tile(int cfg);
// Tile width (BN) of DMA configuration cfg.
int dma_cfg_info_bn(int cfg);
int64_t packed_a_floats(int M, int K, const DmaTile& t);
rtenhip_status launch_pack_a(const float* a, int64_t lda, int M, int K, const DmaTile& t,
                             float* out, hipStream_t s);
// d2: dual GEMM (gemm_dma_kernel DUAL) -- d2's folded values are added to
// d's in d's epilogue (d2 = ResNet's downsample conv, d = conv3).
rtenhip_status launch_gemm_dma(const DmaDesc& d, int cfg, hipStream_t s, const DmaDesc* d2 = nullptr);
bool dma_cfg_dual(int cfg);

// Latency GEMM (gemm_lat.hip): the same DmaDesc addressing and summation
// order, one wave per 16x16 output tile and KC block (small-batch convs).
// variant = 10 * (waves along M: 1, 2, 4) + (16-row tiles per wave: 1, 2),
// 71 / 72 / 74 for the LDS-staged kernel (RW = v - 70 rows x 4 / RW columns),
// 61 / 62 / 63 / 66 for the slab kernel (RW x CW = 1x4, 2x4, 1x8, 2x8;
// gemm_lat4_kernel: one image, a KC block's input planes staged in LDS),
// 85 / 86 for its pipelined 8-wave form (RW x CW = 2x4 / 4x2;
// gemm_lat3_kernel), or 90 + (16-row tiles per wave) for the workgroup-fold
// kernel;
// A packed by launch_pack_lat; kstride > 0 selects koff(k) = k * kstride
// (no K table); with K > 256, ws / counters sized by lat_split_plan.
bool lat_variant_ok(int variant);
int64_t lat_packed_floats(int M, int K);
rtenhip_status launch_pack_lat(const float* a, int64_t lda, int M, int K, float* out, hipStream_t s);
DmaSplit lat_split_plan(int M, int N, int K, int variant);
rtenhip_status launch_gemm_lat(const DmaDesc& d, int variant, hipStream_t s);
// Two latency GEMMs in one launch (LDS-staged variants 71 / 72 / 74; d0 with
// 16-byte B copies): the bits of the two launches apart.
bool lat_pair_variants_ok(int v0, int v1);
rtenhip_status launch_gemm_lat_pair(const DmaDesc& d0, int v0, const DmaDesc& d1, int v1, hipStream_t s);

}  // namespace rtenhip
