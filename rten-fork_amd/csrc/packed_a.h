// The dense GEMM's packed-A layout (pack_a_kernel, gemm_dma.hip) as a store
// target for producers of a MatMul's A operand (Plan::pk_cons): a tile of BM
// rows x BK k is [BK/4][BM][4] floats, float (q * BM + r) * 4 + j holding row
// r, k = 8 * (q >> 1) + 2 * j + (q & 1); tiles are [tiles_m][tiles_k].
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace rtenhip {

struct PackedOut {
  float* p = nullptr;  // zero-initialised buffer of the consumer's packed_a_floats(M, K, tile)
  int lbm = 0, lbk = 0, tiles_k = 0;  // log2 BM, log2 BK (>= 3), tiles along K
};

// Row m, k = n .. n + 3 (n % 4 == 0): k-quad planes q = 2g (k even) and
// 2g + 1 (k odd), slots j = 2u, 2u + 1 -- two 8-byte stores.
__device__ __forceinline__ void store_packed_a4(float* pk, int lbm, int lbk, int tiles_k, int64_t m, int n,
                                                float4 x) {
  const int kk = n & ((1 << lbk) - 1);
  const int q0 = 2 * (kk >> 3), u = (kk >> 2) & 1;
  const int r = (int)(m & ((1 << lbm) - 1));
  float* tb = pk + (((m >> lbm) * tiles_k + (n >> lbk)) << (lbm + lbk));
  *(float2*)(tb + (((int64_t)q0 << lbm) + r) * 4 + 2 * u) = make_float2(x.x, x.z);
  *(float2*)(tb + (((int64_t)(q0 + 1) << lbm) + r) * 4 + 2 * u) = make_float2(x.y, x.w);
}

}  // namespace rtenhip
