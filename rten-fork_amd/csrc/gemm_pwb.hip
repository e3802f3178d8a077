// Pointwise-conv GEMM with the B panel held in LDS ("B-stationary"): latency
// GEMM variants 61 / 62 / 64 (launch_gemm_lat), for 1x1 convs with K <= 256
// (one KC block) at large batch -- ResNet-50's layer1-3 conv1 / conv3 at
// batch 64, MobileNetV2's expand / project convs.
//
// Those convs are short-K: 16..64 MFMA steps per output tile.  The DMA GEMM
// streams A and B through a K-stage LDS ring per 64x64 tile, so every tile
// pays the ring's fill, one barrier per K stage and an LDS-staged epilogue
// for a handful of MFMA steps, and B (the activations, the large operand) is
// fetched again for every 64-row tile of the output.  Here a workgroup
//   1. copies the B panel of its 64 output columns -- all K rows -- into LDS
//      once (K x 64 floats, zero past K), one barrier;
//   2. walks MR chunks of 64 output rows: each wave owns 16 rows x the 64
//      columns (four v_mfma_f32_16x16x4_f32 chains sharing the A operand),
//      A comes straight from global memory in the latency GEMM's packing
//      (launch_pack_lat: a lane's 4 MFMA steps are one float4) and the next
//      chunk's A is in flight while this chunk's chains run; B is read from
//      LDS as one 16-byte read per step ([k][column % 16][column / 16]);
//   3. finishes each 16x16 tile with lat_unit.h's epilogue (bias, column
//      bias, BatchNormalization, residual, activation, strided / zero-bordered
//      outputs) -- no barriers after the copy.
// Summation contract as the latency GEMM's (lat_unit.h): one chain per
// element from +0 over k in order (K <= 256: a single KC block), then
// alpha * chain + bias and the rest of the epilogue -- bit-identical to every
// other configuration of the conv.
#include "gemm_dma_kernel.h"  // LDS-DMA helpers
#include "lat_unit.h"

namespace rtenhip {

constexpr int kPwbCols = 64;  // output columns per workgroup

// Grid: 8 * m_ranges * ceil(n_tiles / 8) workgroups; block b runs on XCD
// b % 8 (round-robin dispatch), and its work id o = b / 8 enumerates
// (column tile group, row range) with the row range fastest, so the row
// ranges of one column tile run back to back on ONE XCD and its B panel is
// read from HBM once and from that XCD's L2 after.
template <int MR>
__global__ __launch_bounds__(256, 2) void gemm_pwb_kernel(DmaDesc d, int m_ranges, int n_tiles, int subs) {
  extern __shared__ float bl[];  // [kpad][16][4]: k row, column % 16, column / 16
  const int b = blockIdx.x;
  const int o = b >> 3;
  const int mr = o % m_ranges;
  const int nt = (o / m_ranges) * 8 + (b & 7);
  if (nt >= n_tiles) return;  // whole workgroup: no barrier reached
  const int n0 = nt * kPwbCols;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int K = d.K;
  const int ng = (K + 15) >> 4;  // 16-k groups (4 MFMA steps each)

  // 1. B panel, by LDS DMA (buffer_load_dword ... lds: lane l of the
  // instruction writes LDS word m0 / 4 + l, so no VGPR holds the panel).
  // Copy lane l fetches column (l % 4) * 16 + l / 4, so LDS row k is
  // [column % 16][column / 16]; wave w copies rows w, w + 4, ...  Rows past K
  // and columns past N read 0 (DMA_OOB).  Every copy is issued before the
  // one wait.
  {
    const int col = (lane & 3) * 16 + (lane >> 2);
    const int n = n0 + col;
    uint32_t vcol = DMA_OOB;
    if (n < d.N) {
      const int img = fdiv(n, d.fdP);
      const int p = n - img * d.P;
      const int oy = fdiv(p, d.fdOW);
      const int ox = p - oy * d.OW;
      vcol = (uint32_t)(((int64_t)img * d.x_img + (int64_t)oy * d.ystride + (int64_t)ox * d.xstride) * 4);
    }
    const u32x4 xr = make_rsrc(d.x, d.x_bytes);
    const uint32_t kstep = (uint32_t)d.kstride * 4u;
    const uint32_t l0 = lds_addr(bl);
    const int rows = ng * 16;
    for (int k = wave; k < rows; k += 4)
      lds_dma4(xr, l0 + (uint32_t)k * 256u, (k < K && vcol != DMA_OOB) ? vcol + (uint32_t)k * kstep : DMA_OOB, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();

  // 2. Row chunks.  Wave w of chunk q owns 16-row subtile (mr * MR + q) * 4 + w.
  typedef unsigned int pwb_u32x4 __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t ar =
      __builtin_amdgcn_make_buffer_rsrc((void*)d.apk, 0, (int)((int64_t)subs * LGROUPS * 64 * 16), 0x00020000);
  auto load_a = [&](int sub, pwb_u32x4 (&av)[LGROUPS]) {
#pragma unroll
    for (int g = 0; g < LGROUPS; g++) {
      const uint32_t off = (sub < subs && g < ng) ? (uint32_t)(((sub * LGROUPS) + g) * 64 + lane) * 16u : DMA_OOB;
      av[g] = __builtin_amdgcn_raw_buffer_load_b128(ar, off, 0, 0);
    }
  };
  LatCol cols[4];
#pragma unroll
  for (int ct = 0; ct < 4; ct++) cols[ct] = lat_col(d, n0 + ct * 16);
  const int h = lane >> 4, c = lane & 15;
  const float* brow = bl + h * 64 + c * 4;  // step s reads row 4s + h

  pwb_u32x4 av[LGROUPS], an[LGROUPS];
  load_a((mr * MR) * 4 + wave, av);
#pragma unroll
  for (int q = 0; q < MR; q++) {
    const int sub = (mr * MR + q) * 4 + wave;
    if (sub >= subs) break;  // wave-uniform; nothing after this waits on other waves
    if (q + 1 < MR) load_a(sub + 4, an);
    LatEpi<1> e[4];
#pragma unroll
    for (int ct = 0; ct < 4; ct++) lat_epi_loads<1>(d, sub, cols[ct], e[ct]);
    lat_f32x4 acc[4];
#pragma unroll
    for (int ct = 0; ct < 4; ct++) acc[ct] = (lat_f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < LGROUPS; g++) {
      if (g < ng) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const float4 bv = *reinterpret_cast<const float4*>(brow + (16 * g + 4 * j) * 64);
          const float a = __uint_as_float(av[g][j]);
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv.x, acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv.y, acc[1], 0, 0, 0);
          acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv.z, acc[2], 0, 0, 0);
          acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv.w, acc[3], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int ct = 0; ct < 4; ct++) {
      lat_f32x4 sum[1];
#pragma unroll
      for (int r = 0; r < 4; r++) sum[0][r] = lat_first_block(d, acc[ct][r], e[ct].bias[0][r]);
      lat_finish<1>(d, sub, cols[ct], e[ct], sum);
    }
    if (q + 1 < MR) {
#pragma unroll
      for (int g = 0; g < LGROUPS; g++) av[g] = an[g];
    }
  }
}

bool pwb_ok(const DmaDesc& d) { return d.kstride > 0 && !d.k3x3 && d.K >= 1 && d.K <= LKC && !d.cin; }

rtenhip_status launch_gemm_pwb(const DmaDesc& d, int mr, hipStream_t s) {
  if (!pwb_ok(d)) return fail(RTENHIP_UNSUPPORTED_VALUE, "B-stationary pointwise GEMM: 1x1 convs with K <= 256 only");
  const int subs = (d.M + 15) / 16;
  const int chunks = (subs + 3) / 4;
  const int m_ranges = (chunks + mr - 1) / mr;
  const int n_tiles = (d.N + kPwbCols - 1) / kPwbCols;
  const int64_t wgs = 8LL * m_ranges * ((n_tiles + 7) / 8);
  if (wgs > 0x7fffffff) return fail(RTENHIP_UNSUPPORTED_VALUE, "B-stationary pointwise GEMM grid too large");
  const size_t lds = (size_t)((d.K + 15) / 16) * 16 * 64 * 4;
  const dim3 grid((unsigned)wgs), blk(256);
  switch (mr) {
    case 1: hipLaunchKernelGGL((gemm_pwb_kernel<1>), grid, blk, lds, s, d, m_ranges, n_tiles, subs); break;
    case 2: hipLaunchKernelGGL((gemm_pwb_kernel<2>), grid, blk, lds, s, d, m_ranges, n_tiles, subs); break;
    case 4: hipLaunchKernelGGL((gemm_pwb_kernel<4>), grid, blk, lds, s, d, m_ranges, n_tiles, subs); break;
    default: return fail(RTENHIP_INVALID_VALUE, "B-stationary pointwise GEMM: chunks per workgroup must be 1, 2 or 4");
  }
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

}  // namespace rtenhip
