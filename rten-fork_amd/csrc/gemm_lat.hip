// Latency GEMM for small-batch convolutions (ResNet-50 at batch 1).
//
// At batch 1 a ResNet-50 conv is 25..230 MFLOP: spread over 1024 SIMDs that
// is 0.4..1.5 us of MFMA, so the DMA GEMM's 64x64 tiles (few blocks, each
// paying an LDS-DMA prologue, 16 barriers per KC block and an LDS-staged
// epilogue) leave most of the chip idle and the launch latency-bound.  This
// kernel keeps the reference's summation contract (src/gemm.rs:733-1050, as
// the DMA kernel states it: one fma chain per output element and KC = 256
// block, starting from +0, the blocks folded in K order after the bias) and
// instead cuts the work into the smallest units MFMA allows:
//   - one wave = one 16-row x 16-column output tile of ONE KC block
//     (v_mfma_f32_16x16x4_f32 is bitwise the k-ordered fmaf chain, see
//     profiles/r2_mfma_shape_probe.txt), MI such tiles stacked along M;
//   - every operand goes straight from global memory into registers (no LDS
//     staging, no barriers in the K loop): A is pre-packed per (16 rows, KC
//     block) so a lane's 4 MFMA steps are one float4, B is gathered with
//     buffer loads whose per-lane offset is colbase(n) + koff(k) (the DMA
//     kernel's addressing: zero-bordered inputs, out-of-range reads return 0);
//   - all of a block's loads are issued before the first MFMA, so a unit
//     costs one memory round trip plus 64 MFMA steps;
//   - with K > 256 every tile's chains go to a workspace and the last KC
//     block to arrive folds them in K order (agent-scope counter), exactly
//     as the DMA kernel's split tiles do.
// Workgroups of 4 waves: WMW waves along M (sharing B) x 4/WMW along N
// (sharing A); workgroup ids are remapped XCD-contiguously so the units that
// share an A panel run on one XCD's L2.  Variants 91 / 92 instead keep all
// K blocks of a tile in one workgroup and fold them through LDS.
#include "lat_unit.h"

namespace rtenhip {

// Timing experiments only (rtenhip_debug_set_lat_stamps): each launch writes
// 8 u64 per wave at the next free records of this buffer.
static unsigned long long* g_lat_stamps = nullptr;
static int64_t g_lat_stamps_cap = 0, g_lat_stamps_used = 0;
static int g_lat_seq = 0;

template <int WMW, int MI>
__global__ __launch_bounds__(256) void gemm_lat_kernel(DmaDesc d, int wg_m, int wg_n, int nkb, int subs) {
  constexpr int WNW = 4 / WMW;
  __shared__ uint32_t ktl[4][LKC];  // per wave: this block's k offsets, [k % 4][k / 4]
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // XCD-contiguous remap (dispatch is round-robin over the 8 XCDs): XCD x
  // owns a contiguous range of work ids, ordered (kb, tm, tn) with tn fastest.
  const int G = gridDim.x, bid = blockIdx.x;
  const int qq = G >> 3, rr = G & 7, xcd = bid & 7;
  const int o = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int tn = o % wg_n;
  const int t2 = o / wg_n;
  const int tm = t2 % wg_m;
  const int kb = t2 / wg_m;
  const int wm = wave / WNW, wn = wave - (wave / WNW) * WNW;
  const int sub0 = (tm * WMW + wm) * MI;  // first 16-row subtile of this wave
  const int n0 = (tn * WNW + wn) * 16;
  if (sub0 >= subs || n0 >= d.N) return;  // wave past the matrix edge (no counters touched)
  const int wt = (tm * WMW + wm) * (wg_n * WNW) + (n0 >> 4);
  lat_unit<MI>(d, sub0, n0, kb, nkb, subs, wt, ktl[wave]);
}

// LDS-staged variant (71 / 72 / 74): a workgroup of 4 waves computes RW x CW
// 16x16 tiles of one KC block, one chain per wave.  The RW packed A panels
// (16 rows x 256 k each) and the CW B tiles (256 k x 16 columns each) are
// staged in LDS once per workgroup -- A with 16-byte loads, B gathered by all
// 256 threads -- so a panel read from L2 / the Infinity Cache serves CW waves
// and a gathered B element RW waves (the one-wave-per-unit kernel above loads
// both once per wave).  The chains then read their operands from LDS as
// 16-byte groups in the same k order, so the bits are those of every other
// variant; the fold and the epilogue are lat_fold_finish's.
//
// BVEC (pointwise stride-1 convs with P % 4 == 0, DmaDesc::bvec): B is copied
// 16 bytes per lane -- 4 adjacent columns of one k row, inside one image --
// into a [CW][256 k][16 columns] tile, and the chains read it one float per
// MFMA step: a quarter of the gather's load instructions.
// The body of gemm_lat2_kernel for work id o (kb, tm, tn), its A panels and
// B tiles staged at lds_a / lds_b (the caller's LDS: the pair kernel below
// runs two problems' bodies over one allocation).
template <int RW, int CW, bool BVEC>
__device__ __forceinline__ void lat2_body(const DmaDesc& d, int o, int wg_m, int wg_n, int nkb, int subs,
                                          float4 (*lds_a)[LGROUPS][64], float4 (*lds_b)[LGROUPS][64]) {
  static_assert(RW * CW == 4, "one chain per wave");
  float* ldsk = reinterpret_cast<float*>(&lds_b[0][0][0]);  // BVEC: [CW][LKC][16]
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int tn = o % wg_n;
  const int t2 = o / wg_n;
  const int tm = t2 % wg_m;
  const int kb = t2 / wg_m;
  const int K = d.K;
  const int k0 = kb * LKC;
  const int ng = min(LGROUPS, (K - k0 + 15) >> 4);
  const int wr = wave / CW, wc = wave - (wave / CW) * CW;
  const int sub0 = tm * RW + wr;
  const int n0 = (tn * CW + wc) * 16;
  LatStamps stp = lat_stamps_init(d, kb, sub0, n0);

  // A: RW panels of [16 groups][64 lanes] float4 (launch_pack_lat: zero past
  // K inside a block); rows past M read past the buffer, which returns 0.
  // All loads are issued before any LDS store (one memory round trip).
  const __amdgpu_buffer_rsrc_t ar =
      __builtin_amdgcn_make_buffer_rsrc((void*)d.apk, 0, (int)((int64_t)subs * nkb * LGROUPS * 64 * 16), 0x00020000);
  typedef unsigned int lat_u32x4 __attribute__((ext_vector_type(4)));
  lat_u32x4 av[RW * 4];
#pragma unroll
  for (int i = 0; i < RW * 4; i++) {
    const int idx = (int)threadIdx.x + 256 * i;
    const int r = idx >> 10, gl = idx & 1023;
    const int sub = tm * RW + r;
    const uint32_t off = sub < subs ? (uint32_t)(((sub * nkb + kb) * LGROUPS * 64 + gl) * 16) : DMA_OOB;
    av[i] = __builtin_amdgcn_raw_buffer_load_b128(ar, off, 0, 0);
  }

  // B: thread (wave w, lane (c, h)) gathers groups 4w..4w+3 of each of the CW
  // column tiles: k = k0 + 16g + 4j + h for j = 0..3, column n0 + c.
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)d.x, 0, (int)d.x_bytes, 0x00020000);
  const int h = lane >> 4;
  const bool linear = d.kstride > 0;
  // 3x3 windows: koff(k) for k = 9c + 3ky + kx (see lat_chain); this thread
  // visits k = k0 + h + 4s for s = 16w .. 16w + 15.
  uint32_t k3off[9];
  const uint32_t k3step = 16u * (uint32_t)d.kt_plane;
  if (!linear) {
    const uint32_t kh0 = (uint32_t)(k0 + h + 64 * wave);
    const int c0 = (int)(__umulhi(kh0, 0x38E38E39u) >> 1);
    const int r0 = (int)kh0 - 9 * c0;
#pragma unroll
    for (int s9 = 0; s9 < 9; s9++) {
      const int kk = r0 + 4 * s9;
      const int q = (kk * 57) >> 9;
      const int rr2 = kk - 9 * q;
      const int ky = (rr2 * 11) >> 5;
      const int kx = rr2 - 3 * ky;
      k3off[s9] = (uint32_t)((c0 + q) * d.kt_plane + ky * d.kt_row + kx * d.kt_col) * 4u;
    }
  }
  float bv[CW][4][4];
  typedef unsigned int lat2_u32x4 __attribute__((ext_vector_type(4)));
  lat2_u32x4 bq[CW][4];
  const int q4 = threadIdx.x & 3, kr = threadIdx.x >> 2;  // BVEC: column quad, k row (+ 64 i)
  if constexpr (BVEC) {
#pragma unroll
    for (int cw = 0; cw < CW; cw++) {
      const int n = (tn * CW + cw) * 16 + 4 * q4;
      uint32_t cb = DMA_OOB;
      if (n < d.N) {
        const int img = fdiv(n, d.fdP);
        cb = (uint32_t)(((int64_t)img * d.x_img + (n - img * d.P)) * 4);
      }
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int k = k0 + kr + 64 * i;
        const uint32_t off = (k < K && cb != DMA_OOB) ? cb + (uint32_t)k * (uint32_t)d.kstride * 4u : DMA_OOB;
        bq[cw][i] = __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0);
      }
    }
  } else {
    uint32_t koff[16];
#pragma unroll
    for (int st = 0; st < 16; st++) {  // step within this thread's 16
      const int k = k0 + 64 * wave + 4 * st + h;
      const uint32_t lin = (uint32_t)k * (uint32_t)d.kstride * 4u;
      const uint32_t win = k3off[st % 9] + (uint32_t)(st / 9) * k3step;
      koff[st] = k < K ? (linear ? lin : win) : DMA_OOB;
    }
#pragma unroll
    for (int cw = 0; cw < CW; cw++) {
      const LatCol col = lat_col(d, (tn * CW + cw) * 16);
#pragma unroll
      for (int gi = 0; gi < 4; gi++)
#pragma unroll
        for (int j = 0; j < 4; j++)
          bv[cw][gi][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, col.vcol + koff[4 * gi + j], 0, 0));
    }
  }
  if (stp.p) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stp.at(9);
  }
#pragma unroll
  for (int i = 0; i < RW * 4; i++) {
    const int idx = (int)threadIdx.x + 256 * i;
    lds_a[idx >> 10][(idx >> 6) & 15][idx & 63] =
        make_float4(__uint_as_float(av[i].x), __uint_as_float(av[i].y), __uint_as_float(av[i].z), __uint_as_float(av[i].w));
  }
  if constexpr (BVEC) {
#pragma unroll
    for (int cw = 0; cw < CW; cw++)
#pragma unroll
      for (int i = 0; i < 4; i++)
        *reinterpret_cast<float4*>(ldsk + (cw * LKC + kr + 64 * i) * 16 + 4 * q4) =
            make_float4(__uint_as_float(bq[cw][i].x), __uint_as_float(bq[cw][i].y), __uint_as_float(bq[cw][i].z),
                        __uint_as_float(bq[cw][i].w));
  } else {
#pragma unroll
    for (int cw = 0; cw < CW; cw++)
#pragma unroll
      for (int gi = 0; gi < 4; gi++)
        lds_b[cw][4 * wave + gi][lane] = make_float4(bv[cw][gi][0], bv[cw][gi][1], bv[cw][gi][2], bv[cw][gi][3]);
  }

  // Epilogue operands of this wave's tile, in flight during the chain.
  const bool live = sub0 < subs && n0 < d.N;
  const LatCol col = lat_col(d, n0);
  LatEpi<1> e;
  if (live) lat_epi_loads<1>(d, sub0, col, e);
  __syncthreads();
  if (!live) return;  // (after the barrier: every wave helped stage)
  stp.at(2);

  lat_f32x4 acc[1];
  acc[0] = (lat_f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int g = 0; g < LGROUPS; g++) {
    if (g < ng) {
      const float4 a4 = lds_a[wr][g][lane];
      float4 b4;
      if constexpr (BVEC) {
        const float* bp = ldsk + (wc * LKC + 16 * g + h) * 16 + (lane & 15);
        b4 = make_float4(bp[0], bp[64], bp[128], bp[192]);  // k = 16g + 4j + h, j = 0..3
      } else {
        b4 = lds_b[wc][g][lane];
      }
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.x, b4.x, acc[0], 0, 0, 0);
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.y, b4.y, acc[0], 0, 0, 0);
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.z, b4.z, acc[0], 0, 0, 0);
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.w, b4.w, acc[0], 0, 0, 0);
    }
  }
  if (stp.p) {
    asm volatile("" ::"v"(acc[0][0]), "v"(acc[0][3]));
    stp.at(3);
  }
  const int wt = sub0 * (wg_n * CW) + (n0 >> 4);
  lat_fold_finish<1>(d, sub0, kb, nkb, wt, col, e, acc, stp);
}

// XCD-contiguous work id of this workgroup (dispatch is round-robin over the
// 8 XCDs): XCD x owns a contiguous range of work ids.
__device__ __forceinline__ int lat_xcd_work_id() {
  const int G = gridDim.x, bid = blockIdx.x;
  const int qq = G >> 3, rr = G & 7, xcd = bid & 7;
  return (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
}

template <int RW, int CW, bool BVEC>
__global__ __launch_bounds__(256) void gemm_lat2_kernel(DmaDesc d, int wg_m, int wg_n, int nkb, int subs) {
  __shared__ float4 lds_a[RW][LGROUPS][64];
  __shared__ float4 lds_b[CW][LGROUPS][64];
  lat2_body<RW, CW, BVEC>(d, lat_xcd_work_id(), wg_m, wg_n, nkb, subs, lds_a, lds_b);
}

// Two independent latency GEMMs in one launch (a bottleneck's conv1 and its
// downsample, which read the same input at batch 1): work ids below g0.wgs
// run problem 0's body, the rest problem 1's, each with its own descriptor,
// K-block workspace and fold -- the bits of the two launches apart, without
// the second launch's ramp and drain on the critical path.
struct LatPairGrid {
  int wg_m, wg_n, nkb, subs, wgs;
};
template <int RW0, int CW0, bool BV0, int RW1, int CW1, bool BV1>
__global__ __launch_bounds__(256) void gemm_lat2_pair_kernel(DmaDesc d0, LatPairGrid g0, DmaDesc d1, LatPairGrid g1) {
  constexpr int RA = RW0 > RW1 ? RW0 : RW1, RB = CW0 > CW1 ? CW0 : CW1;
  __shared__ float4 lds_a[RA][LGROUPS][64];
  __shared__ float4 lds_b[RB][LGROUPS][64];
  const int o = lat_xcd_work_id();
  if (o < g0.wgs)
    lat2_body<RW0, CW0, BV0>(d0, o, g0.wg_m, g0.wg_n, g0.nkb, g0.subs, lds_a, lds_b);
  else
    lat2_body<RW1, CW1, BV1>(d1, o - g0.wgs, g1.wg_m, g1.wg_n, g1.nkb, g1.subs, lds_a, lds_b);
}

// Pipelined LDS-staged variant (8x): the workgroup layout of gemm_lat2_kernel
// (RW x CW tiles of one KC block, one chain per wave, A panels and B tiles
// staged in LDS once per workgroup), with two changes.
//  - Phases: the block's 256 k are loaded in four phases of 64 k (4 groups),
//    every phase's loads issued up front in k order.  Phase q goes to LDS as
//    soon as its own loads have landed (vmcnt retires in issue order, so the
//    compiler's wait for phase q leaves the later phases in flight), one raw
//    s_barrier, and the chains run its 16 MFMA steps while phases q+1.. are
//    still arriving -- the operand round trip and the chain overlap instead
//    of adding (the stamps of gemm_lat2_kernel: loads 2.4-3.5 us, then the
//    chain 1.4-1.8 us).  No __syncthreads: it would drain every load.
//  - Wider workgroups: RW x CW up to 4 x 4 (64 * RW * CW threads), so a
//    panel read from L2 / the Infinity Cache serves up to 4 chains -- at
//    batch 1 the operand bytes per CU, not the MFMA, set the load phase.
// Thread t of wave w stages, per phase: A float4s e = t + NT*i (panel e >> 8,
// group (e >> 6) & 3), and B positions e = t + NT*i (tile e >> 8, group
// w & 3, its 4 k values) -- or, with BVEC, 16-byte row pieces (tile e >> 8,
// k row (e >> 2) & 63, column quad e & 3).  Same chains, fold and epilogue
// as gemm_lat2_kernel, so the same bits.
template <int RW, int CW, bool BVEC>
__global__ __launch_bounds__(64 * RW * CW) void gemm_lat3_kernel(DmaDesc d, int wg_m, int wg_n, int nkb, int subs) {
  constexpr int NW = RW * CW, NT = 64 * NW;
  constexpr int A_PT = 4 / CW;  // A float4 loads per thread and phase (RW * 256 / NT)
  constexpr int B_PT = 4 / RW;  // B positions (or BVEC pieces) per thread and phase (CW * 256 / NT)
  static_assert(RW >= 1 && RW <= 4 && CW >= 1 && CW <= 4 && A_PT * CW == 4 && B_PT * RW == 4, "tile shape");
  __shared__ float4 lds_a[RW][LGROUPS][64];
  __shared__ float4 lds_b[CW][LGROUPS][64];
  float* ldsk = reinterpret_cast<float*>(&lds_b[0][0][0]);  // BVEC: [CW][LKC][16]
  const int t = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int lane = t & 63;
  const int G = gridDim.x, bid = blockIdx.x;
  const int qq = G >> 3, rr = G & 7, xcd = bid & 7;
  const int o = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int tn = o % wg_n;
  const int t2 = o / wg_n;
  const int tm = t2 % wg_m;
  const int kb = t2 / wg_m;
  const int K = d.K;
  const int k0 = kb * LKC;
  const int ng = min(LGROUPS, (K - k0 + 15) >> 4);
  const int wr = wave / CW, wc = wave - (wave / CW) * CW;
  const int sub0 = tm * RW + wr;
  const int n0 = (tn * CW + wc) * 16;
  LatStamps stp = lat_stamps_init(d, kb, sub0, n0);

  typedef unsigned int lat3_u32x4 __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t ar =
      __builtin_amdgcn_make_buffer_rsrc((void*)d.apk, 0, (int)((int64_t)subs * nkb * LGROUPS * 64 * 16), 0x00020000);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)d.x, 0, (int)d.x_bytes, 0x00020000);
  const int h = lane >> 4;
  const bool linear = d.kstride > 0;

  // Per-thread constants of the B copies.
  uint32_t bcol[B_PT];  // x byte offset of this thread's column (or column quad) per position
#pragma unroll
  for (int i = 0; i < B_PT; i++) {
    const int e = t + NT * i;
    const int cw = e >> 8;
    if constexpr (BVEC) {
      const int n = (tn * CW + cw) * 16 + 4 * (e & 3);
      uint32_t cb = DMA_OOB;
      if (n < d.N) {
        const int img = fdiv(n, d.fdP);
        cb = (uint32_t)(((int64_t)img * d.x_img + (n - img * d.P)) * 4);
      }
      bcol[i] = cb;
    } else {
      bcol[i] = lat_col(d, (tn * CW + cw) * 16).vcol;
    }
  }
  // 3x3 windows: this thread's k in phase q, step j is kq + 64 q + 4 j with
  // kq = k0 + 16 (w & 3) + h; koff(k) for k = 9c + 3ky + kx (see lat_chain).
  const uint32_t kq = (uint32_t)(k0 + 16 * (wave & 3) + h);
  const int c0 = linear ? 0 : (int)(__umulhi(kq, 0x38E38E39u) >> 1);  // kq / 9
  const int r0 = (int)kq - 9 * c0;
  auto koff = [&](int q, int j) __attribute__((always_inline)) -> uint32_t {
    const int k = (int)kq + 64 * q + 4 * j;
    if (k >= K) return DMA_OOB;
    if (linear) return (uint32_t)k * (uint32_t)d.kstride * 4u;
    const int kk = r0 + 64 * q + 4 * j;  // < 213: (kk * 57) >> 9 == kk / 9
    const int q9 = (kk * 57) >> 9;
    const int rm = kk - 9 * q9;
    const int ky = (rm * 11) >> 5;
    const int kx = rm - 3 * ky;
    return (uint32_t)((c0 + q9) * d.kt_plane + ky * d.kt_row + kx * d.kt_col) * 4u;
  };

  // Every phase's loads, in k order.
  lat3_u32x4 av[4][A_PT];
  float bv[4][BVEC ? 1 : B_PT][4];
  lat3_u32x4 bq[4][BVEC ? B_PT : 1];
#pragma unroll
  for (int q = 0; q < 4; q++) {
#pragma unroll
    for (int i = 0; i < A_PT; i++) {
      const int e = t + NT * i;
      const int r = e >> 8, g = 4 * q + ((e >> 6) & 3);
      const int sub = tm * RW + r;
      const uint32_t off =
          (sub < subs && g < ng) ? (uint32_t)(((sub * nkb + kb) * LGROUPS + g) * 64 + lane) * 16u : DMA_OOB;
      av[q][i] = __builtin_amdgcn_raw_buffer_load_b128(ar, off, 0, 0);
    }
    if constexpr (BVEC) {
#pragma unroll
      for (int i = 0; i < B_PT; i++) {
        const int e = t + NT * i;
        const int k = k0 + 64 * q + ((e >> 2) & 63);
        const uint32_t off =
            (k < K && bcol[i] != DMA_OOB) ? bcol[i] + (uint32_t)k * (uint32_t)d.kstride * 4u : DMA_OOB;
        bq[q][i] = __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0);
      }
    } else {
      uint32_t ko[4];
#pragma unroll
      for (int j = 0; j < 4; j++) ko[j] = koff(q, j);
#pragma unroll
      for (int i = 0; i < B_PT; i++)
#pragma unroll
        for (int j = 0; j < 4; j++)
          bv[q][i][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, bcol[i] + ko[j], 0, 0));
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the phases' loads in k order
  }

  // Epilogue operands of this wave's tile, behind the operand loads.
  const bool live = sub0 < subs && n0 < d.N;
  const LatCol col = lat_col(d, n0);
  LatEpi<1> e;
  if (live) lat_epi_loads<1>(d, sub0, col, e);
  __builtin_amdgcn_sched_barrier(0);

  lat_f32x4 acc[1];
  acc[0] = (lat_f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 4; q++) {
    // Phase q to LDS (the compiler waits for exactly these loads).
#pragma unroll
    for (int i = 0; i < A_PT; i++) {
      const int e2 = t + NT * i;
      lds_a[e2 >> 8][4 * q + ((e2 >> 6) & 3)][lane] =
          make_float4(__uint_as_float(av[q][i].x), __uint_as_float(av[q][i].y), __uint_as_float(av[q][i].z),
                      __uint_as_float(av[q][i].w));
    }
    if constexpr (BVEC) {
#pragma unroll
      for (int i = 0; i < B_PT; i++) {
        const int e2 = t + NT * i;
        *reinterpret_cast<float4*>(ldsk + ((e2 >> 8) * LKC + 64 * q + ((e2 >> 2) & 63)) * 16 + 4 * (e2 & 3)) =
            make_float4(__uint_as_float(bq[q][i].x), __uint_as_float(bq[q][i].y), __uint_as_float(bq[q][i].z),
                        __uint_as_float(bq[q][i].w));
      }
    } else {
#pragma unroll
      for (int i = 0; i < B_PT; i++) {
        const int e2 = t + NT * i;
        lds_b[e2 >> 8][4 * q + (wave & 3)][lane] = make_float4(bv[q][i][0], bv[q][i][1], bv[q][i][2], bv[q][i][3]);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (q == 0) stp.at(2);
    if (live) {
#pragma unroll
      for (int gq = 0; gq < 4; gq++) {
        const int g = 4 * q + gq;
        if (g < ng) {
          const float4 a4 = lds_a[wr][g][lane];
          float4 b4;
          if constexpr (BVEC) {
            const float* bp = ldsk + (wc * LKC + 16 * g + h) * 16 + (lane & 15);
            b4 = make_float4(bp[0], bp[64], bp[128], bp[192]);  // k = 16g + 4j + h, j = 0..3
          } else {
            b4 = lds_b[wc][g][lane];
          }
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.x, b4.x, acc[0], 0, 0, 0);
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.y, b4.y, acc[0], 0, 0, 0);
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.z, b4.z, acc[0], 0, 0, 0);
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.w, b4.w, acc[0], 0, 0, 0);
        }
      }
    }
  }
  if (!live) return;  // (after the last barrier: every wave helped stage)
  if (stp.p) {
    asm volatile("" ::"v"(acc[0][0]), "v"(acc[0][3]));
    stp.at(3);
  }
  const int wt = sub0 * (wg_n * CW) + (n0 >> 4);
  lat_fold_finish<1>(d, sub0, kb, nkb, wt, col, e, acc, stp);
}

// Slab variant (6x), for one-image convs whose KC block reads few input
// values -- the 3x3 convs at 14x14 / 7x7 and the 1x1 convs at 7x7 of
// ResNet-50 at batch 1.  The B operand of such a block is im2col of at most
// 30 (3x3) or 256 (1x1) input planes of 81..256 floats, and every column tile
// of the block reads the same planes.  So a workgroup copies those planes --
// one contiguous run [c_lo * plane, c_hi * plane) of the (zero-bordered)
// input, 16-byte loads -- into LDS with its RW packed A panels, and forms
// every B operand from LDS: lane (c, h) at step s reads slab[colF(n) +
// koffF(k) - base], the same element the gather kernels load from memory
// (k past K and columns past N read a zero slot).  B then costs one linear
// copy per workgroup instead of a 4-byte gather per element and column tile,
// and the workgroup covers CW column tiles (4 or 8) x RW row tiles, one chain
// per wave.  Chains, fold and epilogue as gemm_lat2_kernel: the same bits.
template <int RW, int CW>
__global__ __launch_bounds__(64 * RW * CW) void gemm_lat4_kernel(DmaDesc d, int wg_m, int wg_n, int nkb, int subs) {
  constexpr int NW = RW * CW, NT = 64 * NW;
  constexpr int A_PT = RW * LGROUPS * 64 / NT;  // A float4 loads per thread (16 / CW)
  static_assert(A_PT * NT == RW * LGROUPS * 64, "A split");
  extern __shared__ float4 l4_lds[];
  float4* lds_a = l4_lds;                                             // [RW][16 groups][64 lanes]
  float* slab = reinterpret_cast<float*>(l4_lds + RW * LGROUPS * 64);  // the block's input planes, then a zero slot
  const int t = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int lane = t & 63;
  const int G = gridDim.x, bid = blockIdx.x;
  const int qq = G >> 3, rr = G & 7, xcd = bid & 7;
  const int o = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int tn = o % wg_n;
  const int t2 = o / wg_n;
  const int tm = t2 % wg_m;
  const int kb = t2 / wg_m;
  const int K = d.K;
  const int k0 = kb * LKC;
  const int ng = min(LGROUPS, (K - k0 + 15) >> 4);
  const int wr = wave / CW, wc = wave - (wave / CW) * CW;
  const int sub0 = tm * RW + wr;
  const int n0 = (tn * CW + wc) * 16;
  const int h = lane >> 4;
  LatStamps stp = lat_stamps_init(d, kb, sub0, n0);

  // The block's planes: channels [c_lo, c_hi), copied from the 16-byte
  // aligned element base4 <= c_lo * plane (base4 in the slab is index 0).
  const bool linear = d.kstride > 0;
  const int plane = linear ? d.kstride : d.kt_plane;
  const int k_last = min(K, k0 + LKC) - 1;
  const int c_lo = linear ? k0 : k0 / 9;
  const int c_hi = (linear ? k_last : k_last / 9) + 1;
  const int base4 = (c_lo * plane) & ~3;
  const int n4 = ((c_hi * plane + 3) & ~3) - base4 >> 2;  // float4s
  const int zslot = n4 * 4;

  typedef unsigned int lat4_u32x4 __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t ar =
      __builtin_amdgcn_make_buffer_rsrc((void*)d.apk, 0, (int)((int64_t)subs * nkb * LGROUPS * 64 * 16), 0x00020000);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)d.x, 0, (int)d.x_bytes, 0x00020000);
  lat4_u32x4 av[A_PT];
#pragma unroll
  for (int i = 0; i < A_PT; i++) {
    const int e = t + NT * i;
    const int r = e >> 10, gl = e & 1023;
    const int sub = tm * RW + r;
    const uint32_t off =
        (sub < subs && ((gl >> 6) < ng)) ? (uint32_t)(((sub * nkb + kb) * LGROUPS * 64 + gl) * 16) : DMA_OOB;
    av[i] = __builtin_amdgcn_raw_buffer_load_b128(ar, off, 0, 0);
  }
  // The slab: 8 loads in flight per thread per round (one round for the
  // 7x7 planes, two or three at 14x14 with 256 threads).
  constexpr int SU = 8;
  for (int i0 = t; i0 < n4; i0 += SU * NT) {
    lat4_u32x4 v[SU];
#pragma unroll
    for (int u = 0; u < SU; u++) {
      const int i = i0 + u * NT;
      v[u] = __builtin_amdgcn_raw_buffer_load_b128(xr, i < n4 ? (uint32_t)(base4 + 4 * i) * 4u : DMA_OOB, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < SU; u++) {
      const int i = i0 + u * NT;
      if (i < n4)
        reinterpret_cast<float4*>(slab)[i] = make_float4(__uint_as_float(v[u].x), __uint_as_float(v[u].y),
                                                         __uint_as_float(v[u].z), __uint_as_float(v[u].w));
    }
  }
  if (t == 0) slab[zslot] = 0.f;
#pragma unroll
  for (int i = 0; i < A_PT; i++) {
    const int e = t + NT * i;
    lds_a[e] = make_float4(__uint_as_float(av[i].x), __uint_as_float(av[i].y), __uint_as_float(av[i].z),
                           __uint_as_float(av[i].w));
  }

  // This lane's B address at step s (k = k0 + 4s + h): colF(n) - base4 +
  // koffF(k).  A column past N reads any slab element (its outputs are never
  // stored); a k past K (only in the last, partial group) the zero slot, as
  // A is zero there and the slab may not cover it.
  const bool live = sub0 < subs && n0 < d.N;
  const LatCol col = lat_col(d, n0);
  const int colF = (col.vcol != DMA_OOB ? (int)(col.vcol >> 2) : 0) - base4;
  LatEpi<1> e;
  if (live) lat_epi_loads<1>(d, sub0, col, e);
  __syncthreads();
  if (!live) return;  // (after the barrier: every wave helped stage)
  stp.at(2);

  lat_f32x4 acc[1];
  acc[0] = (lat_f32x4){0.f, 0.f, 0.f, 0.f};
  const bool kpart = ((K - k0) & 15) != 0;  // the last group is partial
  // Group g + 1's LDS reads are issued before group g's MFMAs.
  auto chain = [&](auto addr_of) __attribute__((always_inline)) {
    auto ld = [&](int g, float4& a4, float (&b)[4]) __attribute__((always_inline)) {
      a4 = lds_a[(wr * LGROUPS + g) * 64 + lane];
      int ad[4];
#pragma unroll
      for (int j = 0; j < 4; j++) ad[j] = addr_of(4 * g + j);
      if (kpart && g == ng - 1) {
#pragma unroll
        for (int j = 0; j < 4; j++) ad[j] = k0 + 16 * g + 4 * j + h < K ? ad[j] : zslot;
      }
#pragma unroll
      for (int j = 0; j < 4; j++) b[j] = slab[ad[j]];
    };
    float4 an;
    float bn[4];
    ld(0, an, bn);
#pragma unroll
    for (int g = 0; g < LGROUPS; g++) {
      if (g < ng) {
        const float4 a4 = an;
        const float b0 = bn[0], b1 = bn[1], b2 = bn[2], b3 = bn[3];
        if (g + 1 < LGROUPS && g + 1 < ng) ld(g + 1, an, bn);
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.x, b0, acc[0], 0, 0, 0);
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.y, b1, acc[0], 0, 0, 0);
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.z, b2, acc[0], 0, 0, 0);
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.w, b3, acc[0], 0, 0, 0);
      }
    }
  };
  if (linear) {
    const int lb = colF + (k0 + h) * d.kstride;
    const int s4 = 4 * d.kstride;
    chain([&](int st) { return lb + st * s4; });
  } else {
    // 3x3 windows: koffF(k) for k = 9c + 3ky + kx at k0 + h + 4s, s = 0..8;
    // koffF(k + 36) = koffF(k) + 4 plane.
    int lb[9];
    const uint32_t kh0 = (uint32_t)(k0 + h);
    const int c0 = (int)(__umulhi(kh0, 0x38E38E39u) >> 1);
    const int r0 = (int)kh0 - 9 * c0;
#pragma unroll
    for (int s9 = 0; s9 < 9; s9++) {
      const int kk = r0 + 4 * s9;
      const int q = (kk * 57) >> 9;
      const int rm = kk - 9 * q;
      const int ky = (rm * 11) >> 5;
      const int kx = rm - 3 * ky;
      lb[s9] = colF + (c0 + q) * d.kt_plane + ky * d.kt_row + kx * d.kt_col;
    }
    const int p4 = 4 * d.kt_plane;
    chain([&](int st) { return lb[st % 9] + (st / 9) * p4; });
  }
  if (stp.p) {
    asm volatile("" ::"v"(acc[0][0]), "v"(acc[0][3]));
    stp.at(3);
  }
  const int wt = sub0 * (wg_n * CW) + (n0 >> 4);
  lat_fold_finish<1>(d, sub0, kb, nkb, wt, col, e, acc, stp);
}

// Slab variants: LDS floats of the largest KC block's input planes (with the
// alignment slack and the zero slot), 0 when the conv does not qualify (more
// than one image, or no 1x1 / 3x3 window).
constexpr int64_t kLatSlabCap = 13312;  // 52 KB of planes

int64_t lat_slab_floats(const DmaDesc& d) {
  if (d.N != d.P) return 0;
  const bool linear = d.kstride > 0;
  if (!linear && !d.k3x3) return 0;
  const int64_t plane = linear ? d.kstride : d.kt_plane;
  int64_t best = 0;
  for (int k0 = 0; k0 < d.K; k0 += LKC) {
    const int k_last = (d.K < k0 + LKC ? d.K : k0 + LKC) - 1;
    const int64_t c_lo = linear ? k0 : k0 / 9, c_hi = (linear ? k_last : k_last / 9) + 1;
    const int64_t b4 = (c_lo * plane) & ~int64_t(3);
    const int64_t n = ((c_hi * plane + 3) & ~int64_t(3)) - b4;
    if (n + 4 > best) best = n + 4;
  }
  return best;
}

// All K blocks of one tile in one workgroup: W = min(nkb, 8) waves, wave w
// computes blocks w, w + W, ...; the chains meet in LDS and wave 0 folds them
// in K order -- no workspace, no arrival atomics, no round trip through the
// memory system between the blocks and the fold (variants 91 / 92).
template <int MI>
__global__ __launch_bounds__(512) void gemm_lat_wg_kernel(DmaDesc d, int n16, int nkb, int subs) {
  extern __shared__ float4 lat_wg_lds[];  // [W][LKC] k offsets (uint32), then [nkb][MI][64] chains
  const int W = blockDim.x >> 6;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  uint32_t* ktl = reinterpret_cast<uint32_t*>(lat_wg_lds) + wave * LKC;
  float4* part = lat_wg_lds + W * (LKC / 4);
  const int G = gridDim.x, bid = blockIdx.x;
  const int qq = G >> 3, rr = G & 7, xcd = bid & 7;
  const int o = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int nt = o % n16, sub0 = (o / n16) * MI;
  const LatCol col = lat_col(d, nt * 16);
  LatEpi<MI> e;  // wave 0's epilogue operands, loaded along with its first block's operands
  const bool early = !(d.dbg & 4);  // (d.dbg & 4: A/B experiments only, loaded after the chains)
  if (wave == 0 && early) lat_epi_loads<MI>(d, sub0, col, e);
  for (int kb = wave; kb < nkb; kb += W) {
    lat_f32x4 acc[MI];
    lat_chain<MI>(d, sub0, kb, nkb, subs, col, ktl, acc);
#pragma unroll
    for (int mi = 0; mi < MI; mi++)
      part[(kb * MI + mi) * 64 + lane] = make_float4(acc[mi][0], acc[mi][1], acc[mi][2], acc[mi][3]);
  }
  if (wave == 0 && !early) lat_epi_loads<MI>(d, sub0, col, e);
  __syncthreads();
  if (wave != 0) return;
  lat_f32x4 sum[MI];
  const float alpha = d.alpha;
  for (int kb = 0; kb < nkb; kb++)
#pragma unroll
    for (int mi = 0; mi < MI; mi++) {
      const float4 v = part[(kb * MI + mi) * 64 + lane];
      const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int r = 0; r < 4; r++)
        sum[mi][r] = kb == 0 ? lat_first_block(d, vv[r], e.bias[mi][r]) : __fmaf_rn(vv[r], alpha, sum[mi][r]);
    }
  lat_finish<MI>(d, sub0, col, e, sum);
}

// A[M, K] (row stride lda) -> [ceil(M/16)][nkb][16 groups][64 lanes] float4:
// lane (c, h) of group g of block kb holds row 16*sub + c, k = 256*kb + 16*g +
// 4*j + h for j = 0..3; zero past M and K.
__global__ __launch_bounds__(256) void pack_lat_kernel(const float* __restrict__ a, int64_t lda, int M, int K,
                                                       int nkb, int64_t total4, float4* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total4) return;
  const int lane = (int)(i & 63);
  const int g = (int)((i >> 6) & (LGROUPS - 1));
  const int64_t t = i >> 10;
  const int kb = (int)(t % nkb);
  const int64_t sub = t / nkb;
  const int64_t row = sub * 16 + (lane & 15);
  const int kbase = kb * LKC + 16 * g + (lane >> 4);
  float v[4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int k = kbase + 4 * j;
    v[j] = (row < M && k < K) ? a[row * lda + k] : 0.f;
  }
  out[i] = make_float4(v[0], v[1], v[2], v[3]);
}

int64_t lat_packed_floats(int M, int K) {
  const int64_t subs = (M + 15) / 16, nkb = (K + LKC - 1) / LKC;
  return subs * nkb * LKC * 16;
}

rtenhip_status launch_pack_lat(const float* a, int64_t lda, int M, int K, float* out, hipStream_t s) {
  const int64_t total4 = lat_packed_floats(M, K) / 4;
  if (total4 == 0) return RTENHIP_OK;
  const int nkb = (K + LKC - 1) / LKC;
  hipLaunchKernelGGL(pack_lat_kernel, dim3((unsigned)((total4 + 255) / 256)), dim3(256), 0, s, a, lda, M, K, nkb,
                     total4, reinterpret_cast<float4*>(out));
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

// Pipelined LDS-staged variants (gemm_lat3_kernel): RW x CW tiles per workgroup.
static bool lat3_shape(int v, int& rw, int& cw) {
  // (The 4-wave shapes 1x4 / 2x2 / 4x1 and 4x4 were built and measured:
  // slower than gemm_lat2_kernel on every ResNet-50 batch-1 conv, see
  // profiles/r5_lat3.txt.)
  switch (v) {
    case 85: rw = 2; cw = 4; return true;
    case 86: rw = 4; cw = 2; return true;
    default: return false;
  }
}

// Slab variants (gemm_lat4_kernel): RW x CW tiles per workgroup.
static bool lat4_shape(int v, int& rw, int& cw) {
  switch (v) {
    case 61: rw = 1; cw = 4; return true;
    case 62: rw = 2; cw = 4; return true;
    case 63: rw = 1; cw = 8; return true;
    case 66: rw = 2; cw = 8; return true;
    default: return false;
  }
}

bool lat_variant_ok(int v) {
  int rw, cw;
  if (lat3_shape(v, rw, cw) || lat4_shape(v, rw, cw)) return true;
  if (v == 91 || v == 92) return true;  // workgroup fold
  if (v == 71 || v == 72 || v == 74) return true;  // LDS-staged, RW = v - 70 rows x CW = 4 / RW columns
  const int wmw = v / 10, mi = v % 10;
  return (wmw == 1 || wmw == 2 || wmw == 4) && (mi == 1 || mi == 2);
}

struct LatGrid {
  int subs, wg_m, wg_n, nkb;
  int64_t wgs, tiles;
};
static LatGrid lat_grid(int M, int N, int K, int v) {
  // (LDS-staged variants: RW row tiles x CW column tiles per workgroup, one each per wave)
  const bool lds = v >= 70 && v < 80;
  int rw3 = 0, cw3 = 0;
  const bool p3 = lat3_shape(v, rw3, cw3) || lat4_shape(v, rw3, cw3);
  const int wmw = p3 ? rw3 : (lds ? v - 70 : v / 10), mi = (lds || p3) ? 1 : v % 10, wnw = p3 ? cw3 : 4 / wmw;
  LatGrid g;
  g.subs = (M + 15) / 16;
  g.wg_m = (g.subs + wmw * mi - 1) / (wmw * mi);
  g.wg_n = ((N + 15) / 16 + wnw - 1) / wnw;
  g.nkb = (K + LKC - 1) / LKC;
  g.wgs = (int64_t)g.wg_m * g.wg_n * g.nkb;
  g.tiles = (int64_t)g.wg_m * wmw * g.wg_n * wnw;
  return g;
}

DmaSplit lat_split_plan(int M, int N, int K, int v) {
  DmaSplit sp{0, 0, 0, 0};
  if (!lat_variant_ok(v) || v >= 90) return sp;  // the workgroup-fold variants need no workspace
  const LatGrid g = lat_grid(M, N, K, v);
  if (g.nkb < 2) return sp;
  sp.split_tiles = (int)g.tiles;
  sp.nkb = g.nkb;
  sp.ws_floats = g.tiles * g.nkb * ((v >= 60 && v < 90) ? 1 : v % 10) * 256;
  sp.counters = g.tiles;
  return sp;
}

template <int WMW, int MI>
static void lat_launch(const DmaDesc& d, const LatGrid& g, hipStream_t s) {
  hipLaunchKernelGGL((gemm_lat_kernel<WMW, MI>), dim3((unsigned)g.wgs), dim3(256), 0, s, d, g.wg_m, g.wg_n, g.nkb,
                     g.subs);
}

// Pair launches (gemm_lat2_pair_kernel): LDS-staged variants 71 / 72 / 74 on
// both sides, the instantiated combinations below (problem 0 with 16-byte B
// copies -- a bottleneck's conv1 -- problem 1 either way).
static int lat2_rw(int v) { return v == 71 ? 1 : v == 72 ? 2 : v == 74 ? 4 : 0; }
bool lat_pair_variants_ok(int v0, int v1) {
  const int r0 = lat2_rw(v0), r1 = lat2_rw(v1);
  return r0 && r1 && (r0 == r1 || (r0 == 2 && r1 == 4) || (r0 == 4 && r1 == 2));
}

rtenhip_status launch_gemm_lat_pair(const DmaDesc& d0, int v0, const DmaDesc& d1, int v1, hipStream_t s) {
  if (!lat_pair_variants_ok(v0, v1) || !d0.bvec) return fail(RTENHIP_UNSUPPORTED_VALUE, "latency GEMM pair: variants");
  const DmaDesc* ds[2] = {&d0, &d1};
  const int vs[2] = {v0, v1};
  LatPairGrid pg[2];
  for (int i = 0; i < 2; i++) {
    const DmaDesc& d = *ds[i];
    if (d.M <= 0 || d.N <= 0 || d.K <= 0) return fail(RTENHIP_INVALID_VALUE, "empty latency GEMM");
    if (d.cin) return fail(RTENHIP_UNSUPPORTED_VALUE, "latency GEMM: beta * C not supported");
    if (d.kstride <= 0 && !d.k3x3) return fail(RTENHIP_UNSUPPORTED_VALUE, "LDS latency GEMM: 1x1 or 3x3 windows only");
    const LatGrid g = lat_grid(d.M, d.N, d.K, vs[i]);
    if (g.nkb > 1 && (!d.ws || !d.counters)) return fail(RTENHIP_INVALID_VALUE, "latency GEMM needs its K-block workspace");
    pg[i] = {g.wg_m, g.wg_n, g.nkb, g.subs, (int)g.wgs};
  }
  const int64_t wgs = (int64_t)pg[0].wgs + pg[1].wgs;
  if (wgs > 0x7fffffff) return fail(RTENHIP_UNSUPPORTED_VALUE, "latency GEMM pair grid too large");
  const dim3 grid((unsigned)wgs), blk(256);
  DmaDesc a = d0, b = d1;
  a.stamps = b.stamps = nullptr;
  const int r0 = lat2_rw(v0), r1 = lat2_rw(v1);
#define LATP(R0, R1)                                                                                         \
  if (r0 == R0 && r1 == R1) {                                                                                \
    if (b.bvec)                                                                                              \
      hipLaunchKernelGGL((gemm_lat2_pair_kernel<R0, 4 / R0, true, R1, 4 / R1, true>), grid, blk, 0, s, a, pg[0], b, pg[1]);   \
    else                                                                                                     \
      hipLaunchKernelGGL((gemm_lat2_pair_kernel<R0, 4 / R0, true, R1, 4 / R1, false>), grid, blk, 0, s, a, pg[0], b, pg[1]);  \
  }
  LATP(1, 1)
  LATP(2, 2)
  LATP(4, 4)
  LATP(2, 4)
  LATP(4, 2)
#undef LATP
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

rtenhip_status launch_gemm_lat(const DmaDesc& d0, int v, hipStream_t s) {
  DmaDesc d = d0;
  d.stamps = nullptr;
  if (g_lat_stamps) {
    int rw3 = 1, cw3 = 4;
    if (!lat3_shape(v, rw3, cw3)) lat4_shape(v, rw3, cw3);
    const int64_t waves = v >= 90 ? 0 : lat_grid(d.M, d.N, d.K, v).wgs * rw3 * cw3;
    if (waves > 0 && g_lat_stamps_used + waves <= g_lat_stamps_cap) {
      d.stamps = g_lat_stamps + kLatStampWords * g_lat_stamps_used;
      g_lat_stamps_used += waves;
      d.dbg = (d.dbg & 0xff) | (++g_lat_seq << 8);
    }
  }
  if (d.M <= 0 || d.N <= 0 || d.K <= 0) return fail(RTENHIP_INVALID_VALUE, "empty latency GEMM");
  if (!lat_variant_ok(v)) return fail(RTENHIP_INVALID_VALUE, "unknown latency GEMM variant");
  if (d.cin) return fail(RTENHIP_UNSUPPORTED_VALUE, "latency GEMM: beta * C not supported");
  if (d.kstride <= 0 && !d.ktab4) return fail(RTENHIP_INVALID_VALUE, "latency GEMM: no K table");
  if (v >= 90) {
    const int mi = v - 90;
    const int subs = (d.M + 15) / 16, n16 = (d.N + 15) / 16, nkb = (d.K + LKC - 1) / LKC;
    const int64_t tiles = (int64_t)((subs + mi - 1) / mi) * n16;
    const int W = nkb < 8 ? nkb : 8;
    const size_t lds = (size_t)W * LKC * 4 + (size_t)nkb * mi * 64 * 16;
    if (tiles > 0x7fffffff || lds > 64 * 1024) return fail(RTENHIP_UNSUPPORTED_VALUE, "latency GEMM (workgroup fold) too large");
    if (mi == 1)
      hipLaunchKernelGGL((gemm_lat_wg_kernel<1>), dim3((unsigned)tiles), dim3(64 * W), lds, s, d, n16, nkb, subs);
    else
      hipLaunchKernelGGL((gemm_lat_wg_kernel<2>), dim3((unsigned)tiles), dim3(64 * W), lds, s, d, n16, nkb, subs);
    RTENHIP_LAUNCH_CHECK();
    return RTENHIP_OK;
  }
  const LatGrid g = lat_grid(d.M, d.N, d.K, v);
  if (g.wgs > 0x7fffffff) return fail(RTENHIP_UNSUPPORTED_VALUE, "latency GEMM grid too large");
  if (g.nkb > 1 && (!d.ws || !d.counters)) return fail(RTENHIP_INVALID_VALUE, "latency GEMM needs its K-block workspace");
  int rw3 = 0, cw3 = 0;
  if (lat4_shape(v, rw3, cw3)) {
    const int64_t slab = lat_slab_floats(d);
    if (slab <= 0 || slab > kLatSlabCap)
      return fail(RTENHIP_UNSUPPORTED_VALUE, "slab latency GEMM: one image and a 1x1 / 3x3 window whose planes fit LDS");
    const size_t lds = (size_t)rw3 * LGROUPS * 64 * 16 + (size_t)slab * 4;
    const dim3 grid((unsigned)g.wgs), blk(64 * rw3 * cw3);
#define LAT4(R, C)                                                                                          \
  if (rw3 == R && cw3 == C) {                                                                               \
    static const bool attr = hipFuncSetAttribute((const void*)gemm_lat4_kernel<R, C>,                        \
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) ==   \
                             hipSuccess;                                                                    \
    (void)attr;                                                                                             \
    hipLaunchKernelGGL((gemm_lat4_kernel<R, C>), grid, blk, lds, s, d, g.wg_m, g.wg_n, g.nkb, g.subs);       \
  }
    LAT4(1, 4)
    LAT4(2, 4)
    LAT4(1, 8)
    LAT4(2, 8)
#undef LAT4
    RTENHIP_LAUNCH_CHECK();
    return RTENHIP_OK;
  }
  if (lat3_shape(v, rw3, cw3)) {
    if (d.kstride <= 0 && !d.k3x3) return fail(RTENHIP_UNSUPPORTED_VALUE, "LDS latency GEMM: 1x1 or 3x3 windows only");
    const dim3 grid((unsigned)g.wgs), blk(64 * rw3 * cw3);
#define LAT3(R, C)                                                                                        \
  if (rw3 == R && cw3 == C) {                                                                             \
    if (d.bvec)                                                                                           \
      hipLaunchKernelGGL((gemm_lat3_kernel<R, C, true>), grid, blk, 0, s, d, g.wg_m, g.wg_n, g.nkb, g.subs);  \
    else                                                                                                  \
      hipLaunchKernelGGL((gemm_lat3_kernel<R, C, false>), grid, blk, 0, s, d, g.wg_m, g.wg_n, g.nkb, g.subs); \
  }
    LAT3(2, 4)
    LAT3(4, 2)
#undef LAT3
    RTENHIP_LAUNCH_CHECK();
    return RTENHIP_OK;
  }
  if (v >= 70 && v < 80) {
    if (d.kstride <= 0 && !d.k3x3) return fail(RTENHIP_UNSUPPORTED_VALUE, "LDS latency GEMM: 1x1 or 3x3 windows only");
    const dim3 grid((unsigned)g.wgs), blk(256);
    if (d.bvec) {
      if (v == 71) hipLaunchKernelGGL((gemm_lat2_kernel<1, 4, true>), grid, blk, 0, s, d, g.wg_m, g.wg_n, g.nkb, g.subs);
      else if (v == 72) hipLaunchKernelGGL((gemm_lat2_kernel<2, 2, true>), grid, blk, 0, s, d, g.wg_m, g.wg_n, g.nkb, g.subs);
      else hipLaunchKernelGGL((gemm_lat2_kernel<4, 1, true>), grid, blk, 0, s, d, g.wg_m, g.wg_n, g.nkb, g.subs);
    } else {
      if (v == 71) hipLaunchKernelGGL((gemm_lat2_kernel<1, 4, false>), grid, blk, 0, s, d, g.wg_m, g.wg_n, g.nkb, g.subs);
      else if (v == 72) hipLaunchKernelGGL((gemm_lat2_kernel<2, 2, false>), grid, blk, 0, s, d, g.wg_m, g.wg_n, g.nkb, g.subs);
      else hipLaunchKernelGGL((gemm_lat2_kernel<4, 1, false>), grid, blk, 0, s, d, g.wg_m, g.wg_n, g.nkb, g.subs);
    }
    RTENHIP_LAUNCH_CHECK();
    return RTENHIP_OK;
  }
  switch (v) {
    case 41: lat_launch<4, 1>(d, g, s); break;
    case 21: lat_launch<2, 1>(d, g, s); break;
    case 11: lat_launch<1, 1>(d, g, s); break;
    case 42: lat_launch<4, 2>(d, g, s); break;
    case 22: lat_launch<2, 2>(d, g, s); break;
    default: lat_launch<1, 2>(d, g, s); break;
  }
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

}  // namespace rtenhip

extern "C" void rtenhip_debug_set_lat_stamps(void* buf, int64_t cap_waves) {
  rtenhip::g_lat_stamps = static_cast<unsigned long long*>(buf);
  rtenhip::g_lat_stamps_cap = cap_waves;
  rtenhip::g_lat_stamps_used = 0;
  rtenhip::g_lat_seq = 0;
}
extern "C" int64_t rtenhip_debug_lat_stamps_used() { return rtenhip::g_lat_stamps_used; }
