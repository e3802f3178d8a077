// Building blocks of the latency GEMM (gemm_lat.hip): a wave
// computes the chains of a (16*MI) x 16 output tile for one KC block
// (lat_chain); the blocks of a tile are folded in K order either by the last
// block to arrive through a global workspace (lat_unit) or inside one
// workgroup through LDS (gemm_lat_wg_kernel); lat_finish applies the
// epilogue.  Summation contract (src/gemm.rs:733-1050, as the DMA kernel
// states it): one fma chain per element and KC = 256 block from +0, then
// alpha * chain (+ bias after block 0), later blocks fma'd in K order, then
// the column bias, the residual and the activation.
#pragma once

#include "gemm_dma.h"
#include "fastdiv_dev.h"
#include "vecmath.h"

namespace rtenhip {

typedef float lat_f32x4 __attribute__((ext_vector_type(4)));
constexpr int LKC = 256;           // the reference's KC block
constexpr int LGROUPS = LKC / 16;  // 16-k groups per block (4 MFMA steps each)

__device__ __forceinline__ float lat_f4(const float4& v, int j) {
  return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
}


// The output column of this lane (c = lane % 16) of a tile starting at n0,
// and its x offset colbase(n) in bytes (DMA_OOB past N).
struct LatCol {
  int n, img, p, oy, ox;
  uint32_t vcol;
};
__device__ __forceinline__ LatCol lat_col(const DmaDesc& d, int n0) {
  LatCol col;
  col.n = n0 + ((threadIdx.x & 63) & 15);
  col.img = col.p = col.oy = col.ox = 0;
  col.vcol = DMA_OOB;
  if (col.n < d.N) {
    col.img = fdiv(col.n, d.fdP);
    col.p = col.n - col.img * d.P;
    col.oy = fdiv(col.p, d.fdOW);
    col.ox = col.p - col.oy * d.OW;
    col.vcol = (uint32_t)(((int64_t)col.img * d.x_img + (int64_t)col.oy * d.ystride + (int64_t)col.ox * d.xstride) * 4);
  }
  return col;
}

// The chains of KC block kb: acc[mi] = fma chains over the block's k, from
// +0.  ktl: this wave's 256-word LDS slot.
template <int MI>
__device__ __forceinline__ void lat_chain(const DmaDesc& d, const int sub0, const int kb, const int nkb, const int subs,
                                          const LatCol& col, uint32_t* ktl,
                                          lat_f32x4 (&acc)[MI], const bool drain = false) {
  const int lane = threadIdx.x & 63;
  const int h = lane >> 4;
  const int K = d.K;
  const int k0 = kb * LKC;
  const int ng = min(LGROUPS, (K - k0 + 15) >> 4);
  const bool linear = d.kstride > 0;
  const bool k3 = !linear && d.k3x3;

  // 3x3 windows: koff(k) for k = 9c + 3ky + kx is c * plane + ky * row +
  // kx * col -- the table's entries (Ctx::dtab) formed here, so the B gathers
  // do not wait for a table load.  This lane visits k = k0 + h + 4s and
  // koff(k + 36) = koff(k) + 4 * plane: nine offsets, the rest by adds.
  uint32_t k3off[9];
  const uint32_t k3step = 16u * (uint32_t)d.kt_plane;  // bytes per +36 in k
  if (k3) {
    const uint32_t kh0 = (uint32_t)(k0 + h);
    const int c0 = (int)(__umulhi(kh0, 0x38E38E39u) >> 1);  // kh0 / 9
    const int r0 = (int)kh0 - 9 * c0;
#pragma unroll
    for (int s = 0; s < 9; s++) {
      const int kk = r0 + 4 * s;          // < 41
      const int q = (kk * 57) >> 9;       // kk / 9
      const int rr = kk - 9 * q;
      const int ky = (rr * 11) >> 5;      // rr / 3
      const int kx = rr - 3 * ky;
      k3off[s] = (uint32_t)((c0 + q) * d.kt_plane + ky * d.kt_row + kx * d.kt_col) * 4u;
    }
  }

  // Table mode: lane L loads entries 4L..4L+3 of the block and stores entry
  // k at [k % 4][k / 4], so the lane with k parity h reads the offsets of 4
  // consecutive MFMA steps as one 16-byte LDS read.  (The slot is private to
  // the wave and LDS operations of a wave complete in order.)
  if (!linear && !k3) {
    const int kpad = (K + DMA_KTAB_PAD - 1) / DMA_KTAB_PAD * DMA_KTAB_PAD;
    int4 t = make_int4((int)DMA_OOB, (int)DMA_OOB, (int)DMA_OOB, (int)DMA_OOB);
    if (k0 + lane * 4 < kpad) t = *(const int4*)(d.ktab4 + k0 + lane * 4);
    ktl[lane] = (uint32_t)t.x;
    ktl[64 + lane] = (uint32_t)t.y;
    ktl[128 + lane] = (uint32_t)t.z;
    ktl[192 + lane] = (uint32_t)t.w;
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }

  // A: packed [subtile][kb][group][lane] float4 (launch_pack_lat: zero past
  // K inside a block); subtiles past M read past the buffer, which returns 0.
  // B: step s = 4g + j covers k = k0 + 4s + h for this lane.
  // Every load below is issued unconditionally (a guarded load would be a
  // branch and a wait each), group by group in k order -- A then B of group
  // g -- so the chain's first steps wait only for group 0 (vmcnt retires in
  // issue order) and run while the later groups are still in flight.
  typedef unsigned int lat_u32x4 __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t ar =
      __builtin_amdgcn_make_buffer_rsrc((void*)d.apk, 0, (int)((int64_t)subs * nkb * LGROUPS * 64 * 16), 0x00020000);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)d.x, 0, (int)d.x_bytes, 0x00020000);
  lat_u32x4 av[LGROUPS][MI];
  float bv[LKC / 4];
#pragma unroll
  for (int g = 0; g < LGROUPS; g++) {
#pragma unroll
    for (int mi = 0; mi < MI; mi++) {
      const uint32_t off = (sub0 + mi < subs && g < ng)
                               ? (uint32_t)((((sub0 + mi) * nkb + kb) * LGROUPS + g) * 64 + lane) * 16u
                               : DMA_OOB;
      av[g][mi] = __builtin_amdgcn_raw_buffer_load_b128(ar, off, 0, 0);
    }
    uint32_t ko[4];
    if (linear || k3) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int st = 4 * g + j;
        const int k = k0 + 16 * g + 4 * j + h;
        const uint32_t lin = (uint32_t)k * (uint32_t)d.kstride * 4u;
        const uint32_t win = k3off[st % 9] + (uint32_t)(st / 9) * k3step;
        ko[j] = k < K ? (linear ? lin : win) : DMA_OOB;
      }
    } else {
      const uint4 t = *(const uint4*)&ktl[h * 64 + 4 * g];  // DMA_OOB past K (padded table)
      ko[0] = t.x;
      ko[1] = t.y;
      ko[2] = t.z;
      ko[3] = t.w;
    }
#pragma unroll
    for (int j = 0; j < 4; j++)
      bv[4 * g + j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, col.vcol + ko[j], 0, 0));
    __builtin_amdgcn_sched_barrier(0);  // keep the groups' loads in k order
  }

  if (drain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // timing experiments only
#pragma unroll
  for (int mi = 0; mi < MI; mi++) acc[mi] = (lat_f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int g = 0; g < LGROUPS; g++) {
    if (g < ng) {
#pragma unroll
      for (int j = 0; j < 4; j++)
#pragma unroll
        for (int mi = 0; mi < MI; mi++)
          acc[mi] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(av[g][mi][j]), bv[4 * g + j], acc[mi], 0, 0, 0);
    }
  }
}

// Epilogue operands of this lane's accumulator elements: the row bias and the
// residual.  Element r of lane (c, h) is row
// 4h + r, column c.
template <int MI>
struct LatEpi {
  float bias[MI][4], res[MI][4];
  float cbv;
};
template <int MI>
__device__ __forceinline__ void lat_epi_loads(const DmaDesc& d, const int sub0, const LatCol& col,
                                              LatEpi<MI>& e) {
  const int h = (threadIdx.x & 63) >> 4;
  const int64_t rbase = (int64_t)col.img * d.res_img + col.p;
#pragma unroll
  for (int mi = 0; mi < MI; mi++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int m = (sub0 + mi) * 16 + 4 * h + r;
      const int mc = min(m, d.M - 1);
      e.bias[mi][r] = d.bias ? d.bias[mc] : 0.f;
      e.res[mi][r] = 0.f;
      if (d.residual && col.n < d.N) {
        const float* rp = d.residual + rbase + (int64_t)mc * d.res_c;
        e.res[mi][r] = *rp;
      }
    }
  e.cbv = (d.colbias && col.n < d.N) ? d.colbias[col.p] : 0.f;
}

// End of K block 0: alpha * chain + bias (gemm.rs:1004-1050).
__device__ __forceinline__ float lat_first_block(const DmaDesc& d, float a, float b) {
  float x = d.alpha == 1.f ? a : __fmul_rn(a, d.alpha);
  if (d.bias) x = __fadd_rn(x, b);
  return x;
}

// Column bias, residual, activation and the store of the folded tile.
template <int MI>
__device__ __forceinline__ void lat_finish(const DmaDesc& d, const int sub0, const LatCol& col, const LatEpi<MI>& e,
                                           const lat_f32x4 (&sum)[MI]) {
  const int h = (threadIdx.x & 63) >> 4;
  const bool act_relu = d.act == RTENHIP_ACT_RELU, act_clip = d.act == RTENHIP_ACT_CLIP;
  const bool act_gelu = d.act == RTENHIP_ACT_GELU;
  const float lo = d.act_lo, hi = d.act_hi;
  const int64_t obase = (int64_t)col.img * d.out_img + (int64_t)col.oy * d.out_row + col.ox + d.out_off;
  if (col.n >= d.N) return;
  // Fused BatchNormalization (DmaDesc::bn): its parameters are loaded here,
  // after the chains, so convs without one keep the registers.
  float bnp[MI][4][3];
  if (d.bn) {
#pragma unroll
    for (int mi = 0; mi < MI; mi++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int mc = min((sub0 + mi) * 16 + 4 * h + r, d.M - 1);
        bnp[mi][r][0] = d.bn[mc];
        bnp[mi][r][1] = d.bn[d.bn_c + mc];
        bnp[mi][r][2] = d.bn[2 * d.bn_c + mc];
      }
  }
#pragma unroll
  for (int mi = 0; mi < MI; mi++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int m = (sub0 + mi) * 16 + 4 * h + r;
      float x = sum[mi][r];
      if (d.colbias) x = __fadd_rn(x, e.cbv);
      if (d.bn) x = __fadd_rn(__fmul_rn(__fsub_rn(x, bnp[mi][r][0]), bnp[mi][r][1]), bnp[mi][r][2]);
      if (d.residual) x = __fadd_rn(x, e.res[mi][r]);
      if (act_gelu) {
        x = vm_gelu(x);
      } else {
        const float rl = fmaxf(x, 0.f);
        const float cl = rust_clamp(x, lo, hi);
        x = act_relu ? rl : (act_clip ? cl : x);
      }
      if (m < d.M) {
        float* op = d.out + obase + (int64_t)m * d.out_c;
        *op = x;
      }
    }
}

// Timing experiments only (rtenhip_debug_set_lat_stamps; d.stamps null in
// every product launch): per wave kLatStampWords u64 = {launch seq << 48 |
// XCC << 40 | hw id bits << 32 | kb << 16 | wave-in-grid low 16 bits, t_entry,
// t_loaded, t_chain, t_arrived, t_folded, t_end, sub0 << 32 | n0, then for the
// LDS-staged kernel t_a_landed, t_b_landed}, s_memrealtime (100 MHz).
constexpr int kLatStampWords = 10;
struct LatStamps {
  unsigned long long* p = nullptr;
  __device__ __forceinline__ void at(int i) {
    if (p && (threadIdx.x & 63) == 0) p[i] = __builtin_amdgcn_s_memrealtime();
  }
};
__device__ __forceinline__ LatStamps lat_stamps_init(const DmaDesc& d, int kb, int sub0, int n0) {
  LatStamps st;
  if (!d.stamps) return st;
  const unsigned gw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  st.p = d.stamps + kLatStampWords * (size_t)gw;
  if ((threadIdx.x & 63) == 0) {
    unsigned xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    st.p[0] = ((unsigned long long)((unsigned)d.dbg >> 8) << 48) | ((unsigned long long)(xcc & 0xff) << 40) |
              ((unsigned long long)((hw >> 8) & 0xff) << 32) | ((unsigned long long)(kb & 0xffff) << 16) | (gw & 0xffff);
    st.p[7] = ((unsigned long long)(unsigned)sub0 << 32) | (unsigned)n0;
    for (int i = 2; i < kLatStampWords; i++)
      if (i != 7) st.p[i] = 0;
  }
  st.at(1);
  return st;
}

// The K-block fold of one unit's chains and the tile's epilogue: with
// nkb == 1 directly; else the chains go to the workspace ([tile][kb][mi][lane]
// x 16 bytes, 8-byte agent-scope stores), drained before the arrival count,
// and the last block of the tile to arrive folds all chains in K order.
// Returns false for a unit that did not store the tile.
template <int MI>
__device__ __forceinline__ bool lat_fold_finish(const DmaDesc& d, const int sub0, const int kb, const int nkb,
                                                const int wt, const LatCol& col, const LatEpi<MI>& e,
                                                const lat_f32x4 (&acc)[MI], LatStamps& stp) {
  const int lane = threadIdx.x & 63;
  const float alpha = d.alpha;

  lat_f32x4 sum[MI];
  if (nkb == 1) {
#pragma unroll
    for (int mi = 0; mi < MI; mi++)
#pragma unroll
      for (int r = 0; r < 4; r++) sum[mi][r] = lat_first_block(d, acc[mi][r], e.bias[mi][r]);
  } else {
    unsigned long long* wsq = reinterpret_cast<unsigned long long*>(d.ws);
    auto qi = [&](int kbi, int mi) { return ((((int64_t)wt * nkb + kbi) * MI + mi) * 64 + lane) * 2; };
#pragma unroll
    for (int mi = 0; mi < MI; mi++) {
      const unsigned long long q0 =
          (unsigned long long)__float_as_uint(acc[mi][0]) | ((unsigned long long)__float_as_uint(acc[mi][1]) << 32);
      const unsigned long long q1 =
          (unsigned long long)__float_as_uint(acc[mi][2]) | ((unsigned long long)__float_as_uint(acc[mi][3]) << 32);
      __hip_atomic_store(wsq + qi(kb, mi), q0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(wsq + qi(kb, mi) + 1, q1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int prev = 0;
    if (lane == 0) prev = __hip_atomic_fetch_add(d.counters + wt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    prev = __builtin_amdgcn_readfirstlane(prev);
    stp.at(4);
    if (prev != nkb - 1) return false;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only
    auto ldq = [&](int64_t i) { return __hip_atomic_load(wsq + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    constexpr int FG = 16;  // chains loaded per round
    for (int kb0 = 0; kb0 < nkb; kb0 += FG) {
      unsigned long long part[FG][MI][2];
#pragma unroll
      for (int i = 0; i < FG; i++)
#pragma unroll
        for (int mi = 0; mi < MI; mi++) {
          part[i][mi][0] = part[i][mi][1] = 0ull;
          if (kb0 + i < nkb) {
            part[i][mi][0] = ldq(qi(kb0 + i, mi));
            part[i][mi][1] = ldq(qi(kb0 + i, mi) + 1);
          }
        }
#pragma unroll
      for (int i = 0; i < FG; i++) {
        if (kb0 + i >= nkb) break;
#pragma unroll
        for (int mi = 0; mi < MI; mi++) {
          float v[4];
          v[0] = __uint_as_float((unsigned)(part[i][mi][0] & 0xffffffffu));
          v[1] = __uint_as_float((unsigned)(part[i][mi][0] >> 32));
          v[2] = __uint_as_float((unsigned)(part[i][mi][1] & 0xffffffffu));
          v[3] = __uint_as_float((unsigned)(part[i][mi][1] >> 32));
#pragma unroll
          for (int r = 0; r < 4; r++)
            sum[mi][r] = kb0 + i == 0 ? lat_first_block(d, v[r], e.bias[mi][r]) : __fmaf_rn(v[r], alpha, sum[mi][r]);
        }
      }
    }
    if (lane == 0) __hip_atomic_store(d.counters + wt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (stp.p) {
      asm volatile("" ::"v"(sum[0][0]));
      stp.at(5);
    }
  }

  lat_finish<MI>(d, sub0, col, e, sum);
  if (stp.p) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stp.at(6);
  }
  return true;
}

// One unit (sub0: first 16-row subtile, n0: first column, kb: KC block, wt:
// the tile's index into ws / counters): the epilogue operands and the block's
// operands in flight together (one memory round trip), the chains, then
// lat_fold_finish.  (d.dbg & 4: A/B experiments only, the epilogue operands
// loaded after the chain.)
template <int MI>
__device__ __forceinline__ void lat_unit(const DmaDesc& d, const int sub0, const int n0, const int kb, const int nkb,
                                         const int subs, const int wt, uint32_t* ktl) {
  LatStamps stp = lat_stamps_init(d, kb, sub0, n0);
  const LatCol col = lat_col(d, n0);
  const bool early = !(d.dbg & 4);
  LatEpi<MI> e;
  if (early) lat_epi_loads<MI>(d, sub0, col, e);
  lat_f32x4 acc[MI];
  lat_chain<MI>(d, sub0, kb, nkb, subs, col, ktl, acc, stp.p != nullptr);
  if (stp.p) {
    stp.at(2);  // operands in registers (lat_chain waited for them)
    asm volatile("" ::"v"(acc[0][0]), "v"(acc[0][3]));
    stp.at(3);  // chain issued
  }
  if (!early) lat_epi_loads<MI>(d, sub0, col, e);
  lat_fold_finish<MI>(d, sub0, kb, nkb, wt, col, e, acc, stp);
}

}  // namespace rtenhip
