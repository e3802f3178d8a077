// One unit of the latency GEMM (gemm_lat.hip, conv_chain.hip): a wave
// computes a (16*MI) x 16 output tile of one KC block and, with K > 256,
// the last of the tile's KC blocks to arrive folds all blocks' chains in K
// order.  Summation contract (src/gemm.rs:733-1050, as the DMA kernel states
// it): one fma chain per element and KC = 256 block from +0, then
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
constexpr int kLoadSc1 = 16;       // buffer-load cache policy: sc1 (L1 bypass, see conv_chain.hip)

__device__ __forceinline__ float lat_f4(const float4& v, int j) {
  return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
}

struct LatNoWait {
  __device__ void operator()() const {}
};
struct LatNoDone {
  __device__ void operator()() const {}
};

// The unit (sub0: first 16-row subtile, n0: first column, kb: KC block, wt:
// the tile's index into ws / counters).  ktl: this wave's 256-word LDS slot.
// wait(): called once the unit's weight and K-table loads are in flight and
// before its first load of x or of the residual (chain: their producers run
// in the same launch).  CHAIN: x and the residual are read with sc1 loads,
// the output is stored sc1 and drained, and the wave that stored the tile
// then calls done() (the inter-layer hand-off of conv_chain.hip).
template <int MI, bool CHAIN, typename Wait, typename Done>
__device__ __forceinline__ void lat_unit(const DmaDesc& d, const int sub0, const int n0, const int kb, const int nkb,
                                         const int subs, const int wt, uint32_t* ktl, Wait wait, Done done,
                                         int dbg = 0) {
  // dbg (timing experiments only, results not valid across XCDs): bit 0 plain
  // x / residual loads, bit 1 plain output stores.
  const bool sc1_ld = CHAIN && !(dbg & 1), sc1_st = CHAIN && !(dbg & 2);
  const int lane = threadIdx.x & 63;
  const int c = lane & 15, h = lane >> 4;
  const int M = d.M, N = d.N, K = d.K;
  const int k0 = kb * LKC;
  const int ng = min(LGROUPS, (K - k0 + 15) >> 4);
  const bool linear = d.kstride > 0;

  // Table mode: lane L loads entries 4L..4L+3 of the block and stores entry
  // k at [k % 4][k / 4], so the lane with k parity h reads the offsets of 4
  // consecutive MFMA steps as one 16-byte LDS read.  (The slot is private to
  // the wave and LDS operations of a wave complete in order.)
  if (!linear) {
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

  // A: packed [subtile][kb][group][lane] float4 (launch_pack_lat).
  const float4* __restrict__ ap = reinterpret_cast<const float4*>(d.apk);
  float4 av[LGROUPS][MI];
#pragma unroll
  for (int g = 0; g < LGROUPS; g++)
#pragma unroll
    for (int mi = 0; mi < MI; mi++) {
      av[g][mi] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (g < ng && sub0 + mi < subs)
        av[g][mi] = ap[(((int64_t)(sub0 + mi) * nkb + kb) * LGROUPS + g) * 64 + lane];
    }

  const int n = n0 + c;
  uint32_t vcol = DMA_OOB;
  int img = 0, p = 0, oy = 0, ox = 0;
  if (n < N) {
    img = fdiv(n, d.fdP);
    p = n - img * d.P;
    oy = fdiv(p, d.fdOW);
    ox = p - oy * d.OW;
    vcol = (uint32_t)(((int64_t)img * d.x_img + (int64_t)oy * d.ystride + (int64_t)ox * d.xstride) * 4);
  }
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)d.x, 0, (int)d.x_bytes, 0x00020000);

  wait();

  // B: step s = 4g + j covers k = k0 + 4s + h for this lane.
  float bv[LKC / 4];
#pragma unroll
  for (int g = 0; g < LGROUPS; g++) {
    bv[4 * g] = bv[4 * g + 1] = bv[4 * g + 2] = bv[4 * g + 3] = 0.f;
    if (g < ng) {
      uint32_t ko[4];
      if (linear) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const int k = k0 + 16 * g + 4 * j + h;
          ko[j] = k < K ? (uint32_t)k * (uint32_t)d.kstride * 4u : DMA_OOB;
        }
      } else {
        const uint4 t = *(const uint4*)&ktl[h * 64 + 4 * g];
        ko[0] = t.x;
        ko[1] = t.y;
        ko[2] = t.z;
        ko[3] = t.w;
      }
#pragma unroll
      for (int j = 0; j < 4; j++)
        bv[4 * g + j] = __uint_as_float(sc1_ld ? __builtin_amdgcn_raw_buffer_load_b32(xr, vcol + ko[j], 0, kLoadSc1)
                                               : __builtin_amdgcn_raw_buffer_load_b32(xr, vcol + ko[j], 0, 0));
    }
  }

  lat_f32x4 acc[MI];
#pragma unroll
  for (int mi = 0; mi < MI; mi++) acc[mi] = (lat_f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int g = 0; g < LGROUPS; g++) {
    if (g < ng) {
#pragma unroll
      for (int j = 0; j < 4; j++)
#pragma unroll
        for (int mi = 0; mi < MI; mi++)
          acc[mi] = __builtin_amdgcn_mfma_f32_16x16x4f32(lat_f4(av[g][mi], j), bv[4 * g + j], acc[mi], 0, 0, 0);
    }
  }

  // Epilogue operands, issued before any store (vmcnt retires in order).
  // Accumulator element r of lane (c, h) is row 4h + r, column c.
  float bias_v[MI][4], res_v[MI][4];
  const int64_t rbase = (int64_t)img * d.res_img + p;
#pragma unroll
  for (int mi = 0; mi < MI; mi++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int m = (sub0 + mi) * 16 + 4 * h + r;
      const int mc = min(m, M - 1);
      bias_v[mi][r] = d.bias ? d.bias[mc] : 0.f;
      res_v[mi][r] = 0.f;
      if (d.residual && n < N) {
        const float* rp = d.residual + rbase + (int64_t)mc * d.res_c;
        res_v[mi][r] = sc1_ld ? __hip_atomic_load(rp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *rp;
      }
    }
  const float cbv = (d.colbias && n < N) ? d.colbias[p] : 0.f;
  const float alpha = d.alpha;
  // End of K block 0: alpha * chain + bias (gemm.rs:1004-1050).
  auto first_block = [&](float a, float b) __attribute__((always_inline)) {
    float x = alpha == 1.f ? a : __fmul_rn(a, alpha);
    if (d.bias) x = __fadd_rn(x, b);
    return x;
  };

  lat_f32x4 sum[MI];
  if (nkb == 1) {
#pragma unroll
    for (int mi = 0; mi < MI; mi++)
#pragma unroll
      for (int r = 0; r < 4; r++) sum[mi][r] = first_block(acc[mi][r], bias_v[mi][r]);
  } else {
    // This block's chains to the workspace ([tile][kb][mi][lane] x 16 bytes,
    // as 8-byte agent-scope stores), drained before the arrival count; the
    // last block of the tile to arrive folds all chains in K order.
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
    if (prev != nkb - 1) return;
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
            sum[mi][r] = kb0 + i == 0 ? first_block(v[r], bias_v[mi][r]) : __fmaf_rn(v[r], alpha, sum[mi][r]);
        }
      }
    }
    if (lane == 0) __hip_atomic_store(d.counters + wt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  const bool act_relu = d.act == RTENHIP_ACT_RELU, act_clip = d.act == RTENHIP_ACT_CLIP;
  const bool act_gelu = d.act == RTENHIP_ACT_GELU;
  const float lo = d.act_lo, hi = d.act_hi;
  const int64_t obase = (int64_t)img * d.out_img + (int64_t)oy * d.out_row + ox + d.out_off;
  if (n < N) {
#pragma unroll
    for (int mi = 0; mi < MI; mi++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int m = (sub0 + mi) * 16 + 4 * h + r;
        float x = sum[mi][r];
        if (d.colbias) x = __fadd_rn(x, cbv);
        if (d.residual) x = __fadd_rn(x, res_v[mi][r]);
        if (act_gelu) {
          x = vm_gelu(x);
        } else {
          const float rl = fmaxf(x, 0.f);
          const float cl = x < lo ? lo : (x > hi ? hi : x);
          x = act_relu ? rl : (act_clip ? cl : x);
        }
        if (m < M) {
          float* op = d.out + obase + (int64_t)m * d.out_c;
          if (sc1_st)
            __hip_atomic_store(op, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          else
            *op = x;
        }
      }
  }
  if (CHAIN) {
    // Every store of the tile drained, then one lane publishes it.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    done();
  }
}

}  // namespace rtenhip
