// Fused attention: MatMul(Q, K^T) -> [Div|Mul by a scalar] -> [Add(mask)] ->
// Softmax(axis -1) -> MatMul(P, V) [-> Transpose] for one (batch, head) per
// workgroup, with the scores and probabilities kept in registers.
//
// The reference runs these as separate operators (src/ops/matmul.rs:123-239,
// src/ops/binary_elementwise.rs, src/ops/norm.rs:332-448); this kernel keeps
// their arithmetic exactly:
//  - each score is the K = D chain of the batched gemm (one KC block, fma in k
//    order from +0; v_mfma_f32_32x32x2_f32 is bitwise that chain);
//  - then s / c (or s * c) and s + mask as separately rounded f32 ops;
//  - softmax as vec_softmax_in_place (rten-vecmath/src/softmax.rs:14-56):
//    max from f32::MIN, e = exp(s - max), eight partial sums over j = c (mod 8)
//    in index order folded 0 + p0 + ... + p7, p = e / sum;
//  - each output is the K = S chain of the second gemm.
//
// Mapping (4 waves): wave w owns query rows 32w .. 32w + 31 from the scores to
// the stores, so only K and V go through LDS (65 KB: two workgroups per CU)
// and the staging barrier is the only one.
//  - Scores are computed transposed, S^T = K Q^T (K rows are the MFMA's A
//    operand): lane (l, h) holds, for query row 32w + l, the keys
//    j = 32t + 8g + 4h + c of the four 32-key tiles t (g, c < 4).
//  - The reference's softmax chain j mod 8 is then lane-local: chains 0-3 live
//    in half 0 (chain c), chains 4-7 in half 1, each visited in increasing j.
//  - P is the second MFMA's A operand straight from registers: step k takes
//    key k from half 0 and key k + 1 from half 1, one half-wave swap per pair
//    of values.
// Shapes: D = 64, S <= 128 and even (the graph executor checks this and runs
// the unfused operator sequence otherwise).
#include "common.h"
#include "packed_a.h"
#include "vecmath.h"

#include <cfloat>
#include <cmath>

namespace rtenhip {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int AT_D = 64;
constexpr int AT_S = 128;        // max sequence length (query rows and keys)
constexpr int KS = AT_D + 1;     // K rows [j][k]: odd stride, conflict-free columns
constexpr int VS = AT_D;         // V rows [k][n]: each half-wave reads one row
constexpr int AT_THREADS = 256;  // 4 waves

// FULL: S == AT_S, every key and row guard folds away at compile time.
template <bool FULL>
__global__ __launch_bounds__(AT_THREADS, 2) void attention_kernel(AttnDesc d) {
  __shared__ float Ks[AT_S * KS];
  __shared__ float Vs[AT_S * VS];
  __shared__ float Ms[AT_S];  // the mask row when it does not depend on the query row (m_i == 0)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int bh = blockIdx.x;
  const int b = bh / d.H, hd = bh - b * d.H;
  const int S = FULL ? AT_S : d.S;

  const float* q = d.q + b * d.q_b + hd * d.q_h;
  const float* kt = d.k + b * d.k_b + hd * d.k_h;
  const float* v = d.v + b * d.v_b + hd * d.v_h;

  // Stage K (row = key) and V (row = key), zero rows past S; rows of 64
  // contiguous floats are read as float4 when 16-byte aligned.  All of a
  // thread's loads are issued before its LDS stores (one memory round trip
  // for the whole staging, not one per row group).
  const bool v4 = ((uintptr_t)v % 16 == 0) && d.v_s % 4 == 0;
  const bool k4 = d.k_d == 1 && ((uintptr_t)kt % 16 == 0) && d.k_s % 4 == 0;
  constexpr int ST = AT_S * (AT_D / 4) / AT_THREADS;  // float4 positions per thread (8)
  float4 kk[ST], vv[ST];
#pragma unroll
  for (int u = 0; u < ST; u++) {
    const int t = tid + u * AT_THREADS;
    const int j = t >> 4, c = (t & 15) * 4;
    kk[u] = vv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (FULL || j < S) {
      const float* vp = v + (int64_t)j * d.v_s + c;
      vv[u] = v4 ? *(const float4*)vp : make_float4(vp[0], vp[1], vp[2], vp[3]);
      if (k4) {
        kk[u] = *(const float4*)(kt + (int64_t)j * d.k_s + c);
      } else {
        const float* kp = kt + (int64_t)j * d.k_s + (int64_t)c * d.k_d;
        kk[u] = make_float4(kp[0], kp[d.k_d], kp[2 * d.k_d], kp[3 * d.k_d]);
      }
    }
  }
  // A query-independent mask row ([B, 1, 1, S], BERT's) is staged with K and
  // V, so the softmax phase reads it from LDS instead of making 64 global
  // loads per lane on the critical path.
  const bool mask_lds = d.mask && d.m_i == 0;
  float mv = 0.f;
  if (mask_lds && tid < S) mv = d.mask[b * d.m_b + hd * d.m_h + (int64_t)tid * d.m_j];
#pragma unroll
  for (int u = 0; u < ST; u++) {
    const int t = tid + u * AT_THREADS;
    const int j = t >> 4, c = (t & 15) * 4;
    float* kd = Ks + j * KS + c;
    kd[0] = kk[u].x;
    kd[1] = kk[u].y;
    kd[2] = kk[u].z;
    kd[3] = kk[u].w;
    *(float4*)(Vs + j * VS + c) = vv[u];
  }
  if (mask_lds && tid < S) Ms[tid] = mv;
  const int i0 = wave * 32;
  const int i = i0 + l32;  // this lane's query row
  const bool row_ok = FULL || i < S;
  // This lane's Q fragment, qf[s] = Q[i][2s + h] (the MFMA's B operand),
  // loaded while the K / V stores land.
  float qf[AT_D / 2];
  if (((uintptr_t)q % 16) == 0 && d.q_s % 4 == 0) {
    // The whole row as 16 float4s (16 load instructions instead of 32 strided
    // dwords); this lane keeps elements h and h + 2 of each 4.
    const float4* qr4 = reinterpret_cast<const float4*>(q + (int64_t)(row_ok ? i : 0) * d.q_s);
    float4 q4[AT_D / 4];
#pragma unroll
    for (int m = 0; m < AT_D / 4; m++) q4[m] = qr4[m];
#pragma unroll
    for (int m = 0; m < AT_D / 4; m++) {
      qf[2 * m] = row_ok ? (h ? q4[m].y : q4[m].x) : 0.f;
      qf[2 * m + 1] = row_ok ? (h ? q4[m].w : q4[m].z) : 0.f;
    }
  } else {
    const float* qr = q + (int64_t)(row_ok ? i : 0) * d.q_s + h;
#pragma unroll
    for (int s = 0; s < AT_D / 2; s++) qf[s] = row_ok ? qr[2 * s] : 0.f;
  }
  __syncthreads();
  if (i0 >= S) return;  // no barrier follows


  // acc[t][e]: score of (row i, key 32t + (e & 3) + 8(e >> 2) + 4h).
  f32x16 acc[4];
#pragma unroll
  for (int t = 0; t < 4; t++) acc[t] = (f32x16){0};
#pragma unroll
  for (int s = 0; s < AT_D / 2; s++) {
    const float* kr = Ks + l32 * KS + 2 * s + h;
#pragma unroll
    for (int t = 0; t < 4; t++)
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(kr[t * 32 * KS], qf[s], acc[t], 0, 0, 0);
  }

  // Scale and mask (separately rounded, as the Div|Mul and Add operators),
  // then the row max over the keys < S.
  const float* mrow =
      (d.mask && row_ok && !mask_lds) ? d.mask + b * d.m_b + hd * d.m_h + (int64_t)i * d.m_i : nullptr;
  float m = -FLT_MAX;
#pragma unroll
  for (int t = 0; t < 4; t++)
#pragma unroll
    for (int e = 0; e < 16; e++) {
      const int j = 32 * t + (e & 3) + 8 * (e >> 2) + 4 * h;
      float x = acc[t][e];
      if (d.scale_op == 1)
        x = __fdiv_rn(x, d.scale);
      else if (d.scale_op == 2)
        x = __fmul_rn(x, d.scale);
      if (FULL || j < S) {
        if (mask_lds) x = __fadd_rn(x, Ms[j]);
        else if (mrow) x = __fadd_rn(x, mrow[(int64_t)j * d.m_j]);
        m = rust_max(m, x);
      }
      acc[t][e] = x;
    }
  m = rust_max(m, __shfl_xor(m, 32));

  // e = exp(x - max) and the eight partial sums: chain 4h + c runs over
  // j = 32t + 8g + 4h + c in increasing j (t, then g).
  float part[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 4; t++)
#pragma unroll
    for (int g = 0; g < 4; g++)
#pragma unroll
      for (int c = 0; c < 4; c++)
        if (FULL || 32 * t + 8 * g + 4 * h + c < S) {
          const float ex = vm_exp(__fsub_rn(acc[t][4 * g + c], m));
          acc[t][4 * g + c] = ex;
          part[c] = __fadd_rn(part[c], ex);
        }
  // 0 + p0 + ... + p7 (half 0 holds p0..p3, half 1 p4..p7): both halves fold
  // the same eight values in the same order.
  float other[4];
#pragma unroll
  for (int c = 0; c < 4; c++) other[c] = __shfl_xor(part[c], 32);
  float sum = 0.f;
#pragma unroll
  for (int c = 0; c < 4; c++) sum = __fadd_rn(sum, h ? other[c] : part[c]);
#pragma unroll
  for (int c = 0; c < 4; c++) sum = __fadd_rn(sum, h ? part[c] : other[c]);
#pragma unroll
  for (int t = 0; t < 4; t++)
#pragma unroll
    for (int e = 0; e < 16; e++)
      if (FULL || 32 * t + (e & 3) + 8 * (e >> 2) + 4 * h < S) acc[t][e] = __fdiv_rn(acc[t][e], sum);

  // out[i][n] = sum over k < S of P[i][k] V[k][n] in k order.  Keys kb + 0..3
  // of an 8-key group are in half 0, kb + 4..7 in half 1; MFMA step k needs
  // key k in half 0 and key k + 1 in half 1.
  f32x16 o[2];
  o[0] = (f32x16){0};
  o[1] = (f32x16){0};
#pragma unroll
  for (int t = 0; t < 4; t++)
#pragma unroll
    for (int g = 0; g < 4; g++) {
      const int kb = 32 * t + 8 * g;
      if (FULL || kb < S) {
        const float s01 = __shfl_xor(h ? acc[t][4 * g] : acc[t][4 * g + 1], 32);
        const float s23 = __shfl_xor(h ? acc[t][4 * g + 2] : acc[t][4 * g + 3], 32);
        const float a[4] = {h ? s01 : acc[t][4 * g], h ? s23 : acc[t][4 * g + 2],
                            h ? acc[t][4 * g + 1] : s01, h ? acc[t][4 * g + 3] : s23};
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const int k = kb + 2 * u;  // S even: k < S implies k + 1 < S
          if (FULL || k < S) {
            const float* vr = Vs + (k + h) * VS + l32;
            o[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u], vr[0], o[0], 0, 0, 0);
            o[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u], vr[32], o[1], 0, 0, 0);
          }
        }
      }
    }
  float* dst = d.out + b * d.o_b + hd * d.o_h + l32;
  if (!d.pk_only) {
#pragma unroll
    for (int n2 = 0; n2 < 2; n2++)
#pragma unroll
      for (int e = 0; e < 16; e++) {
        const int r = i0 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (FULL || r < S) dst[(int64_t)r * d.o_s + 32 * n2] = o[n2][e];
      }
  }
  if (d.pk) {
    // Packed-A copy for the output projection: a lane quad (4g .. 4g + 3)
    // holds a 4 x 4 block (rows e & 3 of group e >> 2, one column per lane);
    // transposed through 4 rotations so lane 4g + c holds row c's 4 columns,
    // stored as one k-quad (store_packed_a4).  Same values, new places.
    const int c = l32 & 3, g4 = l32 & ~3;
#pragma unroll
    for (int n2 = 0; n2 < 2; n2++)
#pragma unroll
      for (int a = 0; a < 4; a++) {
        float w[4];
#pragma unroll
        for (int t = 0; t < 4; t++) {
          const int si = (c - t) & 3;  // element this lane sends in round t
          const float sv = si == 0 ? o[n2][4 * a] : si == 1 ? o[n2][4 * a + 1] : si == 2 ? o[n2][4 * a + 2] : o[n2][4 * a + 3];
          const float rv = __shfl(sv, h * 32 + g4 + ((c + t) & 3));
          const int di = (c + t) & 3;  // column of the received value
          if (t == 0) w[0] = w[1] = w[2] = w[3] = 0.f;
          w[0] = di == 0 ? rv : w[0];
          w[1] = di == 1 ? rv : w[1];
          w[2] = di == 2 ? rv : w[2];
          w[3] = di == 3 ? rv : w[3];
        }
        const int r = i0 + c + 8 * a + 4 * h;
        if (FULL || r < S)
          store_packed_a4(d.pk, d.pk_lbm, d.pk_lbk, d.pk_tiles_k, (int64_t)b * S + r, hd * AT_D + 32 * n2 + g4,
                          make_float4(w[0], w[1], w[2], w[3]));
      }
  }
}

bool attention_fast_ok(const AttnDesc& d) {
  return d.D == AT_D && d.S >= 2 && d.S <= AT_S && d.S % 2 == 0 && d.B > 0 && d.H > 0 &&
         (int64_t)d.B * d.H < (int64_t(1) << 31);
}

rtenhip_status launch_attention(const AttnDesc& d, hipStream_t s) {
  if (!attention_fast_ok(d)) return fail(RTENHIP_UNSUPPORTED_VALUE, "attention shape not supported");
  // x / 2^k and x * 2^-k are the same correctly rounded value (both scale
  // the exact x by an exact power of two), so a power-of-two divisor -- BERT's
  // sqrt(64) = 8 -- becomes a multiply: bit-identical, no division per score.
  AttnDesc e = d;
  int ex = 0;
  if (d.scale_op == 1 && std::frexp(d.scale, &ex) == 0.5f && ex > -120 && ex < 120) {
    e.scale_op = 2;
    e.scale = std::ldexp(1.f, 1 - ex);
  }
  if (d.S == AT_S)
    hipLaunchKernelGGL(attention_kernel<true>, dim3((unsigned)(d.B * d.H)), dim3(AT_THREADS), 0, s, e);
  else
    hipLaunchKernelGGL(attention_kernel<false>, dim3((unsigned)(d.B * d.H)), dim3(AT_THREADS), 0, s, e);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

}  // namespace rtenhip
