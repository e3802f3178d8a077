// Fused attention: MatMul(Q, K^T) -> [Div|Mul by a scalar] -> [Add(mask)] ->
// Softmax(axis -1) -> MatMul(P, V) [-> Transpose], one workgroup per
// (batch, head), everything between the two GEMMs kept in LDS.
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
// Shapes: D = 64, S <= 128 and even (the graph executor checks this and runs
// the unfused operator sequence otherwise).
#include "common.h"
#include "vecmath.h"

#include <cfloat>

namespace rtenhip {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int AT_D = 64;
constexpr int AT_S = 128;       // max sequence length (query rows and keys)
constexpr int QS = AT_D + 1;    // LDS row strides (+1: conflict-free columns)
constexpr int KS = AT_S + 1;
constexpr int VS = AT_D + 1;
constexpr int PS = AT_S + 1;
constexpr int Q_FLOATS = AT_S * QS;
constexpr int K_FLOATS = AT_D * KS;
constexpr int V_FLOATS = AT_S * VS;
static_assert(AT_S * PS <= Q_FLOATS + K_FLOATS, "P reuses the Q and K^T regions");

constexpr int AT_THREADS = 512;  // 8 waves: two per SIMD

__global__ __launch_bounds__(AT_THREADS) void attention_kernel(AttnDesc d) {
  __shared__ float lds[Q_FLOATS + K_FLOATS + V_FLOATS];
  float* Qs = lds;                 // [i][k]
  float* Kt = lds + Q_FLOATS;      // [k = dim][j]
  float* Vs = Kt + K_FLOATS;       // [j][n = dim]
  float* P = lds;                  // [i][j], over Q and K^T once the scores exist
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int half = lane >> 5, l32 = lane & 31;
  const int bh = blockIdx.x;
  const int b = bh / d.H, h = bh - b * d.H;
  const int S = d.S;

  const float* q = d.q + b * d.q_b + h * d.q_h;
  const float* kt = d.k + b * d.k_b + h * d.k_h;
  const float* v = d.v + b * d.v_b + h * d.v_h;

  // Stage Q, K^T and V (zero rows / columns past S); rows of 64 contiguous
  // floats are read as float4 when 16-byte aligned.
  const bool q4 = ((uintptr_t)q % 16 == 0) && d.q_s % 4 == 0;
  const bool v4 = ((uintptr_t)v % 16 == 0) && d.v_s % 4 == 0;
  const bool k4 = d.k_d == 1 && ((uintptr_t)kt % 16 == 0) && d.k_s % 4 == 0;
  for (int t = tid; t < AT_S * (AT_D / 4); t += AT_THREADS) {
    const int i = t >> 4, c = (t & 15) * 4;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), w = a, kk = a;
    if (i < S) {
      const float* qp = q + (int64_t)i * d.q_s + c;
      const float* vp = v + (int64_t)i * d.v_s + c;
      a = q4 ? *(const float4*)qp : make_float4(qp[0], qp[1], qp[2], qp[3]);
      w = v4 ? *(const float4*)vp : make_float4(vp[0], vp[1], vp[2], vp[3]);
      if (k4) {
        kk = *(const float4*)(kt + (int64_t)i * d.k_s + c);
      } else {
        const float* kp = kt + (int64_t)i * d.k_s + (int64_t)c * d.k_d;
        kk = make_float4(kp[0], kp[d.k_d], kp[2 * d.k_d], kp[3 * d.k_d]);
      }
    }
    float* qd = Qs + i * QS + c;
    qd[0] = a.x; qd[1] = a.y; qd[2] = a.z; qd[3] = a.w;
    float* vd = Vs + i * VS + c;
    vd[0] = w.x; vd[1] = w.y; vd[2] = w.z; vd[3] = w.w;
    Kt[(c + 0) * KS + i] = kk.x;
    Kt[(c + 1) * KS + i] = kk.y;
    Kt[(c + 2) * KS + i] = kk.z;
    Kt[(c + 3) * KS + i] = kk.w;
  }
  __syncthreads();

  // Scores: wave (rg, cg) computes query rows 32*rg .. +31 against keys
  // 64*cg .. +63 (two 32-key tiles), K = 64.
  const int rg = wave & 3, cg = wave >> 2;
  const int r0 = rg * 32;
  const bool rows = r0 < S;
  f32x16 acc[2];
  acc[0] = (f32x16){0};
  acc[1] = (f32x16){0};
  if (rows) {
#pragma unroll 8
    for (int s = 0; s < AT_D / 2; s++) {
      const int k = 2 * s + half;
      const float a = Qs[(r0 + l32) * QS + k];
      acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, Kt[k * KS + cg * 64 + l32], acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, Kt[k * KS + cg * 64 + 32 + l32], acc[1], 0, 0, 0);
    }
  }
  __syncthreads();  // every wave is done with Q and K^T: P overwrites them

  const float* mrow = d.mask ? d.mask + b * d.m_b + h * d.m_h : nullptr;
  if (rows) {
#pragma unroll
    for (int t = 0; t < 2; t++) {
      const int j = cg * 64 + t * 32 + l32;
#pragma unroll
      for (int e = 0; e < 16; e++) {
        const int i = r0 + (e & 3) + 8 * (e >> 2) + 4 * half;
        float x = acc[t][e];
        if (d.scale_op == 1)
          x = __fdiv_rn(x, d.scale);
        else if (d.scale_op == 2)
          x = __fmul_rn(x, d.scale);
        if (mrow && j < S && i < S) x = __fadd_rn(x, mrow[(int64_t)i * d.m_i + (int64_t)j * d.m_j]);
        P[i * PS + j] = x;
      }
    }
  }
  __syncthreads();

  // Softmax, eight lanes per row: lane c of a row's group owns the
  // elements j = c (mod 8), i.e. exactly the reference's partial-sum chain c.
  {
    const int c = lane & 7;
#pragma unroll
    for (int round = 0; round < AT_S / 64; round++) {
      const int i = round * 64 + wave * 8 + (lane >> 3);
      float* pr = P + i * PS;
      const bool live = i < S;
      float m = -FLT_MAX;
      if (live)
        for (int j = c; j < S; j += 8) m = rust_max(m, pr[j]);
      m = rust_max(m, __shfl_xor(m, 1));
      m = rust_max(m, __shfl_xor(m, 2));
      m = rust_max(m, __shfl_xor(m, 4));
      float part = 0.f;
      if (live)
        for (int j = c; j < S; j += 8) {
          const float e = vm_exp(__fsub_rn(pr[j], m));
          pr[j] = e;
          part = __fadd_rn(part, e);
        }
      float sum = 0.f;
      const int base = lane & ~7;
#pragma unroll
      for (int u = 0; u < 8; u++) sum = __fadd_rn(sum, __shfl(part, base + u));
      if (live)
        for (int j = c; j < S; j += 8) pr[j] = __fdiv_rn(pr[j], sum);
    }
  }
  __syncthreads();
  if (!rows) return;

  // Output: wave (rg, cg) computes rows 32*rg .. +31, head dims 32*cg .. +31
  // of P [S][S] @ V [S][64], K = S.
  f32x16 o = (f32x16){0};
#pragma unroll 8
  for (int s = 0; s < S / 2; s++) {
    const int k = 2 * s + half;
    o = __builtin_amdgcn_mfma_f32_32x32x2f32(P[(r0 + l32) * PS + k], Vs[k * VS + cg * 32 + l32], o,
                                             0, 0, 0);
  }
  float* out = d.out + b * d.o_b + h * d.o_h + cg * 32 + l32;
#pragma unroll
  for (int e = 0; e < 16; e++) {
    const int i = r0 + (e & 3) + 8 * (e >> 2) + 4 * half;
    if (i < S) out[(int64_t)i * d.o_s] = o[e];
  }
}

bool attention_fast_ok(const AttnDesc& d) {
  return d.D == AT_D && d.S >= 2 && d.S <= AT_S && d.S % 2 == 0 && d.B > 0 && d.H > 0 &&
         (int64_t)d.B * d.H < (int64_t(1) << 31);
}

rtenhip_status launch_attention(const AttnDesc& d, hipStream_t s) {
  if (!attention_fast_ok(d)) return fail(RTENHIP_UNSUPPORTED_VALUE, "attention shape not supported");
  hipLaunchKernelGGL(attention_kernel, dim3((unsigned)(d.B * d.H)), dim3(AT_THREADS), 0, s, d);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

}  // namespace rtenhip
