// Softmax and LayerNormalization: one wavefront per row.
//
// Both reproduce the reference's summation order so results are bit-exact:
//  - Softmax = vec_softmax_in_place (rten-vecmath/src/softmax.rs:14-56) on the
//    AVX2 width (8 lanes): max from f32::MIN, e_i = exp(x_i - max), eight
//    partial sums over i = j (mod 8) in index order, folded 0 + p0 + ... + p7,
//    then y_i = e_i / sum.  The exps run on all 64 lanes; only the eight short
//    chains and the final fold are serial.
//  - LayerNorm = layer_normalization (src/ops/norm.rs:245-299): mean via
//    slice_sum (8-element chunks, src/slice_reductions.rs:37-53), x - mean,
//    1/sqrt(iter_sum(d*d)/n + eps) (iter_sum: groups of 4,
//    slice_reductions.rs:57-84), then * inv, * scale, + bias.
#include "common.h"
#include "packed_a.h"
#include "vecmath.h"

#include <algorithm>
#include <cfloat>
#include <cstdlib>

namespace rtenhip {

constexpr int ROWS_PER_BLOCK = 4;

// rows handled by one wave each; `lds` holds ROWS_PER_BLOCK * len floats.
__global__ __launch_bounds__(256) void softmax_kernel(const float* __restrict__ x,
                                                      float* __restrict__ y, int64_t rows,
                                                      int len, int use_lds) {
  extern __shared__ float lds[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * ROWS_PER_BLOCK + wave;
  const bool active = row < rows;
  const float* xr = x + (active ? row : 0) * len;
  float* yr = y + (active ? row : 0) * len;
  float* buf = use_lds ? lds + wave * len : yr;

  float m = -FLT_MAX;
  if (active)
    for (int i = lane; i < len; i += 64) m = rust_max(m, xr[i]);
  for (int off = 32; off > 0; off >>= 1) m = rust_max(m, __shfl_xor(m, off));
  if (active)
    for (int i = lane; i < len; i += 64) buf[i] = vm_exp(__fsub_rn(xr[i], m));
  __syncthreads();
  float part = 0.f;
  if (active && lane < 8)
    for (int i = lane; i < len; i += 8) part = __fadd_rn(part, buf[i]);
  float sum = 0.f;
  for (int j = 0; j < 8; j++) sum = __fadd_rn(sum, __shfl(part, j));
  if (active)
    for (int i = lane; i < len; i += 64) yr[i] = __fdiv_rn(buf[i], sum);
}

rtenhip_status launch_softmax(const float* x, float* y, int64_t rows, int64_t len,
                              hipStream_t s) {
  if (rows == 0 || len == 0) return RTENHIP_OK;
  const int use_lds = len <= 4096;
  // Without LDS the exps are staged in y itself; in-place (x == y) is safe
  // because each row is read fully (max) before any write... except the
  // exp pass reads x_i and writes y_i at the same index, which is fine.
  size_t shmem = use_lds ? (size_t)ROWS_PER_BLOCK * len * sizeof(float) : 0;
  int64_t blocks = (rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK;
  hipLaunchKernelGGL(softmax_kernel, dim3((unsigned)blocks), dim3(256), shmem, s, x, y, rows,
                     (int)len, use_lds);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

// Per-wave LDS floats of layer_norm_kernel's partial sums (multiple of 4).
__host__ __device__ constexpr int ln_part_stride(int len) { return (len / 4 + 8 + 3) & ~3; }

// 0 + p[0] + p[1] + ... + p[n-1], strictly in index order (the reference's
// serial fold); the LDS reads are issued 16 at a time as 16-byte loads so the
// chain waits on adds, not on LDS latency.  p is 16-byte aligned.
__device__ __forceinline__ float serial_sum(const float* p, int n) {
  float acc = 0.f;
  int i = 0;
  for (; i + 16 <= n; i += 16) {
    float4 q[4];
#pragma unroll
    for (int j = 0; j < 4; j++) q[j] = *(const float4*)(p + i + 4 * j);
#pragma unroll
    for (int j = 0; j < 4; j++) {
      acc = __fadd_rn(acc, q[j].x);
      acc = __fadd_rn(acc, q[j].y);
      acc = __fadd_rn(acc, q[j].z);
      acc = __fadd_rn(acc, q[j].w);
    }
  }
  for (; i < n; i++) acc = __fadd_rn(acc, p[i]);
  return acc;
}

__global__ __launch_bounds__(256) void layer_norm_kernel(const float* __restrict__ x,
                                                         float* __restrict__ y, int64_t rows,
                                                         int len, const float* __restrict__ scale,
                                                         const float* __restrict__ bias,
                                                         float eps) {
  extern __shared__ float lds[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * ROWS_PER_BLOCK + wave;
  const bool active = row < rows;
  const float* xr = x + (active ? row : 0) * len;
  float* yr = y + (active ? row : 0) * len;
  // Per-wave scratch: chunk/group partial sums (len/4 + 2 floats max), each
  // wave's slice 16-byte aligned for the vector reads of the serial folds.
  float* part = lds + wave * ln_part_stride(len);

  // slice_sum: full 8-chunks in parallel, then a serial fold.
  const int nchunks = len / 8;
  if (active)
    for (int c = lane; c < nchunks; c += 64) {
      const float* p = xr + 8 * c;
      float z0 = __fadd_rn(p[0], p[4]), z1 = __fadd_rn(p[1], p[5]);
      float z2 = __fadd_rn(p[2], p[6]), z3 = __fadd_rn(p[3], p[7]);
      part[c] = __fadd_rn(__fadd_rn(__fadd_rn(z0, z1), z2), z3);
    }
  __syncthreads();
  float mean = 0.f;
  if (lane == 0 && active) {
    float total = serial_sum(part, nchunks);
    if (nchunks * 8 < len) {
      float t = 0.f;
      for (int i = nchunks * 8; i < len; i++) t = __fadd_rn(t, xr[i]);
      total = __fadd_rn(total, t);
    }
    mean = __fdiv_rn(total, (float)len);
  }
  mean = __shfl(mean, 0);
  __syncthreads();

  // iter_sum of squares of d = x - mean: groups of 4 while n > 4, then the tail.
  const int ngroups = len > 4 ? (len - 1) / 4 : 0;
  if (active)
    for (int g = lane; g < ngroups; g += 64) {
      const float* p = xr + 4 * g;
      float d0 = __fsub_rn(p[0], mean), d1 = __fsub_rn(p[1], mean);
      float d2 = __fsub_rn(p[2], mean), d3 = __fsub_rn(p[3], mean);
      float ab = __fadd_rn(__fmul_rn(d0, d0), __fmul_rn(d1, d1));
      float cd = __fadd_rn(__fmul_rn(d2, d2), __fmul_rn(d3, d3));
      part[g] = __fadd_rn(ab, cd);
    }
  __syncthreads();
  float inv = 0.f;
  if (lane == 0 && active) {
    float sum = serial_sum(part, ngroups);
    for (int i = 4 * ngroups; i < len; i++) {
      float d = __fsub_rn(xr[i], mean);
      sum = __fadd_rn(sum, __fmul_rn(d, d));
    }
    float ms = __fdiv_rn(sum, (float)len);
    inv = __fdiv_rn(1.f, sqrt_rn(__fadd_rn(ms, eps)));
  }
  inv = __shfl(inv, 0);
  if (active)
    for (int i = lane; i < len; i += 64) {
      float v = __fmul_rn(__fsub_rn(xr[i], mean), inv);
      v = __fmul_rn(v, scale[i]);
      if (bias) v = __fadd_rn(v, bias[i]);
      yr[i] = v;
    }
}

// 0 + p[0] + p[s] + ... + p[(n-1)s] in index order, loads issued 8 ahead.
__device__ __forceinline__ float strided_sum(const float* p, int s, int n) {
  float acc = 0.f;
  int i = 0;
  for (; i + 8 <= n; i += 8) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; j++) v[j] = p[(i + j) * s];
#pragma unroll
    for (int j = 0; j < 8; j++) acc = __fadd_rn(acc, v[j]);
  }
  for (; i < n; i++) acc = __fadd_rn(acc, p[i * s]);
  return acc;
}

// The same fold over n contiguous values (n known at compile time), read as
// 16-byte LDS loads -- a quarter of the LDS instructions of the strided form
// (the fold's cost is its reads, not its adds).  Reads round n up to a
// multiple of 4; the values past n are not added.
template <int N>
__device__ __forceinline__ float contiguous_sum_n(const float* p) {
  constexpr int NV = (N + 3) / 4;
  float4 v[NV];
#pragma unroll
  for (int i = 0; i < NV; i++) v[i] = reinterpret_cast<const float4*>(p)[i];
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < N; i++) {
    const float4& q = v[i >> 2];
    acc = __fadd_rn(acc, (i & 3) == 0 ? q.x : (i & 3) == 1 ? q.y : (i & 3) == 2 ? q.z : q.w);
  }
  return acc;
}

// Row stride (floats) of the LayerNorm rows kernel's partial sums: the
// groups rounded up to whole float4s, plus one float4 of padding.
__host__ __device__ inline int ln_part_row_stride(int len) { return ((((len - 1) >> 2) + 3) & ~3) + 4; }
// LDS bytes of the rows kernel: R staged rows, R rows of partials, mean / inv.
inline size_t ln_rows_shm(int R, int64_t len) {
  return ((size_t)R * (len + 4) + (size_t)R * ln_part_row_stride((int)len) + 2 * (size_t)R) * sizeof(float);
}

// LayerNorm for len % 8 == 0 on 16-byte aligned rows, R rows per workgroup:
// the rows are staged in LDS with 16-byte copies, the 8-element chunk sums and
// the 4-element groups of squares are formed in parallel into LDS as
// [row][chunk], and thread r runs row r's two serial folds -- one VALU
// instruction advances R rows' chains, where layer_norm_kernel spends a whole
// wave instruction per add of one row.  Same operations in the same order.
// LEN > 0: instance for that row length (folds fully unrolled); 0: any.
// Timing experiments only (never set in a product build): 1 = no packed-A
// phase, 2 = no serial folds, 3 = no row-major output stores.
#ifndef RTENHIP_LN_EXPERIMENT
#define RTENHIP_LN_EXPERIMENT 0
#endif
// Rows per workgroup: min(16, RTENHIP_LN_ROWS_NUM / len) (8 at BERT's 768).
#ifndef RTENHIP_LN_ROWS_NUM
#define RTENHIP_LN_ROWS_NUM 6144
#endif

template <int LEN>
__global__ __launch_bounds__(256) void layer_norm_rows_kernel(
    const float* __restrict__ x, float* __restrict__ y, int64_t rows, int len_arg, int R,
    const float* __restrict__ scale, const float* __restrict__ bias, float eps, PackedOut pk) {
  const int len = LEN > 0 ? LEN : len_arg;
  extern __shared__ float4 lds4[];
  const int q = len >> 2;              // float4s per row
  const int nchunks = len >> 3;
  const int ngroups = (len - 1) >> 2;  // >= nchunks for len >= 8
  const int ps = ln_part_row_stride(len);  // [row][chunk] stride
  float* xs = reinterpret_cast<float*>(lds4);
  // Rows are q + 1 float4s apart in LDS (one float4 of padding): the
  // packed-A phase reads the same column of 8 consecutive rows, which at a
  // stride of len (a multiple of 32 dwords) would share one bank.
  const int qs = q + 1;
  float* part = xs + R * (len + 4);
  float* stat = part + R * ps;         // mean[R], inv[R]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row0 = (int64_t)blockIdx.x * R;
  const int64_t left = rows - row0;
  const int nr = left < R ? (int)left : R;
  const float4* x4 = reinterpret_cast<const float4*>(x + row0 * len);
  // LEN instances: the lane's scale / bias float4s (columns lane + 64 i) are
  // loaded first, in flight with the staging (loaded per output row instead,
  // each row's stores would wait on a round trip).
  constexpr int NCP = (LEN > 0 && LEN % 256 == 0) ? LEN / 256 : 1;
  float4 scp[NCP], bbp[NCP];
  if constexpr (LEN > 0 && LEN % 256 == 0) {
    const float4* s4p = reinterpret_cast<const float4*>(scale);
    const float4* b4p = reinterpret_cast<const float4*>(bias);
#pragma unroll
    for (int i = 0; i < NCP; i++) {
      scp[i] = s4p[lane + 64 * i];
      bbp[i] = bias ? b4p[lane + 64 * i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  // Staging: a thread's loads are issued together (8 in flight), then stored
  // to LDS -- a load-then-store loop would pay one memory round trip per trip.
  {
    // (Loads past the rows read a clamped in-range index: unconditional, so
    // no branch or wait sits between them; only the LDS stores are guarded.)
    const int n4 = nr * q;
    for (int t = threadIdx.x; t < n4; t += 8 * 256) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; u++) v[u] = x4[min(t + u * 256, n4 - 1)];
#pragma unroll
      for (int u = 0; u < 8; u++)  // an unconditional use: keeps the loads out of the guarded stores
        asm volatile("" ::"v"(v[u].x), "v"(v[u].y), "v"(v[u].z), "v"(v[u].w));
#pragma unroll
      for (int u = 0; u < 8; u++)
        if (t + u * 256 < n4) {
          const int e = t + u * 256, rr = e / q;
          lds4[rr * qs + (e - rr * q)] = v[u];
        }
    }
  }
  __syncthreads();
  // slice_sum: chunk c = ((x0 + x4) + (x1 + x5)) + (x2 + x6)) + (x3 + x7)
  for (int r = wave; r < nr; r += 4)
    for (int c = lane; c < nchunks; c += 64) {
      const float4 a = lds4[r * qs + 2 * c], b = lds4[r * qs + 2 * c + 1];
      const float z0 = __fadd_rn(a.x, b.x), z1 = __fadd_rn(a.y, b.y);
      const float z2 = __fadd_rn(a.z, b.z), z3 = __fadd_rn(a.w, b.w);
      part[r * ps + c] = __fadd_rn(__fadd_rn(__fadd_rn(z0, z1), z2), z3);
    }
  __syncthreads();
  if ((int)threadIdx.x < nr) {
    const int r = threadIdx.x;
    float total;
    if constexpr (RTENHIP_LN_EXPERIMENT == 2)
      total = part[r * ps];
    else if constexpr (LEN > 0)
      total = contiguous_sum_n<LEN / 8>(part + r * ps);
    else
      total = strided_sum(part + r * ps, 1, nchunks);
    stat[r] = __fdiv_rn(total, (float)len);
  }
  __syncthreads();
  // iter_sum of (x - mean)^2: groups of 4, then the tail.
  for (int r = wave; r < nr; r += 4) {
    const float mean = stat[r];
    for (int g = lane; g < ngroups; g += 64) {
      const float4 v = lds4[r * qs + g];
      const float d0 = __fsub_rn(v.x, mean), d1 = __fsub_rn(v.y, mean);
      const float d2 = __fsub_rn(v.z, mean), d3 = __fsub_rn(v.w, mean);
      const float ab = __fadd_rn(__fmul_rn(d0, d0), __fmul_rn(d1, d1));
      const float cd = __fadd_rn(__fmul_rn(d2, d2), __fmul_rn(d3, d3));
      part[r * ps + g] = __fadd_rn(ab, cd);
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < nr) {
    const int r = threadIdx.x;
    const float mean = stat[r];
    float sum;
    if constexpr (RTENHIP_LN_EXPERIMENT == 2)
      sum = part[r * ps];
    else if constexpr (LEN > 0)
      sum = contiguous_sum_n<(LEN - 1) / 4>(part + r * ps);
    else
      sum = strided_sum(part + r * ps, 1, ngroups);
    for (int i = 4 * ngroups; i < len; i++) {
      const float d = __fsub_rn(xs[r * (len + 4) + i], mean);
      sum = __fadd_rn(sum, __fmul_rn(d, d));
    }
    const float ms = __fdiv_rn(sum, (float)len);
    stat[R + r] = __fdiv_rn(1.f, sqrt_rn(__fadd_rn(ms, eps)));
  }
  __syncthreads();
  float4* y4 = reinterpret_cast<float4*>(y + row0 * len);
  const float4* s4 = reinterpret_cast<const float4*>(scale);
  const float4* b4 = reinterpret_cast<const float4*>(bias);
  auto out_row = [&](int r, const float4* sc, const float4* bb, int c0, int nc) __attribute__((always_inline)) {
    const float mean = stat[r], inv = stat[R + r];
    for (int i = 0; i < nc; i++) {
      const int c = c0 + 64 * i;
      const float4 v = lds4[r * qs + c];
      float4 o;
      o.x = __fmul_rn(__fmul_rn(__fsub_rn(v.x, mean), inv), sc[i].x);
      o.y = __fmul_rn(__fmul_rn(__fsub_rn(v.y, mean), inv), sc[i].y);
      o.z = __fmul_rn(__fmul_rn(__fsub_rn(v.z, mean), inv), sc[i].z);
      o.w = __fmul_rn(__fmul_rn(__fsub_rn(v.w, mean), inv), sc[i].w);
      if (bias) {
        o.x = __fadd_rn(o.x, bb[i].x);
        o.y = __fadd_rn(o.y, bb[i].y);
        o.z = __fadd_rn(o.z, bb[i].z);
        o.w = __fadd_rn(o.w, bb[i].w);
      }
      if (RTENHIP_LN_EXPERIMENT != 3) y4[r * q + c] = o;
      if (pk.p) lds4[r * qs + c] = o;  // this thread's own element: no hazard
    }
  };
  if constexpr (LEN > 0 && LEN % 256 == 0) {
    for (int r = wave; r < nr; r += 4) out_row(r, scp, bbp, lane, NCP);
  } else {
    for (int r = wave; r < nr; r += 4)
      for (int c = lane; c < q; c += 64) {
        const float4 sc = s4[c], bb = bias ? b4[c] : make_float4(0.f, 0.f, 0.f, 0.f);
        out_row(r, &sc, &bb, c, 1);
      }
  }
  if (pk.p && RTENHIP_LN_EXPERIMENT != 1) {
    // The MatMul's packed A (packed_a.h): one 16-byte chunk per (k tile,
    // plane, row) with the row fastest, so consecutive threads write
    // consecutive chunks of a plane (rows are 16 bytes apart in it).
    __syncthreads();
    const int BK = 1 << pk.lbk, nq = BK >> 2;
    const int ktiles = (len + BK - 1) >> pk.lbk;
    const int total = nr * nq * ktiles;
    // (A full block of an instance has nr = R known at compile time (the host
    // picks R the same way): the index split below is then shifts and
    // multiplies instead of two integer divisions per chunk.)
    constexpr int RC = LEN > 0 ? (RTENHIP_LN_ROWS_NUM / LEN < 16 ? RTENHIP_LN_ROWS_NUM / LEN : 16) : 0;
    const bool rc = RC > 0 && nr == RC;
    for (int i = threadIdx.x; i < total; i += 256) {
      const int r = rc ? i % (RC > 0 ? RC : 1) : i % nr, t2 = rc ? i / (RC > 0 ? RC : 1) : i / nr;
      const int qq = t2 & (nq - 1), tk = t2 >> (pk.lbk - 2);
      const int kb = tk * BK + 8 * (qq >> 1) + (qq & 1);
      const float* xr = xs + r * (len + 4);
      const float4 v = make_float4(kb < len ? xr[kb] : 0.f, kb + 2 < len ? xr[kb + 2] : 0.f,
                                   kb + 4 < len ? xr[kb + 4] : 0.f, kb + 6 < len ? xr[kb + 6] : 0.f);
      const int64_t m = row0 + r;
      float* tb = pk.p + (((m >> pk.lbm) * pk.tiles_k + tk) << (pk.lbm + pk.lbk));
      *(float4*)(tb + (((int64_t)qq << pk.lbm) + (m & ((1 << pk.lbm) - 1))) * 4) = v;
    }
  }
}

bool layer_norm_rows_ok(const float* x, float* y, int64_t len, const float* scale, const float* bias) {
  if (len % 8 != 0 || (uintptr_t)x % 16 || (uintptr_t)y % 16 || (uintptr_t)scale % 16 ||
      (bias && (uintptr_t)bias % 16))
    return false;
  const int R = (int)std::max<int64_t>(1, std::min<int64_t>(16, RTENHIP_LN_ROWS_NUM / len));
  return ln_rows_shm(R, len) <= 64 * 1024;
}

rtenhip_status launch_layer_norm(const float* x, float* y, int64_t rows, int64_t len,
                                 const float* scale, const float* bias, float eps,
                                 hipStream_t s, const PackedOut* pk) {
  if (rows == 0 || len == 0) return RTENHIP_OK;
  if (pk && !layer_norm_rows_ok(x, y, len, scale, bias))
    return fail(RTENHIP_UNSUPPORTED_VALUE, "LayerNorm: packed output needs the rows kernel");
  const PackedOut pko = pk ? *pk : PackedOut{};
  const bool rows_ok = len % 8 == 0 && (uintptr_t)x % 16 == 0 && (uintptr_t)y % 16 == 0 &&
                       (uintptr_t)scale % 16 == 0 && (!bias || (uintptr_t)bias % 16 == 0);
  if (rows_ok) {
    static const int env_rows = [] {
      const char* e = getenv("RTENHIP_LN_ROWS");  // tuning experiments
      return e ? atoi(e) : 0;
    }();
    const int R = env_rows > 0 ? std::min(env_rows, 64)
                               : (int)std::max<int64_t>(1, std::min<int64_t>(16, RTENHIP_LN_ROWS_NUM / len));
    const size_t rshm = ln_rows_shm(R, len);
    if (rshm <= 64 * 1024) {
      const int64_t rblocks = (rows + R - 1) / R;
      // BERT-base / BERT-large widths get the unrolled-fold instances.
      auto kern = len == 768    ? layer_norm_rows_kernel<768>
                  : len == 1024 ? layer_norm_rows_kernel<1024>
                                : layer_norm_rows_kernel<0>;
      hipLaunchKernelGGL(kern, dim3((unsigned)rblocks), dim3(256), rshm, s, x, y, rows, (int)len, R,
                         scale, bias, eps, pko);
      RTENHIP_LAUNCH_CHECK();
      return RTENHIP_OK;
    }
  }
  size_t shmem = (size_t)ROWS_PER_BLOCK * ln_part_stride((int)len) * sizeof(float);
  if (shmem > 160 * 1024) return fail(RTENHIP_UNSUPPORTED_VALUE, "LayerNorm row too long");
  int64_t blocks = (rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK;
  hipLaunchKernelGGL(layer_norm_kernel, dim3((unsigned)blocks), dim3(256), shmem, s, x, y, rows,
                     (int)len, scale, bias, eps);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

// ReduceMean over the last axis (reduce.rs:270-286: reduce_slice = slice_sum
// / len).  One wave per row: lane j forms the sums of chunks j, j+64, ... (a
// full chunk as ((x0+x4) + (x1+x5)) + (x2+x6)) + (x3+x7), a partial one as a
// fold from 0, slice_reductions.rs:38-55); lane 0 then folds the chunk sums in
// order from 0 and divides by the row length.
__global__ __launch_bounds__(256) void reduce_mean_rows_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                               int64_t rows, int64_t len) {
  extern __shared__ float chunk_sums[];  // [4 waves][nchunks]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + wave;
  const int64_t nchunks = (len + 7) / 8;
  float* cs = chunk_sums + (int64_t)wave * nchunks;
  if (row < rows) {
    const float* xr = x + row * len;
    for (int64_t c = lane; c < nchunks; c += 64) {
      const int64_t b = c * 8;
      float sum;
      if (b + 8 <= len) {
        const float z0 = __fadd_rn(xr[b], xr[b + 4]), z1 = __fadd_rn(xr[b + 1], xr[b + 5]);
        const float z2 = __fadd_rn(xr[b + 2], xr[b + 6]), z3 = __fadd_rn(xr[b + 3], xr[b + 7]);
        sum = __fadd_rn(__fadd_rn(__fadd_rn(z0, z1), z2), z3);
      } else {
        sum = 0.f;
        for (int64_t k = b; k < len; k++) sum = __fadd_rn(sum, xr[k]);
      }
      cs[c] = sum;
    }
  }
  __syncthreads();
  if (row < rows && lane == 0) {
    float total = 0.f;
    for (int64_t c = 0; c < nchunks; c++) total = __fadd_rn(total, cs[c]);
    y[row] = __fdiv_rn(total, (float)len);
  }
}

rtenhip_status launch_reduce_mean_rows(const float* x, float* y, int64_t rows, int64_t len, hipStream_t s) {
  if (rows == 0) return RTENHIP_OK;
  const size_t shmem = 4 * (size_t)((len + 7) / 8) * sizeof(float);
  if (shmem > 64 * 1024) return fail(RTENHIP_UNSUPPORTED_VALUE, "ReduceMean row too long");
  hipLaunchKernelGGL(reduce_mean_rows_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), shmem, s, x, y, rows,
                     len);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

// ReduceMean over any other axes (reduce.rs:287-318): per output element, the
// reduced sub-block in row-major order (lanes along one axis, or the slow
// path's slice iteration) summed with iter_sum -- groups of four as
// sum + ((a + b) + (c + d)) while more than four remain, then one at a time
// (slice_reductions.rs:58-85) -- divided by the element count.
__global__ __launch_bounds__(256) void reduce_mean_iter_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                               ReduceDesc d) {
  for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < d.n_out;
       o += (int64_t)gridDim.x * blockDim.x) {
    int64_t rem = o, base = 0;
    for (int k = d.nk - 1; k >= 0; k--) {
      base += (rem % d.kshape[k]) * d.kstride[k];
      rem /= d.kshape[k];
    }
    auto at = [&](int64_t r) {
      int64_t off = base;
      for (int k = d.nr - 1; k >= 0; k--) {
        off += (r % d.rshape[k]) * d.rstride[k];
        r /= d.rshape[k];
      }
      return x[off];
    };
    float sum = 0.f;
    int64_t r = 0, left = d.n_red;
    while (left > 4) {
      left -= 4;
      const float a = at(r), b = at(r + 1), c = at(r + 2), e = at(r + 3);
      sum = __fadd_rn(sum, __fadd_rn(__fadd_rn(a, b), __fadd_rn(c, e)));
      r += 4;
    }
    for (; r < d.n_red; r++) sum = __fadd_rn(sum, at(r));
    y[o] = __fdiv_rn(sum, (float)d.n_red);
  }
}

rtenhip_status launch_reduce_mean_iter(const float* x, float* y, const ReduceDesc& d, hipStream_t s) {
  if (d.n_out == 0) return RTENHIP_OK;
  int64_t blocks = (d.n_out + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(reduce_mean_iter_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x, y, d);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

// ---------------------------------------------------------------------------
// LogSoftmax (log_softmax_in_place, src/ops/norm.rs:381-406) and
// InstanceNormalization (instance_normalization_in_place, norm.rs:144-198):
// one wave per lane / plane.  Their folds are serial in index order in the
// reference (Iterator::fold / sum, slice_sum's chunk fold), so the wave forms
// 64 terms at a time in parallel and every lane runs the same serial chain
// over them through v_readlane (no LDS, any length, in place safe).
// exp / ln are Rust's f32::exp / f32::ln (libm expf / logf, not rten-vecmath):
// evaluated here in f64 and rounded once, i.e. the correctly rounded value,
// which libm's expf / logf (< 0.51 ULP) return in all but rare ties.

__device__ __forceinline__ float lane_f(float v, int j) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
}

// acc + t_0 + t_1 + ... + t_{n-1}, t_j held by lane j (n <= 64).
__device__ __forceinline__ float wave_serial_fold(float acc, float t, int n) {
  if (n == 64) {
#pragma unroll
    for (int j = 0; j < 64; j++) acc = __fadd_rn(acc, lane_f(t, j));
  } else {
    for (int j = 0; j < n; j++) acc = __fadd_rn(acc, lane_f(t, j));
  }
  return acc;
}

// Rows: row r = (o, i) with o = r / inner, i = r % inner; element k of the row
// at o * len * inner + i + k * inner (the axis need not be last: each lane's
// arithmetic is independent of where its elements sit).
__global__ __launch_bounds__(256) void log_softmax_kernel(const float* x, float* y, int64_t rows, int len,
                                                          int64_t inner) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + wave;
  if (row >= rows) return;
  const int64_t o = row / inner, i = row - o * inner;
  const float* xr = x + o * len * inner + i;
  float* yr = y + o * len * inner + i;
  // slice_max: max is exact and order-free on the values it sees (f32::max
  // ignores NaN like fmaxf), from f32::MIN.
  float m = -FLT_MAX;
  for (int k = lane; k < len; k += 64) m = rust_max(m, xr[(int64_t)k * inner]);
  for (int off = 32; off > 0; off >>= 1) m = rust_max(m, __shfl_xor(m, off));
  // fold(0., |s, x| s + (x - max).exp())
  float s = 0.f;
  for (int k0 = 0; k0 < len; k0 += 64) {
    const int k = k0 + lane;
    const float e = k < len ? (float)exp((double)__fsub_rn(xr[(int64_t)k * inner], m)) : 0.f;
    s = wave_serial_fold(s, e, min(64, len - k0));
  }
  const float lse = (float)log((double)s);
  for (int k = lane; k < len; k += 64) {
    const int64_t at = (int64_t)k * inner;
    yr[at] = __fsub_rn(__fsub_rn(xr[at], m), lse);
  }
}

rtenhip_status launch_log_softmax(const float* x, float* y, int64_t outer, int64_t len, int64_t inner,
                                  hipStream_t s) {
  const int64_t rows = outer * inner;
  if (rows == 0 || len == 0) return RTENHIP_OK;
  if (len > INT32_MAX) return fail(RTENHIP_INVALID_VALUE, "LogSoftmax: axis too long");
  hipLaunchKernelGGL(log_softmax_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, x, y, rows, (int)len,
                     inner);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

// Plane p = (n, c) of len contiguous floats, channel c = p % C.
__global__ __launch_bounds__(256) void instance_norm_kernel(const float* x, float* y, int64_t planes, int C,
                                                            int64_t len, const float* __restrict__ scale,
                                                            const float* __restrict__ bias, float eps) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t p = (int64_t)blockIdx.x * 4 + wave;
  if (p >= planes) return;
  const float* xr = x + p * len;
  float* yr = y + p * len;
  const int c = (int)(p % C);
  // slice_sum (slice_reductions.rs:37-53): 8-element chunks
  // ((x0+x4)+(x1+x5))+(x2+x6))+(x3+x7), folded in order from 0, then the
  // tail chunk's own fold from 0.
  const int64_t nchunks = len / 8;
  float total = 0.f;
  for (int64_t c0 = 0; c0 < nchunks; c0 += 64) {
    const int64_t ck = c0 + lane;
    float cs = 0.f;
    if (ck < nchunks) {
      const float* q = xr + 8 * ck;
      const float z0 = __fadd_rn(q[0], q[4]), z1 = __fadd_rn(q[1], q[5]);
      const float z2 = __fadd_rn(q[2], q[6]), z3 = __fadd_rn(q[3], q[7]);
      cs = __fadd_rn(__fadd_rn(__fadd_rn(z0, z1), z2), z3);
    }
    total = wave_serial_fold(total, cs, (int)min<int64_t>(64, nchunks - c0));
  }
  if (nchunks * 8 < len) {
    const int64_t k = nchunks * 8 + lane;
    const float t = k < len ? xr[k] : 0.f;
    total = __fadd_rn(total, wave_serial_fold(0.f, t, (int)(len - nchunks * 8)));
  }
  const float mean = __fdiv_rn(total, (float)len);
  // slice.iter().map(|x| (x - mean)^2).sum() / len: one serial chain.
  float var = 0.f;
  for (int64_t k0 = 0; k0 < len; k0 += 64) {
    const int64_t k = k0 + lane;
    float d2 = 0.f;
    if (k < len) {
      const float d = __fsub_rn(xr[k], mean);
      d2 = __fmul_rn(d, d);
    }
    var = wave_serial_fold(var, d2, (int)min<int64_t>(64, len - k0));
  }
  var = __fdiv_rn(var, (float)len);
  const float r = __fdiv_rn(scale[c], sqrt_rn(__fadd_rn(var, eps)));
  const float b = bias[c];
  for (int64_t k = lane; k < len; k += 64) yr[k] = __fadd_rn(__fmul_rn(__fsub_rn(xr[k], mean), r), b);
}

rtenhip_status launch_instance_norm(const float* x, float* y, int64_t N, int64_t C, int64_t len,
                                    const float* scale, const float* bias, float eps, hipStream_t s) {
  const int64_t planes = N * C;
  if (planes == 0 || len == 0) return RTENHIP_OK;
  hipLaunchKernelGGL(instance_norm_kernel, dim3((unsigned)((planes + 3) / 4)), dim3(256), 0, s, x, y, planes,
                     (int)C, len, scale, bias, eps);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

}  // namespace rtenhip
