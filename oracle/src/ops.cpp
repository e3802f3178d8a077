// CPU restatement of RTen's elementwise, normalization and matmul operators
// (test infrastructure; see rten_oracle.h).
//
// Numerics follow rten-vecmath (exp.rs:73-148, erf.rs:29-91, tanh.rs:14-65,
// softmax.rs:14-56), src/ops/unary_elementwise.rs, src/ops/binary_elementwise.rs,
// src/ops/norm.rs:18-448, src/ops/reduce.rs:334-387, src/slice_reductions.rs and
// src/ops/matmul.rs:27-239.  Built with -ffp-contract=off: every `fmaf` below is
// a `mul_add` in the reference; every other mul/add rounds separately.
#include <omp.h>

#include <algorithm>
#include <cfloat>
#include <limits>

#include "common.h"

namespace orc {

static inline uint32_t f2u(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}
static inline float u2f(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}

// simd_exp (exp.rs:73-133).
static inline float vm_exp(float x) {
  const float INV_LOG2 = 1.44269504088896340736f, MAGIC = 12582912.f;
  const float LN2_HI = -6.93145752e-1f, LN2_LO = -1.42860677e-6f;
  float j = fmaf(x, INV_LOG2, MAGIC);
  j = j - MAGIC;
  float r = fmaf(j, LN2_HI, x);
  r = fmaf(j, LN2_LO, r);
  // _mm256_cvttps_epi32: out-of-range / NaN -> INT_MIN.
  int32_t k;
  if (std::isnan(j) || j >= 2147483648.f || j < -2147483648.f)
    k = INT32_MIN;
  else
    k = (int32_t)j;
  float t = 1.37805939e-3f;
  t = fmaf(t, r, 8.37312452e-3f);
  t = fmaf(t, r, 4.16695364e-2f);
  t = fmaf(t, r, 1.66664720e-1f);
  t = fmaf(t, r, 4.99999851e-1f);
  t = fmaf(t, r, 1.0f);
  r = fmaf(t, r, 1.0f);
  uint32_t ia = k > 0 ? 0u : 0x83000000u;
  uint32_t is = ia + 0x7f000000u;
  uint32_t it = ((uint32_t)k << 23) - ia;
  r = r * u2f(is);
  r = r * u2f(it);
  if (x >= 104.f) r = std::numeric_limits<float>::infinity();
  if (x <= -104.f) r = 0.f;
  return r;
}

// simd_sigmoid (exp.rs:144-148).
static inline float vm_sigmoid(float x) {
  float denom = 1.f + vm_exp(0.f - x);
  return 1.f / denom;
}

// simd_erf (erf.rs:29-58).
static inline float vm_erf(float x) {
  bool neg = x < 0.f;
  float ax = neg ? 0.f - x : x;
  float t = 1.f / fmaf(ax, 0.3275911f, 1.f);
  float y = 1.061405429f;
  y = fmaf(y, t, -1.453152027f);
  y = fmaf(y, t, 1.421413741f);
  y = fmaf(y, t, -0.284496736f);
  y = fmaf(y, t, 0.254829592f);
  float at = y * t;
  float xm2 = 0.f - ax * ax;
  float e = vm_exp(xm2);
  float r = 1.f - at * e;
  return neg ? 0.f - r : r;
}

// simd_gelu (erf.rs:85-91).
static inline float vm_gelu(float x) {
  const float SQRT_2_RCP = 0.70710678118654752440f;
  float half_x = x * 0.5f;
  float y = x * SQRT_2_RCP;
  y = vm_erf(y) + 1.f;
  return half_x * y;
}

// simd_tanh (tanh.rs:14-65).
static inline float vm_tanh(float x) {
  bool x_neg = x <= 0.f;
  float ax = std::fabs(x);
  bool cutoff = ax >= 9.02f, tiny = ax <= 0.0004f, small = ax <= 0.55f;
  float xs = x * x;
  float ys = fmaf(1.5497927553951740264892578125e-2f, xs, -5.21197654306888580322265625e-2f);
  ys = fmaf(ys, xs, 0.13310669362545013427734375f);
  ys = fmaf(ys, xs, -0.33332359790802001953125f);
  ys = fmaf(ys, xs, 0.999999940395355224609375f);
  ys = ys * ax;
  float e = vm_exp(ax * 2.f);
  float ym = (e - 1.f) / (e + 1.f);
  float y = cutoff ? 1.f : ym;
  y = small ? ys : y;
  y = tiny ? ax : y;
  return x_neg ? 0.f - y : y;
}

static inline float rust_max(float a, float b) { return std::fmax(a, b); }

// src/slice_reductions.rs:37-53.
static float slice_sum(const float* xs, int64_t n) {
  float total = 0.f;
  int64_t i = 0;
  for (; i + 8 <= n; i += 8) {
    float z0 = xs[i] + xs[i + 4], z1 = xs[i + 1] + xs[i + 5];
    float z2 = xs[i + 2] + xs[i + 6], z3 = xs[i + 3] + xs[i + 7];
    float c = ((z0 + z1) + z2) + z3;
    total = total + c;
  }
  if (i < n) {
    float c = 0.f;
    for (; i < n; i++) c = c + xs[i];
    total = total + c;
  }
  return total;
}

// iter_sum (src/slice_reductions.rs:57-84) over squares (reduce_inverse_rms).
static float iter_sum_sq(const float* xs, int64_t len) {
  float sum = 0.f;
  int64_t n = len, i = 0;
  while (n > 4) {
    n -= 4;
    float a = xs[i] * xs[i], b = xs[i + 1] * xs[i + 1];
    float c = xs[i + 2] * xs[i + 2], d = xs[i + 3] * xs[i + 3];
    float ab = a + b, cd = c + d, abcd = ab + cd;
    sum = sum + abcd;
    i += 4;
  }
  for (; i < len; i++) sum = sum + xs[i] * xs[i];
  return sum;
}

// broadcast_shapes (binary_elementwise.rs:23-45).
static bool broadcast_shapes(const int64_t* a, int an, const int64_t* b, int bn, int64_t* out,
                             int* on) {
  int n = std::max(an, bn);
  for (int i = 0; i < n; i++) {
    int64_t ad = i < an ? a[an - 1 - i] : 1, bd = i < bn ? b[bn - 1 - i] : 1;
    int64_t r;
    if (ad == bd)
      r = ad;
    else if (ad == 1)
      r = bd;
    else if (bd == 1)
      r = ad;
    else
      return false;
    out[n - 1 - i] = r;
  }
  *on = n;
  return true;
}

// Element strides of `shape` broadcast to `out` (0 on broadcast dims).
static void bcast_strides(const int64_t* shape, int nd, const int64_t* out, int on,
                          int64_t* strides) {
  int64_t s = 1;
  for (int i = on - 1; i >= 0; i--) {
    int si = i - (on - nd);
    if (si < 0) {
      strides[i] = 0;
      continue;
    }
    strides[i] = (shape[si] == 1 && out[i] != 1) ? 0 : s;
    s *= shape[si];
  }
}

template <typename F>
static void binary_apply(const float* a, const int64_t* as, int an, const float* b,
                         const int64_t* bs, int bn, float* out, const int64_t* os, int on, F f) {
  int64_t sa[16], sb[16];
  bcast_strides(as, an, os, on, sa);
  bcast_strides(bs, bn, os, on, sb);
  int64_t total = numel(os, on);
  int64_t inner = on ? os[on - 1] : 1;
  int64_t outer = inner ? total / inner : 0;
#pragma omp parallel for if (total > 65536)
  for (int64_t o = 0; o < outer; o++) {
    int64_t rem = o, oa = 0, ob = 0;
    for (int d = on - 2; d >= 0; d--) {
      int64_t idx = rem % os[d];
      rem /= os[d];
      oa += idx * sa[d];
      ob += idx * sb[d];
    }
    int64_t ia = on ? sa[on - 1] : 0, ib = on ? sb[on - 1] : 0;
    float* po = out + o * inner;
    for (int64_t i = 0; i < inner; i++) po[i] = f(a[oa + i * ia], b[ob + i * ib]);
  }
}

static void permute_copy(const float* x, const int64_t* shape, int nd, const int* perm,
                         float* out) {
  // out[idx] = x[permuted idx]; out shape = shape[perm[i]].
  int64_t os[16], xs[16], st[16];
  int64_t s = 1;
  for (int i = nd - 1; i >= 0; i--) {
    xs[i] = s;
    s *= shape[i];
  }
  for (int i = 0; i < nd; i++) {
    os[i] = shape[perm[i]];
    st[i] = xs[perm[i]];
  }
  int64_t total = numel(shape, nd);
  for (int64_t o = 0; o < total; o++) {
    int64_t rem = o, off = 0;
    for (int d = nd - 1; d >= 0; d--) {
      off += (rem % os[d]) * st[d];
      rem /= os[d];
    }
    out[o] = x[off];
  }
}

// simd_softmax over one contiguous lane, AVX2 width (S::LEN = 8).
static void softmax_lane(const float* x, float* y, int64_t n) {
  const int L = 8;
  float mx[L];
  for (int j = 0; j < L; j++) mx[j] = -FLT_MAX;
  for (int64_t i = 0; i < n; i++) mx[i % L] = rust_max(mx[i % L], x[i]);
  // _mm256_max_ps(max, x) returns x when either is NaN; restate for finite data.
  float m = -FLT_MAX;
  for (int j = 0; j < L; j++) m = rust_max(m, mx[j]);
  float es[L] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t i = 0; i < n; i++) {
    float e = vm_exp(x[i] - m);
    y[i] = e;
    es[i % L] = es[i % L] + e;
  }
  float sum = 0.f;
  for (int j = 0; j < L; j++) sum = sum + es[j];
  for (int64_t i = 0; i < n; i++) y[i] = y[i] / sum;
}

}  // namespace orc

using namespace orc;

extern "C" {

int orc_unary(int op, const float* x, int64_t n, float* y, float p0, float p1) {
#pragma omp parallel for if (n > 32768)
  for (int64_t i = 0; i < n; i++) {
    float v = x[i], r;
    switch (op) {
      case ORC_RELU:
        r = rust_max(v, 0.f);
        break;
      case ORC_CLIP: {  // Clamp::clamp = max(lo).min(hi), the trait's own max / min (unary_elementwise.rs:263-323)
        const float m = v > p0 ? v : p0;
        r = m < p1 ? m : p1;
        break;
      }
      case ORC_GELU:
        r = vm_gelu(v);
        break;
      case ORC_ERF:
        r = vm_erf(v);
        break;
      case ORC_SIGMOID:
        r = vm_sigmoid(v);
        break;
      case ORC_TANH:
        r = vm_tanh(v);
        break;
      case ORC_EXP:
        r = vm_exp(v);
        break;
      case ORC_SILU:
        r = v * vm_sigmoid(v);
        break;
      default:
        r = v;
    }
    y[i] = r;
  }
  return ORC_OK;
}

int orc_binary(int op, const float* a, const int64_t* a_shape, int a_ndim, const float* b,
               const int64_t* b_shape, int b_ndim, float* out, int64_t* out_shape,
               int* out_ndim) {
  if (!broadcast_shapes(a_shape, a_ndim, b_shape, b_ndim, out_shape, out_ndim))
    return fail(ORC_INCOMPATIBLE_INPUT_SHAPES, "Cannot broadcast inputs");
  switch (op) {
    case 0:
      binary_apply(a, a_shape, a_ndim, b, b_shape, b_ndim, out, out_shape, *out_ndim,
                   [](float p, float q) { return p + q; });
      break;
    case 1:
      binary_apply(a, a_shape, a_ndim, b, b_shape, b_ndim, out, out_shape, *out_ndim,
                   [](float p, float q) { return p - q; });
      break;
    case 2:
      binary_apply(a, a_shape, a_ndim, b, b_shape, b_ndim, out, out_shape, *out_ndim,
                   [](float p, float q) { return p * q; });
      break;
    case 3:
      binary_apply(a, a_shape, a_ndim, b, b_shape, b_ndim, out, out_shape, *out_ndim,
                   [](float p, float q) { return p / q; });
      break;
    default:
      return fail(ORC_UNSUPPORTED_VALUE, "unknown binary op");
  }
  return ORC_OK;
}

int orc_batch_norm(const float* x, const int64_t* shape, int ndim, const float* scale,
                   const float* bias, const float* mean, const float* var, float epsilon,
                   float* out) {
  if (ndim < 3) return fail(ORC_INVALID_VALUE, "Input must have at least 3 dims");
  int64_t N = shape[0], C = shape[1], inner = numel(shape + 2, ndim - 2);
#pragma omp parallel for collapse(2)
  for (int64_t n = 0; n < N; n++)
    for (int64_t c = 0; c < C; c++) {
      // batch_norm_in_place (norm.rs:18-54)
      float s = scale[c] / std::sqrt(var[c] + epsilon);
      const float* p = x + (n * C + c) * inner;
      float* q = out + (n * C + c) * inner;
      for (int64_t i = 0; i < inner; i++) q[i] = (p[i] - mean[c]) * s + bias[c];
    }
  return ORC_OK;
}

// log_softmax_in_place (src/ops/norm.rs:381-406) over lanes along `axis`
// (softmax_lanes moves the axis last; the per-lane arithmetic does not depend
// on where the elements sit).  exp / ln are Rust's f32::exp / f32::ln, i.e.
// libm expf / logf -- the same functions std::exp / std::log call here.
int orc_log_softmax(const float* x, const int64_t* shape, int ndim, int64_t axis, float* out) {
  if (axis < 0) axis += ndim;
  if (axis < 0 || axis >= ndim) return fail(ORC_INVALID_VALUE, "Axis is invalid");
  const int64_t len = shape[axis];
  const int64_t outer = numel(shape, (int)axis), inner = numel(shape + axis + 1, ndim - (int)axis - 1);
#pragma omp parallel for collapse(2) if (outer * inner > 64)
  for (int64_t o = 0; o < outer; o++)
    for (int64_t i = 0; i < inner; i++) {
      const float* p = x + o * len * inner + i;
      float* q = out + o * len * inner + i;
      // slice_max (slice_reductions.rs:16-36): f32::max from f32::MIN
      float m = -FLT_MAX;
      for (int64_t k = 0; k < len; k++) m = rust_max(m, p[k * inner]);
      float s = 0.f;
      for (int64_t k = 0; k < len; k++) s = s + std::exp(p[k * inner] - m);
      const float lse = std::log(s);
      for (int64_t k = 0; k < len; k++) q[k * inner] = (p[k * inner] - m) - lse;
    }
  return ORC_OK;
}

// instance_normalization_in_place (src/ops/norm.rs:144-198).
int orc_instance_norm(const float* x, const int64_t* shape, int ndim, const float* scale, int64_t n_scale,
                      const float* bias, int64_t n_bias, float epsilon, float* out) {
  if (ndim < 2) return fail(ORC_INVALID_VALUE, "expected input with >= 2 dims");
  const int64_t N = shape[0], C = shape[1], len = numel(shape + 2, ndim - 2);
  if (n_scale != C) return fail(ORC_INVALID_VALUE, "scale length should match channel count");
  if (n_bias != C) return fail(ORC_INVALID_VALUE, "bias length should match channel count");
#pragma omp parallel for collapse(2)
  for (int64_t n = 0; n < N; n++)
    for (int64_t c = 0; c < C; c++) {
      const float* p = x + (n * C + c) * len;
      float* q = out + (n * C + c) * len;
      const float mean = slice_sum(p, len) / (float)len;
      float var = 0.f;  // Iterator::sum: one chain in index order
      for (int64_t i = 0; i < len; i++) {
        const float d = p[i] - mean;
        var = var + d * d;
      }
      var = var / (float)len;
      const float r = scale[c] / std::sqrt(var + epsilon);
      for (int64_t i = 0; i < len; i++) q[i] = (p[i] - mean) * r + bias[c];
    }
  return ORC_OK;
}

int orc_softmax(const float* x, const int64_t* shape, int ndim, int64_t axis, float* out) {
  if (axis < 0) axis += ndim;
  if (axis < 0 || axis >= ndim) return fail(ORC_INVALID_VALUE, "Axis is invalid");
  int64_t total = numel(shape, ndim);
  if (axis == ndim - 1) {
    int64_t lane = ndim ? shape[ndim - 1] : total;
    int64_t lanes = lane ? total / lane : 0;
#pragma omp parallel for if (total > 4096)
    for (int64_t l = 0; l < lanes; l++) softmax_lane(x + l * lane, out + l * lane, lane);
    return ORC_OK;
  }
  // softmax_lanes (norm.rs:332-379): move axis last, make contiguous, apply,
  // move back.
  int perm[16], inv[16];
  int k = 0;
  for (int i = 0; i < ndim; i++)
    if (i != axis) perm[k++] = i;
  perm[k] = (int)axis;
  int64_t pshape[16];
  for (int i = 0; i < ndim; i++) pshape[i] = shape[perm[i]];
  for (int i = 0; i < ndim; i++) inv[perm[i]] = i;
  std::vector<float> t(total), u(total);
  permute_copy(x, shape, ndim, perm, t.data());
  int64_t lane = shape[axis];
  for (int64_t l = 0; l < total / lane; l++) softmax_lane(&t[l * lane], &u[l * lane], lane);
  permute_copy(u.data(), pshape, ndim, inv, out);
  return ORC_OK;
}

int orc_layer_norm(const float* x, const int64_t* shape, int ndim, const float* scale,
                   const float* bias, int64_t axis, float epsilon, float* out) {
  if (axis < 0) axis += ndim;
  if (axis < 0 || axis >= ndim) return fail(ORC_INVALID_VALUE, "Axis is invalid");
  int64_t row = numel(shape + axis, ndim - (int)axis);
  int64_t rows = row ? numel(shape, ndim) / row : 0;
#pragma omp parallel for if (rows > 16)
  for (int64_t r = 0; r < rows; r++) {
    // layer_normalization (norm.rs:245-299): reduce_mean -> sub ->
    // reduce_inverse_rms -> mul -> mul(scale) -> add(bias).
    const float* p = x + r * row;
    float* q = out + r * row;
    float mean = slice_sum(p, row) / (float)row;
    for (int64_t i = 0; i < row; i++) q[i] = p[i] - mean;
    float ms = iter_sum_sq(q, row) / (float)row;
    float inv = 1.f / std::sqrt(ms + epsilon);
    for (int64_t i = 0; i < row; i++) q[i] = q[i] * inv;
    for (int64_t i = 0; i < row; i++) q[i] = q[i] * scale[i];
    if (bias)
      for (int64_t i = 0; i < row; i++) q[i] = q[i] + bias[i];
  }
  return ORC_OK;
}

int orc_gemm_op(const float* a, const int64_t a_shape[2], const float* b, const int64_t b_shape[2],
                const float* c, const int64_t* c_shape, int c_ndim, float alpha, float beta,
                int trans_a, int trans_b, float* out) {
  // gemm_op (matmul.rs:27-81): transposes are views.
  Mat A = trans_a ? Mat{a, a_shape[1], a_shape[0], 1, a_shape[1]}
                  : Mat{a, a_shape[0], a_shape[1], a_shape[1], 1};
  Mat B = trans_b ? Mat{b, b_shape[1], b_shape[0], 1, b_shape[1]}
                  : Mat{b, b_shape[0], b_shape[1], b_shape[1], 1};
  if (A.cols != B.rows)
    return fail(ORC_INCOMPATIBLE_INPUT_SHAPES,
                "Columns of matrix `a` must match rows of matrix `b`");
  int64_t M = A.rows, N = B.cols;
  if (c && beta != 0.f) {
    int64_t os[2] = {M, N}, ob[2];
    int on;
    if (!broadcast_shapes(c_shape, c_ndim, os, 2, ob, &on) || ob[0] != M || ob[1] != N)
      return fail(ORC_INCOMPATIBLE_INPUT_SHAPES, "Cannot broadcast c to output shape");
    int64_t sc[2];
    bcast_strides(c_shape, c_ndim, os, 2, sc);
    for (int64_t i = 0; i < M; i++)
      for (int64_t j = 0; j < N; j++) out[i * N + j] = c[i * sc[0] + j * sc[1]];
    gemm_impl(out, N, A, &B, nullptr, alpha, beta, nullptr, false);
  } else {
    gemm_impl(out, N, A, &B, nullptr, alpha, 0.f, nullptr, false);
  }
  return ORC_OK;
}

int orc_matmul(const float* a, const int64_t* a_shape, int a_ndim, const float* b,
               const int64_t* b_shape, int b_ndim, float* out, int64_t* out_shape, int* out_ndim) {
  // matmul_impl (matmul.rs:123-239).
  if (a_ndim < 2 || b_ndim < 2) return fail(ORC_INVALID_VALUE, "Inputs must have >= 2 dimensions");
  int64_t M = a_shape[a_ndim - 2], K = a_shape[a_ndim - 1];
  int64_t KB = b_shape[b_ndim - 2], N = b_shape[b_ndim - 1];
  if (K != KB)
    return fail(ORC_INCOMPATIBLE_INPUT_SHAPES,
                "Columns of first matrix does not match rows of second matrix");
  int64_t na = numel(a_shape, a_ndim - 2), nb = numel(b_shape, b_ndim - 2);
  int64_t prefix[16];
  int pn;
  if (!broadcast_shapes(a_shape, a_ndim - 2, b_shape, b_ndim - 2, prefix, &pn))
    return fail(ORC_INCOMPATIBLE_INPUT_SHAPES, "Cannot broadcast shapes");
  for (int i = 0; i < pn; i++) out_shape[i] = prefix[i];
  out_shape[pn] = M;
  out_shape[pn + 1] = N;
  *out_ndim = pn + 2;
  if (na > 1 && nb == 1) {
    // Fold the batch into M: one [A*M, K] x [K, N] GEMM.
    Mat A{a, na * M, K, K, 1}, B{b, K, N, N, 1};
    gemm_impl(out, N, A, &B, nullptr, 1.f, 0.f, nullptr, false);
    return ORC_OK;
  }
  int64_t nout = numel(prefix, pn);
  int64_t sa[16], sb[16];
  bcast_strides(a_shape, a_ndim - 2, prefix, pn, sa);
  bcast_strides(b_shape, b_ndim - 2, prefix, pn, sb);
  bool par = nout > 1;
#pragma omp parallel for schedule(dynamic, 1) if (par)
  for (int64_t o = 0; o < nout; o++) {
    int64_t rem = o, ia = 0, ib = 0;
    for (int d = pn - 1; d >= 0; d--) {
      int64_t idx = rem % prefix[d];
      rem /= prefix[d];
      ia += idx * sa[d];
      ib += idx * sb[d];
    }
    Mat A{a + ia * M * K, M, K, K, 1}, B{b + ib * K * N, K, N, N, 1};
    gemm_impl(out + o * M * N, N, A, &B, nullptr, 1.f, 0.f, nullptr, par);
  }
  return ORC_OK;
}

}  // extern "C"
