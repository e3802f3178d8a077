// C ABI operator entry points other than Conv / GEMM (include/rten_hip.h):
// Gemm, MatMul, pooling, normalisation, softmax, unary and binary ops.
// Shape checks and error messages follow the reference operators cited at
// each function.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "common.h"
#include "ctx.h"

namespace rtenhip {

bool broadcast_shapes(const int64_t* a, int an, const int64_t* b, int bn, int64_t* out, int* on) {
  int n = std::max(an, bn);
  if (n > RTENHIP_MAX_DIMS) return false;
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

// Element strides of tensor t broadcast to `out` (0 on broadcast dims).
static void bcast_strides(const rtenhip_tensor& t, const int64_t* out, int on, int64_t* strides) {
  for (int i = on - 1; i >= 0; i--) {
    int ti = i - (on - t.ndim);
    if (ti < 0) {
      strides[i] = 0;
      continue;
    }
    strides[i] = (t.shape[ti] == 1 && out[i] != 1) ? 0 : t.strides[ti];
  }
}

static rtenhip_status check_out_shape(const rtenhip_tensor* y, const int64_t* shape, int nd) {
  if (!y) return fail(RTENHIP_INCORRECT_OUTPUT_TYPE, "Missing output");
  bool ok = y->ndim == nd;
  for (int i = 0; ok && i < nd; i++) ok = y->shape[i] == shape[i];
  if (!ok) return fail(RTENHIP_INCORRECT_OUTPUT_TYPE, "Output has wrong shape");
  if (!is_contiguous(*y)) return fail(RTENHIP_UNSUPPORTED_VALUE, "Output must be contiguous");
  return RTENHIP_OK;
}

// Pointer to contiguous data of t, copying to scratch slot if needed.
static const float* contiguous(Ctx* c, const rtenhip_tensor& t, int slot, rtenhip_status* st) {
  *st = RTENHIP_OK;
  if (is_contiguous(t)) return t.data;
  float* tmp = c->scratch_floats(numel(t), slot);
  if (!tmp) {
    *st = fail(RTENHIP_HIP_ERROR, "scratch allocation failed");
    return nullptr;
  }
  *st = launch_copy_strided(t, tmp, c->stream);
  return tmp;
}

static rtenhip_status binary_impl(Ctx* c, int op, const rtenhip_tensor& a, const rtenhip_tensor& b,
                                  rtenhip_tensor* y) {
  int64_t os[RTENHIP_MAX_DIMS];
  int on;
  if (!broadcast_shapes(a.shape, a.ndim, b.shape, b.ndim, os, &on))
    return fail(RTENHIP_INCOMPATIBLE_INPUT_SHAPES, "Cannot broadcast inputs");
  rtenhip_status st = check_out_shape(y, os, on);
  if (st) return st;
  int64_t n = 1;
  for (int i = 0; i < on; i++) n *= os[i];
  BcastDesc d{};
  d.ndim = on;
  for (int i = 0; i < on; i++) d.shape[i] = os[i];
  bcast_strides(a, os, on, d.sa);
  bcast_strides(b, os, on, d.sb);
  // Fast modes when a is contiguous with the output shape.
  bool a_full = is_contiguous(a) && a.ndim == on;
  for (int i = 0; a_full && i < on; i++) a_full = a.shape[i] == os[i];
  int mode = 3;
  int64_t inner = 1, nb = 1;
  if (a_full && is_contiguous(b)) {
    // b's dims right-aligned; find the span of its non-1 dims.
    int lo = on, hi = -1;
    for (int i = 0; i < b.ndim; i++)
      if (b.shape[i] != 1) {
        int oi = i + (on - b.ndim);
        lo = std::min(lo, oi);
        hi = std::max(hi, oi);
      }
    bool span_full = true;
    for (int i = lo; i <= hi && hi >= 0; i++) {
      int bi = i - (on - b.ndim);
      if (b.shape[bi] != os[i]) span_full = false;
    }
    if (span_full) {
      if (hi < 0) {
        mode = 2;  // scalar b
        inner = n;
        nb = 1;
      } else {
        int64_t tail = 1;
        for (int i = hi + 1; i < on; i++) tail *= os[i];
        nb = 1;
        for (int i = lo; i <= hi; i++) nb *= os[i];
        if (lo == 0 && tail == 1)
          mode = 0;
        else if (tail == 1) {
          mode = 1;
          inner = nb;
        } else {
          mode = 2;
          inner = tail;
        }
      }
    }
  }
  return launch_binary(op, a.data, b.data, y->data, n, d, mode, inner, nb, c->stream);
}

}  // namespace rtenhip

using namespace rtenhip;
static Ctx* C_(rtenhip_ctx* c) { return reinterpret_cast<Ctx*>(c); }

extern "C" {

// gemm_op (src/ops/matmul.rs:27-81).
rtenhip_status rtenhip_gemm_op_f32(rtenhip_ctx* ctx, const rtenhip_tensor* a,
                                   const rtenhip_tensor* b, const rtenhip_tensor* c, float alpha,
                                   float beta, int trans_a, int trans_b, rtenhip_tensor* y) {
  Ctx* cx = C_(ctx);
  if (!a || !b) return fail(RTENHIP_MISSING_INPUTS, "Missing inputs");
  if (a->ndim != 2) return fail(RTENHIP_INVALID_VALUE, "Expected a to have 2 dims");
  if (b->ndim != 2) return fail(RTENHIP_INVALID_VALUE, "Expected b to have 2 dims");
  // Transposes are views.
  int64_t M = trans_a ? a->shape[1] : a->shape[0], K = trans_a ? a->shape[0] : a->shape[1];
  int64_t a_rs = trans_a ? a->strides[1] : a->strides[0], a_cs = trans_a ? a->strides[0] : a->strides[1];
  int64_t KB = trans_b ? b->shape[1] : b->shape[0], N = trans_b ? b->shape[0] : b->shape[1];
  int64_t b_rs = trans_b ? b->strides[1] : b->strides[0], b_cs = trans_b ? b->strides[0] : b->strides[1];
  if (K != KB)
    return fail(RTENHIP_INCOMPATIBLE_INPUT_SHAPES,
                "Columns of matrix `a` must match rows of matrix `b`");
  int64_t os[2] = {M, N};
  rtenhip_status st = check_out_shape(y, os, 2);
  if (st) return st;
  if (c && c->data && beta != 0.f) {
    int64_t bs[RTENHIP_MAX_DIMS];
    int bn;
    if (!broadcast_shapes(c->shape, c->ndim, os, 2, bs, &bn) || bn != 2 || bs[0] != M || bs[1] != N)
      return fail(RTENHIP_INCOMPATIBLE_INPUT_SHAPES, "Cannot broadcast c to output shape");
    // expand_to(c, out_shape): out = c broadcast, then gemm with beta.
    rtenhip_tensor cz = *c;
    BcastDesc d{};
    d.ndim = 2;
    d.shape[0] = M;
    d.shape[1] = N;
    bcast_strides(cz, os, 2, d.sb);
    // One output row (the FC layer at batch 1): the gemv reads the broadcast
    // C itself (same beta * C + alpha * acc arithmetic, no copy launch).
    if (M == 1 && K > 0 && a_cs == 1)
      return launch_gemv(N, K, a->data, b->data, b_rs, b_cs, y->data, alpha, beta, nullptr, cx->ref_threads,
                         cx->stream, c->data, d.sb[1]);
    // A plain strided copy of the broadcast view.
    rtenhip_tensor view{};
    view.data = c->data;
    view.ndim = 2;
    view.shape[0] = M;
    view.shape[1] = N;
    view.strides[0] = d.sb[0];
    view.strides[1] = d.sb[1];
    st = launch_copy_strided(view, y->data, cx->stream);
    if (st) return st;
    return gemm_impl(cx, M, N, K, a->data, a_rs, a_cs, b->data, b_rs, b_cs, y->data, N, alpha,
                     beta, nullptr, 0);
  }
  return gemm_impl(cx, M, N, K, a->data, a_rs, a_cs, b->data, b_rs, b_cs, y->data, N, alpha, 0.f,
                   nullptr, 0);
}

// matmul_impl (src/ops/matmul.rs:123-239).
rtenhip_status rtenhip_matmul_f32(rtenhip_ctx* ctx, const rtenhip_tensor* a,
                                  const rtenhip_tensor* b, rtenhip_tensor* y) {
  Ctx* cx = C_(ctx);
  if (!a || !b) return fail(RTENHIP_MISSING_INPUTS, "Missing inputs");
  if (a->ndim < 2 || b->ndim < 2) return fail(RTENHIP_INVALID_VALUE, "Inputs must have >= 2 dimensions");
  const int an = a->ndim, bn = b->ndim;
  const int64_t M = a->shape[an - 2], K = a->shape[an - 1];
  const int64_t KB = b->shape[bn - 2], N = b->shape[bn - 1];
  if (K != KB)
    return fail(RTENHIP_INCOMPATIBLE_INPUT_SHAPES,
                "Columns of first matrix does not match rows of second matrix");
  int64_t prefix[RTENHIP_MAX_DIMS];
  int pn;
  if (!broadcast_shapes(a->shape, an - 2, b->shape, bn - 2, prefix, &pn))
    return fail(RTENHIP_INCOMPATIBLE_INPUT_SHAPES, "Cannot broadcast shapes");
  int64_t os[RTENHIP_MAX_DIMS];
  for (int i = 0; i < pn; i++) os[i] = prefix[i];
  os[pn] = M;
  os[pn + 1] = N;
  rtenhip_status st = check_out_shape(y, os, pn + 2);
  if (st) return st;
  int64_t na = 1, nb = 1, nout = 1;
  for (int i = 0; i < an - 2; i++) na *= a->shape[i];
  for (int i = 0; i < bn - 2; i++) nb *= b->shape[i];
  for (int i = 0; i < pn; i++) nout *= prefix[i];
  if (nout * M * N == 0) return RTENHIP_OK;
  const int64_t b_rs = b->strides[bn - 2], b_cs = b->strides[bn - 1];
  if (na > 1 && nb == 1) {
    // Fold the batch into M: [A*M, K] @ [K, N] (matmul.rs:162-169).
    const float* ad = contiguous(cx, *a, 0, &st);
    if (st) return st;
    return gemm_impl(cx, na * M, N, K, ad, K, 1, b->data, b_rs, b_cs, y->data, N, 1.f, 0.f,
                     nullptr, 0);
  }
  if (M == 1) {
    // One gemv per output matrix (A has a single row -> gemv path).
    int64_t sa[RTENHIP_MAX_DIMS], sb[RTENHIP_MAX_DIMS];
    rtenhip_tensor ap = *a, bp = *b;
    ap.ndim = an - 2;
    bp.ndim = bn - 2;
    bcast_strides(ap, prefix, pn, sa);
    bcast_strides(bp, prefix, pn, sb);
    for (int64_t o = 0; o < nout; o++) {
      int64_t rem = o, oa = 0, ob = 0;
      for (int i = pn - 1; i >= 0; i--) {
        int64_t idx = rem % prefix[i];
        rem /= prefix[i];
        oa += idx * sa[i];
        ob += idx * sb[i];
      }
      if (a->strides[an - 1] != 1) return fail(RTENHIP_UNSUPPORTED_VALUE, "gemv needs unit-stride A row");
      st = launch_gemv(N, K, a->data + oa, b->data + ob, b_rs, b_cs, y->data + o * N, 1.f, 0.f,
                       nullptr, cx->ref_threads, cx->stream);
      if (st) return st;
    }
    return RTENHIP_OK;
  }
  if (pn > 4) return fail(RTENHIP_UNSUPPORTED_VALUE, "MatMul supports up to 4 batch dims");
  GemmDesc d{};
  d.M = (int)M;
  d.N = (int)N;
  d.K = (int)K;
  d.a = a->data;
  d.a_m = a->strides[an - 2];
  d.a_k = a->strides[an - 1];
  d.bmode = 0;
  d.b = b->data;
  d.b_k = b_rs;
  d.b_n = b_cs;
  d.omode = 0;
  d.out = y->data;
  d.out_m = N;
  d.alpha = 1.f;
  d.beta = 0.f;
  d.nbatch = (int)nout;
  d.nbp = pn;
  rtenhip_tensor ap = *a, bp = *b;
  ap.ndim = an - 2;
  bp.ndim = bn - 2;
  bcast_strides(ap, prefix, pn, d.pa);
  bcast_strides(bp, prefix, pn, d.pb);
  int64_t so = M * N;
  for (int i = pn - 1; i >= 0; i--) {
    d.pshape[i] = prefix[i];
    d.po[i] = so;
    so *= prefix[i];
  }
  return launch_gemm(d, cx->stream);
}

static rtenhip_status pool_common(rtenhip_ctx* ctx, int is_max, const rtenhip_tensor* x,
                                  const int64_t kernel[2], const int64_t strides[2], int pad_mode,
                                  const int64_t pads[4], int count_include_pad, rtenhip_tensor* y) {
  Ctx* cx = C_(ctx);
  if (!x) return fail(RTENHIP_MISSING_INPUTS, "Missing inputs");
  if (x->ndim != 4) return fail(RTENHIP_INVALID_VALUE, "Expected input to have 4 dims");
  int64_t ohw[2], fp[4];
  int64_t st2[2] = {strides ? strides[0] : 1, strides ? strides[1] : 1};
  rtenhip_status st = output_size_and_padding(x->shape[2], x->shape[3], kernel[0], kernel[1],
                                              st2[0], st2[1], pad_mode, pads, 1, 1, ohw, fp);
  if (st) return st;
  int64_t os[4] = {x->shape[0], x->shape[1], ohw[0], ohw[1]};
  st = check_out_shape(y, os, 4);
  if (st) return st;
  const float* xd = contiguous(cx, *x, 0, &st);
  if (st) return st;
  return launch_pool(is_max, xd, y->data, x->shape[0] * x->shape[1], (int)x->shape[2],
                     (int)x->shape[3], (int)ohw[0], (int)ohw[1], (int)kernel[0], (int)kernel[1],
                     (int)st2[0], (int)st2[1], (int)fp[0], (int)fp[1], count_include_pad,
                     cx->stream);
}

rtenhip_status rtenhip_max_pool_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x,
                                    const int64_t kernel[2], const int64_t strides[2],
                                    int pad_mode, const int64_t pads[4], rtenhip_tensor* y) {
  return pool_common(ctx, 1, x, kernel, strides, pad_mode, pads, 0, y);
}

rtenhip_status rtenhip_average_pool_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x,
                                        const int64_t kernel[2], const int64_t strides[2],
                                        int pad_mode, const int64_t pads[4],
                                        int count_include_pad, rtenhip_tensor* y) {
  return pool_common(ctx, 0, x, kernel, strides, pad_mode, pads, count_include_pad, y);
}

rtenhip_status rtenhip_global_average_pool_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x,
                                               rtenhip_tensor* y) {
  Ctx* cx = C_(ctx);
  if (!x) return fail(RTENHIP_MISSING_INPUTS, "Missing inputs");
  if (x->ndim != 4) return fail(RTENHIP_INVALID_VALUE, "Expected input to have 4 dims");
  int64_t os[4] = {x->shape[0], x->shape[1], 1, 1};
  rtenhip_status st = check_out_shape(y, os, 4);
  if (st) return st;
  const float* xd = contiguous(cx, *x, 0, &st);
  if (st) return st;
  return launch_gap(xd, y->data, x->shape[0] * x->shape[1], x->shape[2] * x->shape[3],
                    cx->stream);
}

rtenhip_status rtenhip_batch_norm_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x,
                                      const float* scale, const float* bias, const float* mean,
                                      const float* var, float epsilon, rtenhip_tensor* y) {
  Ctx* cx = C_(ctx);
  if (!x || !scale || !bias || !mean || !var) return fail(RTENHIP_MISSING_INPUTS, "Missing inputs");
  if (x->ndim < 3) return fail(RTENHIP_INVALID_VALUE, "Input must have at least 3 dims");
  rtenhip_status st = check_out_shape(y, x->shape, x->ndim);
  if (st) return st;
  const float* xd = contiguous(cx, *x, 0, &st);
  if (st) return st;
  int64_t inner = 1;
  for (int i = 2; i < x->ndim; i++) inner *= x->shape[i];
  return launch_batch_norm(xd, y->data, x->shape[0], x->shape[1], inner, scale, bias, mean, var,
                           epsilon, cx->stream);
}

static int64_t resolve_axis(int64_t axis, int ndim, bool* ok) {
  *ok = true;
  if (axis < 0) axis += ndim;
  if (axis < 0 || axis >= ndim) *ok = false;
  return axis;
}

rtenhip_status rtenhip_log_softmax_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x, int64_t axis,
                                       rtenhip_tensor* y) {
  // LogSoftmax (src/ops/norm.rs:381-430): softmax_lanes' axis move is a
  // layout change only, so the kernel walks the axis in place with stride
  // `inner`.
  Ctx* cx = C_(ctx);
  if (!x) return fail(RTENHIP_MISSING_INPUTS, "Missing inputs");
  bool ok;
  const int64_t ax = resolve_axis(axis, x->ndim, &ok);
  if (!ok) return fail(RTENHIP_INVALID_VALUE, "Axis is invalid");
  rtenhip_status st = check_out_shape(y, x->shape, x->ndim);
  if (st) return st;
  const float* xd = contiguous(cx, *x, 0, &st);
  if (st) return st;
  int64_t outer = 1, inner = 1;
  for (int i = 0; i < ax; i++) outer *= x->shape[i];
  for (int i = (int)ax + 1; i < x->ndim; i++) inner *= x->shape[i];
  return launch_log_softmax(xd, y->data, outer, x->shape[ax], inner, cx->stream);
}

rtenhip_status rtenhip_instance_norm_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x, const float* scale,
                                         const float* bias, int64_t n_channels, float epsilon,
                                         rtenhip_tensor* y) {
  // InstanceNormalization (src/ops/norm.rs:131-198).
  Ctx* cx = C_(ctx);
  if (!x || !scale || !bias) return fail(RTENHIP_MISSING_INPUTS, "Missing inputs");
  if (x->ndim < 2) return fail(RTENHIP_INVALID_VALUE, "expected input with >= 2 dims");
  if (n_channels != x->shape[1]) return fail(RTENHIP_INVALID_VALUE, "scale length should match channel count");
  rtenhip_status st = check_out_shape(y, x->shape, x->ndim);
  if (st) return st;
  const float* xd = contiguous(cx, *x, 0, &st);
  if (st) return st;
  int64_t len = 1;
  for (int i = 2; i < x->ndim; i++) len *= x->shape[i];
  return launch_instance_norm(xd, y->data, x->shape[0], x->shape[1], len, scale, bias, epsilon, cx->stream);
}

rtenhip_status rtenhip_reduce_mean_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x, const int32_t* axes,
                                       int32_t n_axes, int keep_dims, rtenhip_tensor* y) {
  // reduce (src/ops/reduce.rs:225-330) with the MeanReducer (334-353).
  Ctx* cx = C_(ctx);
  if (!x || !y) return fail(RTENHIP_MISSING_INPUTS, "Missing inputs");
  const int nd = x->ndim;
  std::vector<int> res;
  if (n_axes <= 0 || !axes) {
    for (int d = 0; d < nd; d++) res.push_back(d);
  } else {
    for (int i = 0; i < n_axes; i++) {
      bool ok;
      const int64_t a = resolve_axis(axes[i], nd, &ok);
      if (!ok) return fail(RTENHIP_INVALID_VALUE, "Axis is invalid");
      res.push_back((int)a);
    }
  }
  std::sort(res.begin(), res.end());
  const int64_t n = numel(*x);
  if (nd > 0 && n == 0) return fail(RTENHIP_INVALID_VALUE, "Cannot reduce empty tensor");
  std::vector<bool> red(nd, false);
  for (int a : res) red[a] = true;
  int64_t os[RTENHIP_MAX_DIMS];
  int on = 0;
  for (int d = 0; d < nd; d++)
    if (!red[d]) os[on++] = x->shape[d];
    else if (keep_dims) os[on++] = 1;
  rtenhip_status st = check_out_shape(y, os, on);
  if (st) return st;
  if (!is_contiguous(*y)) return fail(RTENHIP_UNSUPPORTED_VALUE, "output must be contiguous");
  // reduced_inner_dims: the sorted axes equal to ndim-1, ndim-2, ... (only a
  // single last axis in practice), with contiguous data -> reduce_slice.
  bool inner = nd > 0;
  for (size_t i = 0; i < res.size(); i++) inner = inner && res[i] == nd - 1 - (int)i;
  if (inner && is_contiguous(*x)) {
    const int64_t len = (int)res.size() == nd ? n : x->strides[nd - 1 - (int)res.size()];
    return launch_reduce_mean_rows(x->data, y->data, n / len, len, cx->stream);
  }
  ReduceDesc d{};
  d.n_out = 1;
  d.n_red = 1;
  for (int k = 0; k < nd; k++) {
    if (red[k]) {
      d.rshape[d.nr] = x->shape[k];
      d.rstride[d.nr++] = x->strides[k];
      d.n_red *= x->shape[k];
    } else {
      d.kshape[d.nk] = x->shape[k];
      d.kstride[d.nk++] = x->strides[k];
      d.n_out *= x->shape[k];
    }
  }
  return launch_reduce_mean_iter(x->data, y->data, d, cx->stream);
}

rtenhip_status rtenhip_layer_norm_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x,
                                      const rtenhip_tensor* scale, const rtenhip_tensor* bias,
                                      int64_t axis, float epsilon, rtenhip_tensor* y) {
  Ctx* cx = C_(ctx);
  if (!x || !scale) return fail(RTENHIP_MISSING_INPUTS, "Missing inputs");
  bool ok;
  int64_t ax = resolve_axis(axis, x->ndim, &ok);
  if (!ok) return fail(RTENHIP_INVALID_VALUE, "Axis is invalid");
  int64_t row = 1;
  for (int i = (int)ax; i < x->ndim; i++) row *= x->shape[i];
  // scale / bias must broadcast to the input; the fused kernel supports the
  // normalized-shape case (the one LayerNormalization models use).
  if (numel(*scale) != row || !is_contiguous(*scale))
    return fail(RTENHIP_UNSUPPORTED_VALUE, "`scale` must have the normalized shape");
  if (bias && bias->data && (numel(*bias) != row || !is_contiguous(*bias)))
    return fail(RTENHIP_UNSUPPORTED_VALUE, "`bias` must have the normalized shape");
  rtenhip_status st = check_out_shape(y, x->shape, x->ndim);
  if (st) return st;
  const float* xd = contiguous(cx, *x, 0, &st);
  if (st) return st;
  int64_t rows = row ? numel(*x) / row : 0;
  return launch_layer_norm(xd, y->data, rows, row, scale->data,
                           bias && bias->data ? bias->data : nullptr, epsilon, cx->stream);
}

rtenhip_status rtenhip_softmax_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x, int64_t axis,
                                   rtenhip_tensor* y) {
  Ctx* cx = C_(ctx);
  if (!x) return fail(RTENHIP_MISSING_INPUTS, "Missing inputs");
  bool ok;
  int64_t ax = resolve_axis(axis, x->ndim, &ok);
  if (!ok) return fail(RTENHIP_INVALID_VALUE, "Axis is invalid");
  rtenhip_status st = check_out_shape(y, x->shape, x->ndim);
  if (st) return st;
  const int nd = x->ndim;
  if (ax == nd - 1) {
    const float* xd = contiguous(cx, *x, 0, &st);
    if (st) return st;
    int64_t len = x->shape[nd - 1];
    return launch_softmax(xd, y->data, len ? numel(*x) / len : 0, len, cx->stream);
  }
  // softmax_lanes (norm.rs:332-379): move the axis last, make contiguous,
  // apply, move back.
  rtenhip_tensor perm = *x;
  int k = 0;
  for (int i = 0; i < nd; i++)
    if (i != ax) {
      perm.shape[k] = x->shape[i];
      perm.strides[k] = x->strides[i];
      k++;
    }
  perm.shape[k] = x->shape[ax];
  perm.strides[k] = x->strides[ax];
  int64_t n = numel(*x);
  float* t0 = cx->scratch_floats(n, 0);
  float* t1 = cx->scratch_floats(n, 1);
  if (!t0 || !t1) return fail(RTENHIP_HIP_ERROR, "scratch allocation failed");
  st = launch_copy_strided(perm, t0, cx->stream);
  if (st) return st;
  int64_t len = x->shape[ax];
  st = launch_softmax(t0, t1, len ? n / len : 0, len, cx->stream);
  if (st) return st;
  // Move back: view t1 (shape perm) with the axis at `ax`.
  rtenhip_tensor back{};
  back.data = t1;
  back.ndim = nd;
  int64_t pstr[RTENHIP_MAX_DIMS];
  int64_t s = 1;
  for (int i = nd - 1; i >= 0; i--) {
    pstr[i] = s;
    s *= perm.shape[i];
  }
  k = 0;
  for (int i = 0; i < nd; i++) {
    back.shape[i] = x->shape[i];
    if (i == ax)
      back.strides[i] = pstr[nd - 1];
    else
      back.strides[i] = pstr[k++];
  }
  return launch_copy_strided(back, y->data, cx->stream);
}

rtenhip_status rtenhip_unary_f32(rtenhip_ctx* ctx, int op, const rtenhip_tensor* x, float p0,
                                 float p1, rtenhip_tensor* y) {
  Ctx* cx = C_(ctx);
  if (!x) return fail(RTENHIP_MISSING_INPUTS, "Missing inputs");
  rtenhip_status st = check_out_shape(y, x->shape, x->ndim);
  if (st) return st;
  const float* xd = contiguous(cx, *x, 0, &st);
  if (st) return st;
  return launch_unary(op, xd, y->data, numel(*x), p0, p1, cx->stream);
}

rtenhip_status rtenhip_binary_f32(rtenhip_ctx* ctx, int op, const rtenhip_tensor* a,
                                  const rtenhip_tensor* b, rtenhip_tensor* y) {
  if (!a || !b) return fail(RTENHIP_MISSING_INPUTS, "Missing inputs");
  return binary_impl(C_(ctx), op, *a, *b, y);
}

}  // extern "C"
