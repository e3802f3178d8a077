// ConvTranspose (src/ops/conv.rs:329-577) on the device: the column matrix
// col[n] = kernel^T @ x[n] of the reference's per-image gemm is one pointwise
// conv over the whole batch (weights transposed to [O*kh*kw, C, 1, 1]; the
// LDS-DMA GEMM keeps the KC = 256 block order, so it is the same gemm), then
// col2im_kernel adds the columns in the reference's (ky, kx) order.
#include <algorithm>

#include "ctx.h"

namespace rtenhip {

struct ConvTransposePlan {
  int64_t N, C, H, W, O, kh, kw, sh, sw, OH, OW, pad_top, pad_left;
  bool one_d;
};

// conv_transpose_output_size_and_padding (conv.rs:382-440) plus the shape and
// stride checks of conv_transpose (443-502).  As in the reference, element [1]
// of the padding is used as the left pad, which for Same padding is the bottom
// one (conv.rs:420-424 orders Same pads [top, bottom, left, right]).
static rtenhip_status plan_conv_transpose(const rtenhip_tensor* x, const rtenhip_tensor* w,
                                          int pad_mode, const int64_t* pads,
                                          const int64_t* strides, ConvTransposePlan& p) {
  if (!x || !w) return fail(RTENHIP_MISSING_INPUTS, "Missing inputs");
  int64_t p4[4] = {0, 0, 0, 0};
  if (x->ndim == 3) {
    if (w->ndim != 3) return fail(RTENHIP_INVALID_VALUE, "Expected kernel to have 3 dims");
    p.one_d = true;
    p.N = x->shape[0], p.C = x->shape[1], p.H = 1, p.W = x->shape[2];
    p.O = w->shape[1], p.kh = 1, p.kw = w->shape[2];
    if (!strides) return fail(RTENHIP_INVALID_VALUE, "expected 1 stride value");
    p.sh = 1, p.sw = strides[0];
    if (pads) p4[1] = pads[0], p4[3] = pads[1];
    if (w->shape[0] != p.C)
      return fail(RTENHIP_INCOMPATIBLE_INPUT_SHAPES,
                  "Input channels does not match kernel input channels");
  } else {
    if (x->ndim != 4) return fail(RTENHIP_INVALID_VALUE, "Expected input to have 4 dims");
    if (w->ndim != 4) return fail(RTENHIP_INVALID_VALUE, "Expected kernel to have 4 dims");
    p.one_d = false;
    p.N = x->shape[0], p.C = x->shape[1], p.H = x->shape[2], p.W = x->shape[3];
    p.O = w->shape[1], p.kh = w->shape[2], p.kw = w->shape[3];
    if (w->shape[0] != p.C)
      return fail(RTENHIP_INCOMPATIBLE_INPUT_SHAPES,
                  "Input channels does not match kernel input channels");
    if (!strides) return fail(RTENHIP_INVALID_VALUE, "expected 2 stride values");
    p.sh = strides[0], p.sw = strides[1];
    if (pads)
      for (int i = 0; i < 4; i++) p4[i] = pads[i];
  }
  if (p.sh == 0 || p.sw == 0) return fail(RTENHIP_INVALID_VALUE, "Strides must be > 0");
  if (p.H == 0 || p.W == 0) return fail(RTENHIP_INVALID_VALUE, "Input width and height must be > 0");
  const int64_t full_h = (p.H - 1) * p.sh + p.kh, full_w = (p.W - 1) * p.sw + p.kw;
  if (pad_mode == 1) {
    p.OH = p.H * p.sh;
    p.OW = p.W * p.sw;
    if (full_h < p.OH || full_w < p.OW) return fail(RTENHIP_INVALID_VALUE, "Input is too small");
    const int64_t pad_h = full_h - p.OH;
    p.pad_top = pad_h / 2;
    p.pad_left = (pad_h + 1) / 2;  // the reference's [1] = bottom pad (see above)
  } else {
    if (full_h < p4[0] + p4[2] || full_w < p4[1] + p4[3])
      return fail(RTENHIP_INVALID_VALUE, "Input is too small");
    p.OH = full_h - (p4[0] + p4[2]);
    p.OW = full_w - (p4[1] + p4[3]);
    p.pad_top = p4[0];
    p.pad_left = p4[1];
  }
  return RTENHIP_OK;
}

rtenhip_status conv_transpose_impl(Ctx* c, const rtenhip_tensor* x, const rtenhip_tensor* w,
                                   const float* bias, int pad_mode, const int64_t* pads,
                                   const int64_t* strides, rtenhip_tensor* y) {
  ConvTransposePlan p;
  rtenhip_status st = plan_conv_transpose(x, w, pad_mode, pads, strides, p);
  if (st) return st;
  int64_t os[4] = {p.N, p.O, p.OH, p.OW};
  if (p.one_d) os[2] = p.OW;
  const int ond = p.one_d ? 3 : 4;
  bool ok = y && y->ndim == ond && is_contiguous(*y);
  for (int i = 0; ok && i < ond; i++) ok = y->shape[i] == os[i];
  if (!ok) return fail(RTENHIP_INCORRECT_OUTPUT_TYPE, "Output has wrong shape");
  if (p.N * p.O * p.OH * p.OW == 0) return RTENHIP_OK;
  const int64_t M = p.O * p.kh * p.kw;
  hipStream_t s = c->stream;
  // kernel^T as conv weights [M, C, 1, 1] (w viewed as [C, M] with any strides
  // collapsing to the reference's reshaped contiguous kernel).
  float* wt = c->scratch_floats((size_t)(M * p.C), 4);
  float* col = c->scratch_floats((size_t)(p.N * M * p.H * p.W), 5);
  if (!wt || !col) return fail(RTENHIP_HIP_ERROR, "scratch allocation failed");
  const float* wdata = w->data;
  if (!is_contiguous(*w)) {
    float* tmp = c->scratch_floats((size_t)(M * p.C), 1);
    if (!tmp) return fail(RTENHIP_HIP_ERROR, "scratch allocation failed");
    if ((st = launch_copy_strided(*w, tmp, s))) return st;
    wdata = tmp;
  }
  rtenhip_tensor wv{};
  wv.data = const_cast<float*>(wdata);
  wv.ndim = 2;
  wv.shape[0] = M, wv.shape[1] = p.C;
  wv.strides[0] = 1, wv.strides[1] = M;
  if ((st = launch_copy_strided(wv, wt, s))) return st;
  rtenhip_tensor x4 = *x, w4{}, col4{};
  if (p.one_d) {
    x4.ndim = 4;
    x4.shape[0] = p.N, x4.shape[1] = p.C, x4.shape[2] = 1, x4.shape[3] = p.W;
    x4.strides[0] = x->strides[0], x4.strides[1] = x->strides[1];
    x4.strides[2] = p.W * x->strides[2], x4.strides[3] = x->strides[2];
  }
  w4.data = wt;
  w4.ndim = 4;
  w4.shape[0] = M, w4.shape[1] = p.C, w4.shape[2] = 1, w4.shape[3] = 1;
  w4.strides[0] = p.C, w4.strides[1] = 1, w4.strides[2] = 1, w4.strides[3] = 1;
  col4.data = col;
  col4.ndim = 4;
  col4.shape[0] = p.N, col4.shape[1] = M, col4.shape[2] = p.H, col4.shape[3] = p.W;
  col4.strides[3] = 1, col4.strides[2] = p.W, col4.strides[1] = p.H * p.W, col4.strides[0] = M * p.H * p.W;
  const int64_t zero_pads[4] = {0, 0, 0, 0}, ones[2] = {1, 1};
  st = conv_impl(c, &x4, &w4, nullptr, 0, zero_pads, ones, ones, 1, nullptr, 0, 0.f, 0.f, &col4);
  if (st) return st;
  return launch_col2im(col, bias, y->data, p.N, p.O, p.OH, p.OW, p.H, p.W, p.kh, p.kw, p.sh, p.sw,
                       p.pad_top, p.pad_left, s);
}

rtenhip_status conv_transpose_output_shape(const rtenhip_tensor* x, const rtenhip_tensor* w,
                                           int pad_mode, const int64_t* pads,
                                           const int64_t* strides, int64_t* out_shape,
                                           int32_t* out_ndim) {
  ConvTransposePlan p;
  rtenhip_status st = plan_conv_transpose(x, w, pad_mode, pads, strides, p);
  if (st) return st;
  out_shape[0] = p.N;
  out_shape[1] = p.O;
  if (p.one_d) {
    out_shape[2] = p.OW;
    *out_ndim = 3;
  } else {
    out_shape[2] = p.OH;
    out_shape[3] = p.OW;
    *out_ndim = 4;
  }
  return RTENHIP_OK;
}

}  // namespace rtenhip

using namespace rtenhip;

extern "C" {

rtenhip_status rtenhip_conv_transpose_output_shape(const rtenhip_tensor* x,
                                                   const rtenhip_tensor* w, int pad_mode,
                                                   const int64_t* pads, const int64_t* strides,
                                                   int64_t* out_shape, int32_t* out_ndim) {
  return conv_transpose_output_shape(x, w, pad_mode, pads, strides, out_shape, out_ndim);
}

rtenhip_status rtenhip_conv_transpose_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x,
                                          const rtenhip_tensor* w, const float* bias,
                                          int pad_mode, const int64_t* pads,
                                          const int64_t* strides, rtenhip_tensor* y) {
  return conv_transpose_impl(reinterpret_cast<Ctx*>(ctx), x, w, bias, pad_mode, pads, strides, y);
}

}  // extern "C"
