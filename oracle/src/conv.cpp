#include <vector>
// CPU restatement of RTen's Conv and pooling operators (test infrastructure;
// see rten_oracle.h).
//
// Follows src/ops/conv.rs:24-280 (dispatcher, pointwise, im2col path),
// src/ops/conv/im2col.rs:75-260 (VirtualIm2Col), src/ops/conv/depthwise.rs:24-203
// and src/ops/pooling.rs:27-375.
#include <immintrin.h>
#include <omp.h>

#include <algorithm>
#include <limits>

#include "common.h"

namespace orc {

// VirtualIm2Col (im2col.rs:44-260): row r = (c, ky, kx), col = (oy, ox).
// VirtualIm2Col::new (im2col.rs:75-181): offset tables built once per conv
// geometry -- per row the channel, y and x offsets, per column (padded to a
// multiple of the panel width) the patch corner's y and x offsets, all
// premultiplied by the image strides -- plus the largest valid y / x offsets.
struct Im2ColTables {
  std::vector<int32_t> row_chan, row_y, row_x;
  std::vector<int32_t> col_y, col_x;
  int32_t max_y = 0, max_x = 0;
  Im2ColTables(int64_t C, int64_t H, int64_t W, int64_t kh, int64_t kw, int64_t sh, int64_t sw, int64_t dh,
               int64_t dw, int64_t pt, int64_t pl, int64_t oh, int64_t ow, int64_t panel) {
    for (int64_t c = 0; c < C; c++)
      for (int64_t ky = 0; ky < kh; ky++)
        for (int64_t kx = 0; kx < kw; kx++) {
          row_chan.push_back((int32_t)(c * H * W));
          row_y.push_back((int32_t)(W * ky * dh));
          row_x.push_back((int32_t)(kx * dw));
        }
    const int64_t n_cols = oh * ow, padded = (n_cols + panel - 1) / panel * panel;
    for (int64_t col = 0; col < padded; col++) {
      const int64_t py = col / ow, px = col % ow;
      col_y.push_back((int32_t)((py * sh - pt) * W));
      col_x.push_back((int32_t)(px * sw - pl));
    }
    max_y = (int32_t)((H - 1) * W);
    max_x = (int32_t)(W - 1);
  }
};

struct Im2Col : VirtualB {
  const float* img;  // [C,H,W] contiguous
  const Im2ColTables* t;
  int64_t n_rows, n_cols;
  int64_t rows() const override { return n_rows; }
  int64_t cols() const override { return n_cols; }
  // pack_b_impl (im2col.rs:190-260) for the AVX2 kernel (NR = 16 = 2 x 8
  // lanes): per column panel, per row, a masked gather of 8 lanes twice;
  // offsets in the padding region read as 0.
  void pack_b(float* out, int64_t nr, int64_t k0, int64_t k1, int64_t c0,
              int64_t c1) const override {
    const int64_t c1p = c0 + (c1 - c0 + nr - 1) / nr * nr;
    const __m256i zero = _mm256_setzero_si256(), neg1 = _mm256_set1_epi32(-1);
    const __m256i ymax1 = _mm256_set1_epi32(t->max_y + 1), xmax1 = _mm256_set1_epi32(t->max_x + 1);
    float* o = out;
    for (int64_t pc = c0; pc < c1p; pc += nr) {
      for (int64_t r = k0; r < k1; r++) {
        const __m256i rc = _mm256_set1_epi32(t->row_chan[r]), ry = _mm256_set1_epi32(t->row_y[r]),
                      rx = _mm256_set1_epi32(t->row_x[r]);
        for (int64_t i = 0; i < nr; i += 8) {
          const __m256i y = _mm256_add_epi32(_mm256_loadu_si256((const __m256i*)(t->col_y.data() + pc + i)), ry);
          const __m256i x = _mm256_add_epi32(_mm256_loadu_si256((const __m256i*)(t->col_x.data() + pc + i)), rx);
          const __m256i off = _mm256_add_epi32(rc, _mm256_add_epi32(y, x));
          const __m256i ok = _mm256_and_si256(
              _mm256_and_si256(_mm256_cmpgt_epi32(y, neg1), _mm256_cmpgt_epi32(ymax1, y)),
              _mm256_and_si256(_mm256_cmpgt_epi32(x, neg1), _mm256_cmpgt_epi32(xmax1, x)));
          const __m256 v = _mm256_mask_i32gather_ps(_mm256_castsi256_ps(zero), img, off, _mm256_castsi256_ps(ok), 4);
          _mm256_storeu_ps(o, v);
          o += 8;
        }
      }
    }
  }
};

// calc_output_size_and_padding (pooling.rs:27-89).
static int output_size_and_padding(int64_t in_h, int64_t in_w, int64_t k_h, int64_t k_w,
                                   int64_t stride_h, int64_t stride_w, int pad_mode,
                                   const int64_t* pads_in, int64_t dil_y, int64_t dil_x,
                                   int64_t out_hw[2], int64_t pads[4]) {
  if (dil_y == 0 || dil_x == 0) return fail(ORC_INVALID_VALUE, "Dilations must be > 0");
  if (stride_h == 0 || stride_w == 0) return fail(ORC_INVALID_VALUE, "Strides must be > 0");
  if (pad_mode == 1) {
    int64_t out_h = (in_h + stride_h - 1) / stride_h, out_w = (in_w + stride_w - 1) / stride_w;
    int64_t th = std::max<int64_t>(0, (out_h - 1) * stride_h + (k_h - 1) * dil_y + 1 - in_h);
    int64_t tw = std::max<int64_t>(0, (out_w - 1) * stride_w + (k_w - 1) * dil_x + 1 - in_w);
    pads[0] = th / 2;
    pads[1] = tw / 2;
    pads[2] = (th + 1) / 2;
    pads[3] = (tw + 1) / 2;
    out_hw[0] = out_h;
    out_hw[1] = out_w;
    return ORC_OK;
  }
  for (int i = 0; i < 4; i++) pads[i] = pads_in[i];
  int64_t ph = in_h + pads[0] + pads[2], pw = in_w + pads[1] + pads[3];
  int64_t dkh = k_h + (k_h - 1) * (dil_y - 1), dkw = k_w + (k_w - 1) * (dil_x - 1);
  if (ph < dkh || pw < dkw) return fail(ORC_INVALID_VALUE, "Input too small for kernel size");
  out_hw[0] = (ph - dil_y * (k_h - 1) - 1) / stride_h + 1;
  out_hw[1] = (pw - dil_x * (k_w - 1) - 1) / stride_w + 1;
  return ORC_OK;
}

// conv_2d_depthwise (depthwise.rs:127-203) + conv_2d_depthwise_block (49-120).
// Per output row: init with bias, then for each (ky, kx) in order
// out += in * w with separate mul/add roundings.
static void conv_depthwise(const float* x, int64_t N, int64_t C, int64_t H, int64_t W,
                           const float* w, int64_t kh, int64_t kw, const float* bias,
                           const int64_t pads[4], int64_t sh, int64_t sw, int64_t dh, int64_t dw,
                           int64_t oh, int64_t ow, float* y) {
  int64_t pt = pads[0], pl = pads[1];
  std::vector<int64_t> omin(kw), omax(kw), imin(kw);
  for (int64_t kx = 0; kx < kw; kx++) {
    // min_max_out_x_coords (depthwise.rs:24-38)
    int64_t mn = std::max<int64_t>(0, pl - kx * dw);
    int64_t t = std::max<int64_t>(0, W + pl - kx * dw);
    int64_t mx = std::min<int64_t>((t + sw - 1) / sw, ow);
    omin[kx] = mn;
    omax[kx] = mx;
    imin[kx] = mn * sw + kx * dw - pl;
  }
#pragma omp parallel for collapse(2) schedule(dynamic, 4)
  for (int64_t n = 0; n < N; n++)
    for (int64_t c = 0; c < C; c++) {
      const float* in = x + (n * C + c) * H * W;
      float* out = y + (n * C + c) * oh * ow;
      const float* kern = w + c * kh * kw;
      float init = bias ? bias[c] : 0.f;
      for (int64_t oy = 0; oy < oh; oy++) {
        float* orow = out + oy * ow;
        for (int64_t ox = 0; ox < ow; ox++) orow[ox] = init;
        for (int64_t ky = 0; ky < kh; ky++) {
          int64_t iy = oy * sh + ky * dh;
          if (iy < pt || iy >= H + pt) continue;
          const float* irow = in + (iy - pt) * W;
          for (int64_t kx = 0; kx < kw; kx++) {
            float s = kern[ky * kw + kx];
            const float* src = irow + imin[kx];
            for (int64_t ox = omin[kx]; ox < omax[kx]; ox++) {
              float prod = src[(ox - omin[kx]) * sw] * s;
              orow[ox] = orow[ox] + prod;
            }
          }
        }
      }
    }
}

static int conv2d(const float* x, const int64_t xs[4], const float* w, const int64_t ws[4],
                  const float* bias, int pad_mode, const int64_t* pads_in,
                  const int64_t strides[2], const int64_t dil[2], int64_t groups, float* y,
                  int64_t ys[4]) {
  int64_t N = xs[0], C = xs[1], H = xs[2], W = xs[3];
  int64_t O = ws[0], KC = ws[1], kh = ws[2], kw = ws[3];
  int64_t out_hw[2], pads[4];
  int st = output_size_and_padding(H, W, kh, kw, strides[0], strides[1], pad_mode, pads_in,
                                   dil[0], dil[1], out_hw, pads);
  if (st) return st;
  int64_t oh = out_hw[0], ow = out_hw[1];
  ys[0] = N;
  ys[1] = O;
  ys[2] = oh;
  ys[3] = ow;
  bool has_pad = pads[0] > 0 || pads[1] > 0 || pads[2] > 0 || pads[3] > 0;
  if (kh == 1 && kw == 1 && !has_pad && groups == 1 && strides[0] == 1 && strides[1] == 1 &&
      dil[0] == 1 && dil[1] == 1) {
    // conv_2d_pointwise (conv.rs:24-68): serial loop over images, one GEMM
    // each (which parallelizes internally).
    Mat A{w, O, C, C, 1};
    for (int64_t n = 0; n < N; n++) {
      Mat B{x + n * C * H * W, C, H * W, H * W, 1};
      gemm_impl(y + n * O * H * W, H * W, A, &B, nullptr, 1.f, 0.f, bias, false);
    }
    return ORC_OK;
  }
  int64_t opg = O / std::max<int64_t>(groups, 1), ipg = C / std::max<int64_t>(groups, 1);
  if (groups == 0 || ipg != KC)
    return fail(ORC_INCOMPATIBLE_INPUT_SHAPES,
                "Input channels (per group) does not match kernel input channels");
  if (C % groups != 0 || O % groups != 0)
    return fail(ORC_INCOMPATIBLE_INPUT_SHAPES,
                "Input channels and output channels must be divisible by group count");
  if (C == O && groups == C) {
    conv_depthwise(x, N, C, H, W, w, kh, kw, bias, pads, strides[0], strides[1], dil[0], dil[1],
                   oh, ow, y);
    return ORC_OK;
  }
  int64_t P = oh * ow;
  for (int64_t g = 0; g < groups; g++) {
    Mat A{w + g * opg * KC * kh * kw, opg, KC * kh * kw, KC * kh * kw, 1};
    const float* gb = bias ? bias + g * opg : nullptr;
    // Per-image parallelism (conv.rs:243-270, par_bridge).  Each image's
    // GEMM then runs on its worker; summation order is unaffected.
    bool par_images = N > 1;
    const Im2ColTables tables(ipg, H, W, kh, kw, strides[0], strides[1], dil[0], dil[1], pads[0], pads[1], oh,
                              ow, 16);
#pragma omp parallel for schedule(dynamic, 1) if (par_images)
    for (int64_t n = 0; n < N; n++) {
      Im2Col im;
      im.img = x + (n * C + g * ipg) * H * W;
      im.t = &tables;
      im.n_rows = ipg * kh * kw;
      im.n_cols = oh * ow;
      gemm_impl(y + (n * O + g * opg) * P, P, A, nullptr, &im, 1.f, 0.f, gb, par_images);
    }
  }
  return ORC_OK;
}

// pool_impl (pooling.rs:104-238).  fold over the window in (ky, kx) order.
template <typename Fold, typename Avg>
static int pool_impl(const float* x, const int64_t xs[4], const int64_t kernel[2],
                     const int64_t strides[2], int pad_mode, const int64_t* pads_in, float init,
                     Fold fold, Avg avg, float* y, int64_t ys[4]) {
  int64_t N = xs[0], C = xs[1], H = xs[2], W = xs[3];
  int64_t out_hw[2], pads[4];
  int st = output_size_and_padding(H, W, kernel[0], kernel[1], strides[0], strides[1], pad_mode,
                                   pads_in, 1, 1, out_hw, pads);
  if (st) return st;
  int64_t oh = out_hw[0], ow = out_hw[1], pt = pads[0], pl = pads[1];
  ys[0] = N;
  ys[1] = C;
  ys[2] = oh;
  ys[3] = ow;
#pragma omp parallel for collapse(2)
  for (int64_t n = 0; n < N; n++)
    for (int64_t c = 0; c < C; c++) {
      const float* in = x + (n * C + c) * H * W;
      float* out = y + (n * C + c) * oh * ow;
      for (int64_t oy = 0; oy < oh; oy++)
        for (int64_t ox = 0; ox < ow; ox++) {
          float acc = init;
          int64_t cnt = 0;
          for (int64_t ky = 0; ky < kernel[0]; ky++)
            for (int64_t kx = 0; kx < kernel[1]; kx++) {
              int64_t iy = oy * strides[0] + ky, ix = ox * strides[1] + kx;
              if (iy >= pt && iy < H + pt && ix >= pl && ix < W + pl) {
                acc = fold(acc, in[(iy - pt) * W + (ix - pl)]);
                cnt++;
              }
            }
          out[oy * ow + ox] = avg(acc, cnt);
        }
    }
  return ORC_OK;
}

}  // namespace orc

using namespace orc;

extern "C" {

int orc_output_size_and_padding(int64_t in_h, int64_t in_w, int64_t k_h, int64_t k_w,
                                int64_t stride_h, int64_t stride_w, int pad_mode,
                                const int64_t pads_in[4], int64_t dil_h, int64_t dil_w,
                                int64_t out_hw[2], int64_t pads_out[4]) {
  return output_size_and_padding(in_h, in_w, k_h, k_w, stride_h, stride_w, pad_mode, pads_in,
                                 dil_h, dil_w, out_hw, pads_out);
}

int orc_conv(const float* x, const int64_t* x_shape, int x_ndim, const float* w,
             const int64_t* w_shape, const float* bias, int pad_mode, const int64_t* pads,
             const int64_t* strides, const int64_t* dilations, int64_t groups, float* out,
             int64_t* out_shape) {
  if (x_ndim == 3) {
    // 1-D conv via 2-D (conv.rs:96-143).
    int64_t xs[4] = {x_shape[0], x_shape[1], 1, x_shape[2]};
    int64_t ws[4] = {w_shape[0], w_shape[1], 1, w_shape[2]};
    int64_t p2[4] = {0, pads ? pads[0] : 0, 0, pads ? pads[1] : 0};
    int64_t s2[2] = {1, strides[0]}, d2[2] = {1, dilations[0]};
    int64_t ys[4];
    int st = conv2d(x, xs, w, ws, bias, pad_mode, p2, s2, d2, groups, out, ys);
    if (st) return st;
    out_shape[0] = ys[0];
    out_shape[1] = ys[1];
    out_shape[2] = ys[3];
    return ORC_OK;
  }
  if (x_ndim != 4) return fail(ORC_INVALID_VALUE, "Input must have 4 dims (NCHW)");
  return conv2d(x, x_shape, w, w_shape, bias, pad_mode, pads, strides, dilations, groups, out,
                out_shape);
}

// conv_transpose_output_size_and_padding (src/ops/conv.rs:382-440).  The
// padding comes back ordered as the reference orders it: Same ->
// [top, bottom, left, right], Fixed -> [top, left, bottom, right];
// conv_transpose then reads elements [0] and [1] as the top and left pads in
// both cases (conv.rs:505, 535-541), which this restatement keeps.
int orc_conv_transpose_output_size(int64_t in_h, int64_t in_w, int64_t k_h, int64_t k_w,
                                   int pad_mode, const int64_t* pads_in, int64_t stride_h,
                                   int64_t stride_w, int64_t out_hw[2], int64_t pads_out[4]) {
  if (stride_h == 0 || stride_w == 0) return fail(ORC_INVALID_VALUE, "Strides must be > 0");
  if (in_h == 0 || in_w == 0) return fail(ORC_INVALID_VALUE, "Input width and height must be > 0");
  if (pad_mode == 1) {
    const int64_t out_h = in_h * stride_h, out_w = in_w * stride_w;
    const int64_t full_h = (in_h - 1) * stride_h + k_h, full_w = (in_w - 1) * stride_w + k_w;
    if (full_h < out_h || full_w < out_w) return fail(ORC_INVALID_VALUE, "Input is too small");
    const int64_t pad_h = full_h - out_h, pad_w = full_w - out_w;
    pads_out[0] = pad_h / 2;
    pads_out[1] = (pad_h + 1) / 2;
    pads_out[2] = pad_w / 2;
    pads_out[3] = (pad_w + 1) / 2;
    out_hw[0] = out_h;
    out_hw[1] = out_w;
    return ORC_OK;
  }
  const int64_t pt = pads_in[0], pl = pads_in[1], pb = pads_in[2], pr = pads_in[3];
  const int64_t full_h = (in_h - 1) * stride_h + k_h, full_w = (in_w - 1) * stride_w + k_w;
  if (full_h < pt + pb || full_w < pl + pr) return fail(ORC_INVALID_VALUE, "Input is too small");
  out_hw[0] = full_h - (pt + pb);
  out_hw[1] = full_w - (pl + pr);
  for (int i = 0; i < 4; i++) pads_out[i] = pads_in[i];
  return ORC_OK;
}

// conv_transpose (src/ops/conv.rs:443-535) + col2im (329-375): per image
// col[out_c*kh*kw, H*W] = kernel^T @ x_n (one gemm, alpha 1, no bias), then
// each output channel is filled with its bias (or 0) and the columns are
// added in (ky, kx, y, x) order.
int orc_conv_transpose(const float* x, const int64_t* x_shape, int x_ndim, const float* w,
                       const int64_t* w_shape, const float* bias, int pad_mode,
                       const int64_t* pads, const int64_t* strides, float* out,
                       int64_t* out_shape) {
  int64_t xs[4], ws[4], p4[4] = {0, 0, 0, 0}, st2[2];
  if (x_ndim == 3) {
    // 1-D as 2-D with H = 1 (conv.rs:453-480; Padding::expand_1d_to_2d).
    xs[0] = x_shape[0], xs[1] = x_shape[1], xs[2] = 1, xs[3] = x_shape[2];
    ws[0] = w_shape[0], ws[1] = w_shape[1], ws[2] = 1, ws[3] = w_shape[2];
    if (pads) p4[1] = pads[0], p4[3] = pads[1];
    st2[0] = 1, st2[1] = strides[0];
  } else if (x_ndim == 4) {
    for (int i = 0; i < 4; i++) xs[i] = x_shape[i], ws[i] = w_shape[i];
    if (pads)
      for (int i = 0; i < 4; i++) p4[i] = pads[i];
    st2[0] = strides[0], st2[1] = strides[1];
  } else {
    return fail(ORC_INVALID_VALUE, "Input must have 4 dims (NCHW)");
  }
  const int64_t N = xs[0], C = xs[1], H = xs[2], W = xs[3];
  const int64_t KC = ws[0], O = ws[1], kh = ws[2], kw = ws[3];
  if (C != KC)
    return fail(ORC_INCOMPATIBLE_INPUT_SHAPES, "Input channels does not match kernel input channels");
  int64_t ohw[2], pp[4];
  int st = orc_conv_transpose_output_size(H, W, kh, kw, pad_mode, p4, st2[0], st2[1], ohw, pp);
  if (st) return st;
  const int64_t OH = ohw[0], OW = ohw[1], pad_top = pp[0], pad_left = pp[1];
  const int64_t M = O * kh * kw, HW = H * W;
  std::vector<float> col((size_t)(M * HW));
  for (int64_t n = 0; n < N; n++) {
    const float* xn = x + n * C * HW;
    orc_gemm(col.data(), HW, w, 1, M, xn, HW, 1, M, HW, C, 1.f, 0.f, nullptr);
    float* on = out + n * O * OH * OW;
    for (int64_t c = 0; c < O; c++) {
      float* img = on + c * OH * OW;
      const float b = bias ? bias[c] : 0.f;
      for (int64_t i = 0; i < OH * OW; i++) img[i] = b;
      for (int64_t ky = 0; ky < kh; ky++)
        for (int64_t kx = 0; kx < kw; kx++) {
          const float* src = col.data() + ((c * kh + ky) * kw + kx) * HW;
          for (int64_t y = 0; y < H; y++) {
            const int64_t oy = y * st2[0] + ky;
            if (oy < pad_top || oy >= OH + pad_top) continue;
            for (int64_t xx = 0; xx < W; xx++) {
              const int64_t ox = xx * st2[1] + kx;
              if (ox < pad_left || ox >= OW + pad_left) continue;
              img[(oy - pad_top) * OW + (ox - pad_left)] += src[y * W + xx];
            }
          }
        }
    }
  }
  if (x_ndim == 3) {
    out_shape[0] = N, out_shape[1] = O, out_shape[2] = OW;
  } else {
    out_shape[0] = N, out_shape[1] = O, out_shape[2] = OH, out_shape[3] = OW;
  }
  return ORC_OK;
}

int orc_max_pool(const float* x, const int64_t x_shape[4], const int64_t kernel[2],
                 const int64_t strides[2], int pad_mode, const int64_t pads[4], float* out,
                 int64_t out_shape[4]) {
  // f32::max ignores NaN operands (returns the other one).
  return pool_impl(
      x, x_shape, kernel, strides, pad_mode, pads, -std::numeric_limits<float>::infinity(),
      [](float a, float b) { return std::fmax(a, b); }, [](float a, int64_t) { return a; }, out,
      out_shape);
}

int orc_average_pool(const float* x, const int64_t x_shape[4], const int64_t kernel[2],
                     const int64_t strides[2], int pad_mode, const int64_t pads[4],
                     int count_include_pad, float* out, int64_t out_shape[4]) {
  float klen = (float)(kernel[0] * kernel[1]);
  return pool_impl(
      x, x_shape, kernel, strides, pad_mode, pads, 0.f, [](float a, float b) { return a + b; },
      [=](float a, int64_t cnt) { return count_include_pad ? a / klen : a / (float)cnt; }, out,
      out_shape);
}

int orc_global_average_pool(const float* x, const int64_t x_shape[4], float* out) {
  // global_average_pool (pooling.rs:294-342): row-major sum per channel.
  int64_t N = x_shape[0], C = x_shape[1], HW = x_shape[2] * x_shape[3];
  float denom = (float)HW;
#pragma omp parallel for collapse(2)
  for (int64_t n = 0; n < N; n++)
    for (int64_t c = 0; c < C; c++) {
      const float* p = x + (n * C + c) * HW;
      float s = 0.f;
      for (int64_t i = 0; i < HW; i++) s += p[i];
      out[n * C + c] = s / denom;
    }
  return ORC_OK;
}

}  // extern "C"
