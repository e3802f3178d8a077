// Internal helpers shared by the HIP kernels and the host runtime.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/rten_hip.h"

namespace rtenhip {

// Division by an invariant divisor for 0 <= n < 2^31: q = (n * mul) >> shift
// with shift = 31 + ceil(log2 d), mul = ceil(2^shift / d) (exact in that range).
struct FastDiv {
  uint64_t mul;
  uint32_t shift;
};
inline FastDiv make_fastdiv(uint32_t d) {
  uint32_t l = 0;
  while ((uint64_t(1) << l) < d) l++;
  const uint32_t shift = 31 + l;
  return FastDiv{((uint64_t(1) << shift) + d - 1) / d, shift};
}

// Thread-local last error (rtenhip_last_error_message).
void set_error(int code, const std::string& msg);
rtenhip_status fail(rtenhip_status code, const char* msg);
rtenhip_status hip_fail(hipError_t e, const char* where);

#define RTENHIP_HIP_CHECK(expr)                              \
  do {                                                       \
    hipError_t _e = (expr);                                  \
    if (_e != hipSuccess) return ::rtenhip::hip_fail(_e, #expr); \
  } while (0)

// Launch-error check after a kernel launch.
#define RTENHIP_LAUNCH_CHECK() RTENHIP_HIP_CHECK(hipGetLastError())

inline int64_t numel(const rtenhip_tensor& t) {
  int64_t n = 1;
  for (int i = 0; i < t.ndim; i++) n *= t.shape[i];
  return n;
}

inline bool is_contiguous(const rtenhip_tensor& t) {
  int64_t s = 1;
  for (int i = t.ndim - 1; i >= 0; i--) {
    if (t.shape[i] != 1 && t.strides[i] != s) return false;
    s *= t.shape[i];
  }
  return true;
}

inline rtenhip_tensor make_tensor(float* data, const int64_t* shape, int ndim) {
  rtenhip_tensor t{};
  t.data = data;
  t.ndim = ndim;
  int64_t s = 1;
  for (int i = ndim - 1; i >= 0; i--) {
    t.shape[i] = shape[i];
    t.strides[i] = s;
    s *= shape[i];
  }
  return t;
}

struct Ctx;
hipStream_t stream_of(rtenhip_ctx* ctx);

// ---- kernel launchers (implemented in the .hip files) ----

// Implicit-GEMM engine (gemm_mfma.hip).  See GemmDesc.
struct GemmDesc {
  int M, N, K;
  // A[m,k] = a[m*a_m + k*a_k]
  const float* a;
  int64_t a_m, a_k;
  // B source: 0 dense B[k,n] = b[k*b_k + n*b_n]; 1 im2col of NCHW x;
  // 2 pointwise (1x1 s1 p0) conv of NCHW x.
  int bmode;
  const float* b;
  int64_t b_k, b_n;
  // conv geometry (bmode 1/2): per-group input [C,H,W] of image stride x_img
  int C, H, W, OW, P, sh, sw, pt, pl;
  int64_t x_img;
  const int2* ktab;  // bmode 1: per k {c*H*W + ky*dh*W + kx*dw, (ky*dh)<<16 | kx*dw}
  // output: omode 0 dense out[m*out_m + n]; 1 conv out[img*out_img + m*P + p]
  int omode;
  float* out;
  int64_t out_m, out_img;
  const float* bias;      // [M] or null
  const float* residual;  // same addressing as out, or null
  const float* cin;       // dense C input for beta != 0 (BMODE 0 only), or null
  float alpha, beta;
  int act;
  float act_lo, act_hi;
  // Batched MatMul (dense modes): blockIdx.y = flat batch index over up to 4
  // broadcast prefix dims; element offsets of a / b / out per prefix dim.
  int nbatch;  // 0 or 1 = not batched
  int nbp;
  int64_t pshape[4], pa[4], pb[4], po[4];
};
// Small-M GEMM split at KC blocks (workspace = gemm_smallm_ws_floats).
bool gemm_smallm_eligible(const GemmDesc& d);
// Tile configuration forced for the general MFMA GEMM (tuning/tests), -1 if none;
// while one is forced, dense GEMMs stay on that kernel.
int gemm_forced_cfg();
int64_t gemm_smallm_ws_floats(const GemmDesc& d);
rtenhip_status launch_gemm_smallm(const GemmDesc& d, float* ws, hipStream_t s);
rtenhip_status launch_gemm(const GemmDesc& d, hipStream_t s);

// gemv with the reference's summation order (gemm.rs:651-704, kernels.rs:26-194).
// cin (optional): the beta * C operand read from cin[c * cin_stride] instead
// of out (a broadcast Gemm C without materialising it into out first).
rtenhip_status launch_gemv(int64_t N, int64_t K, const float* a, const float* b, int64_t b_rs,
                           int64_t b_cs, float* out, float alpha, float beta, const float* bias,
                           int64_t ref_threads, hipStream_t s, const float* cin = nullptr,
                           int64_t cin_stride = 1);

// Holds stream s until *release (pinned host word) is non-zero or max_ms
// passes (timing runs only, elementwise.hip).
rtenhip_status launch_hold(int* word, double max_ms, hipStream_t s);

// Elementwise / pooling / normalisation (elementwise.hip, pool.hip, norm.hip).
rtenhip_status launch_unary(int op, const float* x, float* y, int64_t n, float p0, float p1,
                            hipStream_t s);
struct BcastDesc {
  int ndim;
  int64_t shape[RTENHIP_MAX_DIMS];
  int64_t sa[RTENHIP_MAX_DIMS], sb[RTENHIP_MAX_DIMS];
};
rtenhip_status launch_binary(int op, const float* a, const float* b, float* y, int64_t n,
                             const BcastDesc& d, int mode, int64_t inner, int64_t nb,
                             hipStream_t s);
rtenhip_status launch_batch_norm(const float* x, float* y, int64_t N, int64_t C, int64_t inner,
                                 const float* scale, const float* bias, const float* mean,
                                 const float* var, float eps, hipStream_t s);
rtenhip_status launch_pool(int is_max, const float* x, float* y, int64_t NC, int H, int W,
                           int OH, int OW, int kh, int kw, int sh, int sw, int pt, int pl,
                           int count_include_pad, hipStream_t s);
rtenhip_status launch_gap(const float* x, float* y, int64_t NC, int64_t HW, hipStream_t s);
// Streaming depthwise (dw_stream.hip) for 14x14 / 7x7 planes; false when the
// shape is not one it handles.
bool launch_depthwise_stream(const float* x, const float* w, const float* bias, float* y, int N, int C, int H,
                             int W, int OH, int OW, int kh, int kw, int sh, int sw, int dh, int dw, int pt, int pl,
                             const int* omin, const int* omax, const float* residual, int act, float lo, float hi,
                             hipStream_t s, rtenhip_status& st);
rtenhip_status launch_depthwise(const float* x, const float* w, const float* bias, float* y,
                                int N, int C, int H, int W, int OH, int OW, int kh, int kw,
                                int sh, int sw, int dh, int dw, int pt, int pl,
                                const float* residual, int act, float lo, float hi,
                                hipStream_t s);
rtenhip_status launch_softmax(const float* x, float* y, int64_t rows, int64_t len,
                              hipStream_t s);
// LogSoftmax over the middle axis of [outer, len, inner]; InstanceNorm over the
// contiguous planes of [N, C, len] (norm.hip).
rtenhip_status launch_log_softmax(const float* x, float* y, int64_t outer, int64_t len, int64_t inner,
                                  hipStream_t s);
rtenhip_status launch_instance_norm(const float* x, float* y, int64_t N, int64_t C, int64_t len,
                                    const float* scale, const float* bias, float eps, hipStream_t s);
struct PackedOut;
// pk: also store y as a MatMul's packed A (packed_a.h); only the rows kernel
// does (layer_norm_rows_ok), the call fails otherwise.
rtenhip_status launch_layer_norm(const float* x, float* y, int64_t rows, int64_t len,
                                 const float* scale, const float* bias, float eps,
                                 hipStream_t s, const PackedOut* pk = nullptr);
bool layer_norm_rows_ok(const float* x, float* y, int64_t len, const float* scale, const float* bias);
rtenhip_status launch_copy_strided(const rtenhip_tensor& src, float* dst, hipStream_t s);
// Strided view -> strided view copy of 4-byte elements (either dtype).
rtenhip_status launch_copy_view(const float* src, const int64_t* shape, const int64_t* src_strides, int ndim,
                                float* dst, const int64_t* dst_strides, hipStream_t s);
rtenhip_status launch_fill(void* y, int64_t n, uint32_t bits, hipStream_t s);
// Fused 1x1 expand (+bias, act) -> 3x3 depthwise (+bias, act) (mbconv.hip).
bool expand_dw_eligible(int cin, int H, int W, int S, int pt, int pl, int pb, int pr);
rtenhip_status launch_expand_dw(const float* x, const float* we, const float* be, const float* wd, const float* bd,
                                float* y, int N, int cin, int hidden, int H, int W, int OH, int OW, int S, int pt,
                                int pl, int act_e, float lo_e, float hi_e, int act_d, float lo_d, float hi_d,
                                hipStream_t s);
// Fused 3x3 depthwise (+bias, act) -> 1x1 projection (+bias, residual, act)
// (dw_project.hip): stride 1, pads 1, C = 32, W = 112, M <= 32.
bool dw_project_eligible(int C, int H, int W, int M, int S, int pt, int pl, int pb, int pr);
rtenhip_status launch_dw_project(const float* x, const float* wd, const float* bd, int act_d, float lo_d,
                                 float hi_d, const float* wp, const float* bp, const float* res, int act_p,
                                 float lo_p, float hi_p, float* y, int N, int C, int H, int W, int M,
                                 hipStream_t s);
// MobileNetV2's stem (3 -> 32 channels, 3x3 / 2, pads 1 at the top and left,
// 224 input columns) feeding the depthwise -> projection pair above, as one
// kernel (dw_project.hip): the stem's output never reaches HBM.
bool stem_dw_project_eligible(int C0, int H0, int W0, int kh, int kw, int sh, int sw, int pt, int pl, int O, int OH,
                              int OW);
rtenhip_status launch_stem_dw_project(const float* img, const float* ws, const float* bs, int act_s, float lo_s,
                                      float hi_s, int H0, const float* wd, const float* bd, int act_d, float lo_d,
                                      float hi_d, const float* wp, const float* bp, const float* res, int act_p,
                                      float lo_p, float hi_p, float* y, int N, int H, int M, hipStream_t s);
// A bottleneck's conv3 (1x1, K 64 -> 256, + bias, residual, Relu) and the next
// block's conv1 (1x1, K 256 -> 64, + bias, act) as one launch
// (conv_pair.hip); weights packed [K / 2][2][M] by pack_pair_weights.
bool conv_pair_eligible(int64_t P, int64_t OW, int64_t K3, int64_t M3, int64_t K1, int64_t M1);
rtenhip_status pack_pair_weights(const float* w, int64_t M, int64_t K, float* out, hipStream_t s);
rtenhip_status launch_conv_pair(const float* x, const float* w3p, const float* b3, const float* res, float* y3,
                                const float* w1p, const float* b1, int act1, float* y1, int64_t y1_img,
                                int64_t y1_c, int y1_row, int y1_off, int N, int P, int OW, int M1, hipStream_t s);
// ReduceMean (norm.hip): rows of `len` contiguous elements in slice_sum order,
// or per output element an iter_sum over a strided sub-block (up to 8 kept
// and 8 reduced dims).
rtenhip_status launch_reduce_mean_rows(const float* x, float* y, int64_t rows, int64_t len, hipStream_t s);
struct ReduceDesc {
  int nk, nr;  // kept / reduced dims
  int64_t kshape[RTENHIP_MAX_DIMS], kstride[RTENHIP_MAX_DIMS];
  int64_t rshape[RTENHIP_MAX_DIMS], rstride[RTENHIP_MAX_DIMS];
  int64_t n_out, n_red;
};
rtenhip_status launch_reduce_mean_iter(const float* x, float* y, const ReduceDesc& d, hipStream_t s);
// col2im of ConvTranspose (conv.rs:329-375): col [N, O*kh*kw, H, W] -> y
// [N, O, OH, OW], each output = bias (or 0) + its columns in (ky, kx) order.
rtenhip_status launch_col2im(const float* col, const float* bias, float* y, int64_t N, int64_t O,
                             int64_t OH, int64_t OW, int64_t H, int64_t W, int64_t kh,
                             int64_t kw, int64_t sh, int64_t sw, int64_t pt, int64_t pl,
                             hipStream_t s);

// Fused attention (attention.hip): per (b, h), out = softmax(scale(Q K^T) +
// mask) V with element strides for every operand (unit stride along the head
// dimension of Q, V and out); scale_op 0 none, 1 divide, 2 multiply.
struct AttnDesc {
  int B, H, S, D;
  const float* q;
  int64_t q_b, q_h, q_s;
  const float* k;  // K^T view [B, H, D, S]
  int64_t k_b, k_h, k_d, k_s;
  const float* v;
  int64_t v_b, v_h, v_s;
  const float* mask;  // broadcast view [B, H, S, S] or null
  int64_t m_b, m_h, m_i, m_j;
  float scale;
  int scale_op;
  float* out;
  int64_t o_b, o_h, o_s;
  // Also store the output as the next MatMul's packed A (packed_a.h), the
  // output being row-major [B * S, H * D] (o_s = H * D, o_h = D): null = no.
  float* pk;
  int pk_lbm, pk_lbk, pk_tiles_k;
  int pk_only;  // with pk: skip the row-major store (nothing else reads it)
};
bool attention_fast_ok(const AttnDesc& d);
rtenhip_status launch_attention(const AttnDesc& d, hipStream_t s);
rtenhip_status launch_pad_nchw(const float* x, float* y, int64_t planes, int H, int W, int pt,
                               int pl, int pb, int pr, hipStream_t s);

}  // namespace rtenhip
