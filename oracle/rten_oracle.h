/*
 * rten_oracle.h — CPU restatement of RTen's f32 operator hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker and the timed
 * CPU baseline ("port" of RTen's own algorithm).  Only tests/, the smoke()
 * entry point and bench.py's cpu_baseline leg may load it; the product path
 * (librten_hip.so) never links or calls it.
 *
 * Every function restates the reference implementation cited next to it,
 * including its summation order, so that the GPU kernels can be checked
 * bit-for-bit where the reference's order is reproducible:
 *   - GEMM: K is split in KC=256 blocks; each block is an fma chain started
 *     from +0 (FmaKernel 6x16 micro-kernel), blocks are summed in order and
 *     the bias is added after the first block (src/gemm.rs:733-1050,
 *     src/gemm/kernels.rs:206-316).
 *   - elementwise ops use separate mul/add roundings unless the reference
 *     calls mul_add (the whole library is built with -ffp-contract=off).
 *
 * All tensors are host pointers in row-major (contiguous) layout unless a
 * stride argument says otherwise.  Shapes are int64.
 */
#ifndef RTEN_ORACLE_H
#define RTEN_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes: mirror OpError (src/ops/mod.rs:666-686). */
enum {
  ORC_OK = 0,
  ORC_INCORRECT_INPUT_TYPE = 1,
  ORC_INCORRECT_OUTPUT_TYPE = 2,
  ORC_INCOMPATIBLE_INPUT_SHAPES = 3,
  ORC_MISSING_INPUTS = 4,
  ORC_INVALID_VALUE = 5,
  ORC_UNSUPPORTED_VALUE = 6,
};

const char* orc_last_error(void);

/* Thread pool: physical cores unless RTEN_NUM_THREADS is set
 * (src/threading.rs:41-62). */
int orc_num_threads(void);
void orc_set_num_threads(int n);
/* Re-resolve the thread count from RTEN_NUM_THREADS (src/threading.rs:41-62). */
int orc_reset_threads(void);
/* num_cpus::get / get_physical (num_cpus 1.16, Linux). */
void orc_cpu_counts(int* logical, int* physical);

/* XorShiftRng (rten-tensor/src/rng.rs:6-35): fill `out` with next_f32(). */
void orc_xorshift_fill(uint64_t* state, float* out, int64_t n);

/* GemmExecutor::gemm_bias / gemm_uninit_bias (src/gemm.rs:465-542) over
 * strided A [M,K] and B [K,N]; `out` is row-major with row stride out_rs.
 * beta==0 means out is not read.  bias may be NULL (length M). */
int orc_gemm(float* out, int64_t out_rs, const float* a, int64_t a_rs, int64_t a_cs,
             const float* b, int64_t b_rs, int64_t b_cs, int64_t m, int64_t n, int64_t k,
             float alpha, float beta, const float* bias);

/* ONNX Gemm op: gemm_op (src/ops/matmul.rs:27-81).  c may be NULL; c_shape
 * has c_ndim (0..2) dims and is broadcast to [M,N]. */
int orc_gemm_op(const float* a, const int64_t a_shape[2], const float* b, const int64_t b_shape[2],
                const float* c, const int64_t* c_shape, int c_ndim, float alpha, float beta,
                int trans_a, int trans_b, float* out);

/* MatMul op: matmul_impl (src/ops/matmul.rs:123-239).  Writes out_shape. */
int orc_matmul(const float* a, const int64_t* a_shape, int a_ndim, const float* b,
               const int64_t* b_shape, int b_ndim, float* out, int64_t* out_shape, int* out_ndim);

/* calc_output_size_and_padding (src/ops/pooling.rs:27-89).  pad_mode 0 =
 * Fixed(pads), 1 = Same.  Writes out_hw[2] and fixed pads[4]. */
int orc_output_size_and_padding(int64_t in_h, int64_t in_w, int64_t k_h, int64_t k_w,
                                int64_t stride_h, int64_t stride_w, int pad_mode,
                                const int64_t pads_in[4], int64_t dil_h, int64_t dil_w,
                                int64_t out_hw[2], int64_t pads_out[4]);

/* Conv op: conv (src/ops/conv.rs:86-280).  x is NCHW (or NCW when x_ndim==3),
 * w is OIHW.  pads as [top,left,bottom,right] (pad_mode 0) or SAME_UPPER
 * (pad_mode 1).  Writes out_shape (4 or 3 dims). */
int orc_conv(const float* x, const int64_t* x_shape, int x_ndim, const float* w,
             const int64_t* w_shape, const float* bias, int pad_mode, const int64_t* pads,
             const int64_t* strides, const int64_t* dilations, int64_t groups, float* out,
             int64_t* out_shape);

/* ConvTranspose: conv_transpose (src/ops/conv.rs:443-535) with col2im
 * (329-375).  x NCHW (or NCW), w [C, O, kh, kw]; pads [top,left,bottom,right]
 * (or [left,right] for 1-D), pad_mode 1 = Same.  Output size and the
 * reference's padding order: conv_transpose_output_size_and_padding (382-440). */
int orc_conv_transpose_output_size(int64_t in_h, int64_t in_w, int64_t k_h, int64_t k_w,
                                   int pad_mode, const int64_t* pads_in, int64_t stride_h,
                                   int64_t stride_w, int64_t out_hw[2], int64_t pads_out[4]);
int orc_conv_transpose(const float* x, const int64_t* x_shape, int x_ndim, const float* w,
                       const int64_t* w_shape, const float* bias, int pad_mode,
                       const int64_t* pads, const int64_t* strides, float* out,
                       int64_t* out_shape);

/* MaxPool / AveragePool (src/ops/pooling.rs:104-375), NCHW. */
int orc_max_pool(const float* x, const int64_t x_shape[4], const int64_t kernel[2],
                 const int64_t strides[2], int pad_mode, const int64_t pads[4], float* out,
                 int64_t out_shape[4]);
int orc_average_pool(const float* x, const int64_t x_shape[4], const int64_t kernel[2],
                     const int64_t strides[2], int pad_mode, const int64_t pads[4],
                     int count_include_pad, float* out, int64_t out_shape[4]);
/* global_average_pool (src/ops/pooling.rs:294-342). */
int orc_global_average_pool(const float* x, const int64_t x_shape[4], float* out);

/* batch_norm (src/ops/norm.rs:18-54). */
int orc_batch_norm(const float* x, const int64_t* shape, int ndim, const float* scale,
                   const float* bias, const float* mean, const float* var, float epsilon,
                   float* out);

/* Broadcasting binary ops (src/ops/binary_elementwise.rs:158-256).
 * op: 0 Add, 1 Sub, 2 Mul, 3 Div. */
int orc_binary(int op, const float* a, const int64_t* a_shape, int a_ndim, const float* b,
               const int64_t* b_shape, int b_ndim, float* out, int64_t* out_shape, int* out_ndim);

/* Unary float ops (src/ops/unary_elementwise.rs). */
enum {
  ORC_RELU = 0,
  ORC_CLIP = 1,
  ORC_GELU = 2,
  ORC_ERF = 3,
  ORC_SIGMOID = 4,
  ORC_TANH = 5,
  ORC_EXP = 6,
  ORC_SILU = 7,
};
int orc_unary(int op, const float* x, int64_t n, float* out, float p0, float p1);

/* Softmax over `axis` (src/ops/norm.rs:332-448, rten-vecmath softmax.rs). */
int orc_softmax(const float* x, const int64_t* shape, int ndim, int64_t axis, float* out);
/* LogSoftmax over `axis` (src/ops/norm.rs:381-430; libm expf / logf). */
int orc_log_softmax(const float* x, const int64_t* shape, int ndim, int64_t axis, float* out);
/* InstanceNormalization (src/ops/norm.rs:131-241). */
int orc_instance_norm(const float* x, const int64_t* shape, int ndim, const float* scale, int64_t n_scale,
                      const float* bias, int64_t n_bias, float epsilon, float* out);

/* LayerNormalization (src/ops/norm.rs:245-299) for scale/bias of the
 * normalized shape (same trailing dims). bias may be NULL. */
int orc_layer_norm(const float* x, const int64_t* shape, int ndim, const float* scale,
                   const float* bias, int64_t axis, float epsilon, float* out);

/* Naive triple-loop / 7-loop oracles used by the reference's tests
 * (src/gemm.rs:1126-1147, src/ops/conv.rs:599-673).  Double accumulation
 * is NOT used: they restate the reference's f32 loops. */
void orc_reference_gemm(float* out, const float* a, const float* b, int64_t m, int64_t n,
                        int64_t k, float alpha, float beta, const float* bias);

#ifdef __cplusplus
}
#endif

#endif
