/*
 * rten_hip.h — C ABI of the MI355X (gfx950) operator backend for RTen.
 *
 * This is the drop-in boundary: each entry point replaces the CPU body of one
 * RTen `Operator::run` / `run_in_place` (src/ops/mod.rs:821-913) on the f32 hot
 * path, and the graph entry points replace `Model::run` -> `Graph::run`
 * (src/model.rs:580-592, src/graph.rs:733-1073).  A Rust `impl Operator`
 * registered through `OpRegistry::register_op` (src/op_registry.rs:44-49)
 * binds these with `extern "C"`.
 *
 * Conventions
 *  - Plain C types only.  All float pointers are DEVICE pointers (HBM) unless a
 *    function says "host".  The caller owns every buffer.
 *  - Tensors are described by rtenhip_tensor: shape + ELEMENT strides, like
 *    rten-tensor's DynLayout (rten-tensor/src/layout.rs:518-525).
 *  - Every op returns rtenhip_status; codes 1..6 are RTen's OpError variants
 *    (src/ops/mod.rs:666-686) and rtenhip_last_error_message() returns the same
 *    message string the reference returns.  7 = HIP runtime error.
 *  - Work is enqueued on the context's stream (rtenhip_set_stream); calls are
 *    asynchronous and never allocate or synchronize unless stated, so they can
 *    be captured in a hipGraph.
 *  - In-place (y == x) is allowed exactly where the reference's op has
 *    run_in_place (unary ops, Add/Mul/Sub/Div on the larger operand,
 *    BatchNormalization, Softmax).
 */
#ifndef RTEN_HIP_H
#define RTEN_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  RTENHIP_OK = 0,
  RTENHIP_INCORRECT_INPUT_TYPE = 1,      /* OpError::IncorrectInputType */
  RTENHIP_INCORRECT_OUTPUT_TYPE = 2,     /* OpError::IncorrectOutputType */
  RTENHIP_INCOMPATIBLE_INPUT_SHAPES = 3, /* OpError::IncompatibleInputShapes */
  RTENHIP_MISSING_INPUTS = 4,            /* OpError::MissingInputs */
  RTENHIP_INVALID_VALUE = 5,             /* OpError::InvalidValue */
  RTENHIP_UNSUPPORTED_VALUE = 6,         /* OpError::UnsupportedValue */
  RTENHIP_HIP_ERROR = 7,
} rtenhip_status;

#define RTENHIP_MAX_DIMS 8

typedef struct {
  float* data;                       /* device pointer */
  int32_t ndim;
  int64_t shape[RTENHIP_MAX_DIMS];
  int64_t strides[RTENHIP_MAX_DIMS]; /* element strides */
} rtenhip_tensor;

/* int32 tensor view (Input::IntTensor / Output::IntTensor, src/ops/mod.rs:177-180);
 * same layout as rtenhip_tensor. */
typedef struct {
  int32_t* data;                     /* device pointer */
  int32_t ndim;
  int64_t shape[RTENHIP_MAX_DIMS];
  int64_t strides[RTENHIP_MAX_DIMS]; /* element strides */
} rtenhip_tensor_i32;

/* Fused epilogue applied after bias (and residual) by GEMM / Conv. */
typedef enum {
  RTENHIP_ACT_NONE = 0,
  RTENHIP_ACT_RELU = 1, /* Relu: f32::max(x, 0) (unary_elementwise.rs:571) */
  RTENHIP_ACT_CLIP = 2, /* Clip: f32::clamp(x, lo, hi) (unary_elementwise.rs:314-323) */
  RTENHIP_ACT_GELU = 3, /* Gelu: simd_gelu (rten-vecmath/src/erf.rs:85-91) */
} rtenhip_act;

typedef struct rtenhip_ctx rtenhip_ctx;

/* ---- context ----------------------------------------------------------- */
rtenhip_ctx* rtenhip_create(int device);
void rtenhip_destroy(rtenhip_ctx* ctx);
/* Stream used by all subsequent calls on ctx (a hipStream_t; NULL = default). */
rtenhip_status rtenhip_set_stream(rtenhip_ctx* ctx, void* stream);
void* rtenhip_get_stream(rtenhip_ctx* ctx);
/* The stream the context's graphs execute and capture on (Graph::run's
 * executor; by default a non-blocking stream the library creates on the first
 * graph run).  A caller that submits runs from one stream can make it the
 * executor (a non-blocking stream, never the legacy NULL stream: NULL reverts
 * to a library-owned one); runs issued from the executor stream itself skip
 * the two cross-stream events each run otherwise puts between the caller's
 * stream and the executor.  Synchronizes the previous executor first. */
rtenhip_status rtenhip_set_exec_stream(rtenhip_ctx* ctx, void* stream);
const char* rtenhip_last_error_message(void);
/* Status code of the last error on this thread (for entry points that return
 * a handle rather than a status, e.g. rtenhip_model_load). */
int32_t rtenhip_last_error_code(void);
/* Blocks until the context's stream is idle. */
rtenhip_status rtenhip_synchronize(rtenhip_ctx* ctx);
/* Device memory helpers (hipMalloc / hipFree / hipMemcpy H2D, D2H, D2D). */
void* rtenhip_malloc(rtenhip_ctx* ctx, size_t bytes);
void rtenhip_free(rtenhip_ctx* ctx, void* ptr);
rtenhip_status rtenhip_memcpy_h2d(rtenhip_ctx* ctx, void* dst, const void* src, size_t bytes);
rtenhip_status rtenhip_memcpy_d2h(rtenhip_ctx* ctx, void* dst, const void* src, size_t bytes);
/* Kernel library identification: "gfx950" build tag + version. */
const char* rtenhip_build_info(void);
/* Thread count RTen's CPU path runs with, resolved once per context when it is
 * created (rten::threading::thread_pool, src/threading.rs:41-62): the physical
 * core count, or RTEN_NUM_THREADS clamped to [1, logical cores] (a value that
 * does not parse as usize falls back to the physical count).  It changes
 * results only where the reference's blocking depends on it: the gemv column
 * blocks (src/gemm.rs:676), which the M == 1 GEMM path reproduces. */
int32_t rtenhip_num_threads(rtenhip_ctx* ctx);
/* num_cpus 1.16 on Linux (Cargo.lock:268-269): logical = CPUs in the affinity
 * mask capped by a cgroup CPU quota (num_cpus::get); physical = the sum of
 * "cpu cores" over distinct "physical id"s in /proc/cpuinfo, or logical when
 * that finds none (num_cpus::get_physical).  Host only. */
void rtenhip_cpu_counts(int32_t* logical, int32_t* physical);

/* ---- shape helpers ------------------------------------------------------ */
/* calc_output_size_and_padding (src/ops/pooling.rs:27-89).  pad_mode 0 = Fixed
 * pads [top, left, bottom, right], 1 = Same (SAME_UPPER). */
rtenhip_status rtenhip_output_size_and_padding(int64_t in_h, int64_t in_w, int64_t k_h,
                                               int64_t k_w, int64_t stride_h, int64_t stride_w,
                                               int pad_mode, const int64_t pads_in[4],
                                               int64_t dil_h, int64_t dil_w, int64_t out_hw[2],
                                               int64_t pads_out[4]);

/* ---- GEMM engine -------------------------------------------------------- */
/* GemmExecutor::gemm_bias (src/gemm.rs:465-542, gemm_impl 733-930):
 *   out[M,N] = alpha * A[M,K] @ B[K,N] + beta * out  (+ bias[m])
 * A[m,k] at a[m*a_rs + k*a_cs], B[k,n] at b[k*b_rs + n*b_cs], out row stride
 * out_rs.  beta == 0: out is not read.  K is summed in KC=256 blocks exactly as
 * the reference does, so results are bit-identical to RTen's CPU path for
 * alpha == 1 (and any alpha on full 6x16 tiles).  M == 1 with unpacked
 * inputs takes the reference's gemv path (gemm.rs:651-704) and order. */
rtenhip_status rtenhip_gemm_f32(rtenhip_ctx* ctx, int64_t m, int64_t n, int64_t k,
                                const float* a, int64_t a_rs, int64_t a_cs, const float* b,
                                int64_t b_rs, int64_t b_cs, float* out, int64_t out_rs,
                                float alpha, float beta, const float* bias);

/* ---- operators (Operator::run bodies) ----------------------------------- */
/* Conv (src/ops/conv.rs:86-280).  x NCHW or NCW, w OIHW/OIW, bias [O] or NULL.
 * residual (same shape as y) or NULL is added after the bias, then `act`
 * (fusion of the following Add / Relu / Clip nodes; pass NULL/NONE for the
 * plain operator).  y must be preallocated with the output shape
 * (rtenhip_conv_output_shape). */
rtenhip_status rtenhip_conv_output_shape(const rtenhip_tensor* x, const rtenhip_tensor* w,
                                         int pad_mode, const int64_t* pads,
                                         const int64_t* strides, const int64_t* dilations,
                                         int64_t groups, int64_t* out_shape, int32_t* out_ndim);
rtenhip_status rtenhip_conv_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x,
                                const rtenhip_tensor* w, const float* bias, int pad_mode,
                                const int64_t* pads, const int64_t* strides,
                                const int64_t* dilations, int64_t groups, const float* residual,
                                int act, float act_lo, float act_hi, rtenhip_tensor* y);

/* ConvTranspose (src/ops/conv.rs:443-577).  x NCHW or NCW, w [C, O, kh, kw]
 * or [C, O, kw], bias [O] or NULL; pads [top, left, bottom, right] (NCW:
 * [left, right]) or pad_mode 1 = Same; strides [sh, sw] (NCW: [s]).  Errors
 * and the Same-padding offsets follow conv_transpose_output_size_and_padding
 * (conv.rs:382-440) exactly. */
rtenhip_status rtenhip_conv_transpose_output_shape(const rtenhip_tensor* x,
                                                   const rtenhip_tensor* w, int pad_mode,
                                                   const int64_t* pads, const int64_t* strides,
                                                   int64_t* out_shape, int32_t* out_ndim);
rtenhip_status rtenhip_conv_transpose_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x,
                                          const rtenhip_tensor* w, const float* bias,
                                          int pad_mode, const int64_t* pads,
                                          const int64_t* strides, rtenhip_tensor* y);

/* ONNX Gemm (src/ops/matmul.rs:27-81): y = alpha*op(a)@op(b) + beta*c, c
 * broadcast to [M,N] (c may be NULL). */
rtenhip_status rtenhip_gemm_op_f32(rtenhip_ctx* ctx, const rtenhip_tensor* a,
                                   const rtenhip_tensor* b, const rtenhip_tensor* c, float alpha,
                                   float beta, int trans_a, int trans_b, rtenhip_tensor* y);

/* MatMul (src/ops/matmul.rs:123-239): batched + broadcast. */
rtenhip_status rtenhip_matmul_f32(rtenhip_ctx* ctx, const rtenhip_tensor* a,
                                  const rtenhip_tensor* b, rtenhip_tensor* y);

/* MaxPool / AveragePool (src/ops/pooling.rs:104-375), NCHW. */
rtenhip_status rtenhip_max_pool_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x,
                                    const int64_t kernel[2], const int64_t strides[2],
                                    int pad_mode, const int64_t pads[4], rtenhip_tensor* y);
rtenhip_status rtenhip_average_pool_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x,
                                        const int64_t kernel[2], const int64_t strides[2],
                                        int pad_mode, const int64_t pads[4],
                                        int count_include_pad, rtenhip_tensor* y);
/* GlobalAveragePool (src/ops/pooling.rs:294-342). */
rtenhip_status rtenhip_global_average_pool_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x,
                                               rtenhip_tensor* y);

/* BatchNormalization (src/ops/norm.rs:18-128); y may alias x. */
rtenhip_status rtenhip_batch_norm_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x,
                                      const float* scale, const float* bias, const float* mean,
                                      const float* var, float epsilon, rtenhip_tensor* y);

/* LayerNormalization (src/ops/norm.rs:245-299); bias may be NULL. */
rtenhip_status rtenhip_layer_norm_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x,
                                      const rtenhip_tensor* scale, const rtenhip_tensor* bias,
                                      int64_t axis, float epsilon, rtenhip_tensor* y);

/* Softmax (src/ops/norm.rs:332-448 + rten-vecmath softmax.rs); y may alias x. */
rtenhip_status rtenhip_softmax_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x, int64_t axis,
                                   rtenhip_tensor* y);

/* LogSoftmax (src/ops/norm.rs:381-430, log_softmax_in_place); y may alias x.
 * exp / ln are libm's (Rust f32::exp / f32::ln): computed in f64 and rounded. */
rtenhip_status rtenhip_log_softmax_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x, int64_t axis,
                                       rtenhip_tensor* y);

/* InstanceNormalization (src/ops/norm.rs:131-241): x is [N, C, ...]; scale and
 * bias are device arrays of n_channels (must equal C) floats; y may alias x.
 * The reference's default epsilon is 1e-5. */
rtenhip_status rtenhip_instance_norm_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x, const float* scale,
                                         const float* bias, int64_t n_channels, float epsilon,
                                         rtenhip_tensor* y);

/* Unary float ops (src/ops/unary_elementwise.rs; numerics of rten-vecmath). */
typedef enum {
  RTENHIP_UNARY_RELU = 0,
  RTENHIP_UNARY_CLIP = 1, /* p0 = min, p1 = max */
  RTENHIP_UNARY_GELU = 2,
  RTENHIP_UNARY_ERF = 3,
  RTENHIP_UNARY_SIGMOID = 4,
  RTENHIP_UNARY_TANH = 5,
  RTENHIP_UNARY_EXP = 6,
  RTENHIP_UNARY_SILU = 7,
  RTENHIP_UNARY_SQRT = 8, /* Sqrt (unary_elementwise.rs:653): correctly rounded */
} rtenhip_unary_op;
rtenhip_status rtenhip_unary_f32(rtenhip_ctx* ctx, int op, const rtenhip_tensor* x, float p0,
                                 float p1, rtenhip_tensor* y);

/* Broadcasting binary ops (src/ops/binary_elementwise.rs:158-439). */
typedef enum {
  RTENHIP_BINARY_ADD = 0,
  RTENHIP_BINARY_SUB = 1,
  RTENHIP_BINARY_MUL = 2,
  RTENHIP_BINARY_DIV = 3,
  /* Pow (binary_elementwise.rs:742-770): exponent 2 -> x*x, 3 -> x*x*x (the
   * reference's fast paths, bit-exact); any other exponent is computed in
   * double precision and rounded once, within 1 ULP of the libm powf the
   * reference calls (not bit-pinned). */
  RTENHIP_BINARY_POW = 4,
} rtenhip_binary_op;
rtenhip_status rtenhip_binary_f32(rtenhip_ctx* ctx, int op, const rtenhip_tensor* a,
                                  const rtenhip_tensor* b, rtenhip_tensor* y);

/* ReduceMean (src/ops/reduce.rs:225-400): mean over `axes` (n_axes == 0: all
 * axes) of a contiguous f32 tensor, in the reference's summation order: the
 * 8-wide slice_sum for a reduction over the last axis, the 4-wide iter_sum
 * otherwise (slice_reductions.rs:38-85), divided by the element count.  y has
 * the reduced shape (keep_dims: reduced axes kept as 1).  Errors "Axis is
 * invalid", "Cannot reduce empty tensor". */
rtenhip_status rtenhip_reduce_mean_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x, const int32_t* axes,
                                       int32_t n_axes, int keep_dims, rtenhip_tensor* y);

/* ---- graph executor (Graph::run, src/graph.rs:733-1073) ------------------ */
typedef struct rtenhip_graph rtenhip_graph;

rtenhip_graph* rtenhip_graph_create(rtenhip_ctx* ctx);
void rtenhip_graph_destroy(rtenhip_graph* g);
/* Node ids are returned (>= 0) or -1 on error. */
int32_t rtenhip_graph_add_value(rtenhip_graph* g, const char* name);
/* Constant f32 tensor from HOST data (uploaded once, like a .rten constant). */
int32_t rtenhip_graph_add_constant(rtenhip_graph* g, const char* name, const float* host_data,
                                   const int64_t* shape, int32_t ndim);
/* Operator node.  op_type is the sg::OperatorType name (schema.fbs:12-121),
 * attrs a "key=v1,v2;key=v" string (e.g. "pads=3,3,3,3;strides=2,2;groups=1").
 * Input id -1 = absent optional input. */
int32_t rtenhip_graph_add_op(rtenhip_graph* g, const char* name, const char* op_type,
                             const char* attrs, const int32_t* inputs, int32_t n_inputs,
                             const int32_t* outputs, int32_t n_outputs);
/* Declare the model's input / output value ids (Model::input_ids /
 * output_ids, src/model.rs:616-632); outputs are never fused away. */
rtenhip_status rtenhip_graph_set_io(rtenhip_graph* g, const int32_t* input_ids, int32_t n_inputs,
                                    const int32_t* output_ids, int32_t n_outputs);
/* Load-time optimisation: fuse Conv+Add+Relu/Clip epilogues and fold
 * Flatten/Reshape (metadata).  Numerics are unchanged (bit-identical). */
rtenhip_status rtenhip_graph_optimize(rtenhip_graph* g);
/* Plan + run.  Inputs are device tensors; outputs are written into
 * caller-provided device tensors whose shapes the executor checks.  The plan
 * is cached per (inputs, outputs) like get_cached_plan (graph.rs:768-795). */
rtenhip_status rtenhip_graph_run(rtenhip_graph* g, const int32_t* input_ids,
                                 const rtenhip_tensor* inputs, int32_t n_inputs,
                                 const int32_t* output_ids, rtenhip_tensor* outputs,
                                 int32_t n_outputs);
/* Plan (or fetch the cached plan) and report the output shapes without
 * running: shapes[i*RTENHIP_MAX_DIMS + d], ndims[i]. */
rtenhip_status rtenhip_graph_plan(rtenhip_graph* g, const int32_t* input_ids,
                                  const rtenhip_tensor* inputs, int32_t n_inputs,
                                  const int32_t* output_ids, int32_t n_outputs, int64_t* shapes,
                                  int32_t* ndims);
/* Element types of graph values, in sg::DataType / ConstantDataType order
 * (schema.fbs:136-139, 475-478): Input::IntTensor / FloatTensor
 * (src/ops/mod.rs:177-180).  Int32 values use the same descriptor
 * (rtenhip_tensor, 4-byte elements). */
typedef enum {
  RTENHIP_DTYPE_INT32 = 0,
  RTENHIP_DTYPE_FLOAT32 = 1,
} rtenhip_dtype;
/* Constant int32 tensor from HOST data (a .rten IntData / Int32 constant). */
int32_t rtenhip_graph_add_constant_i32(rtenhip_graph* g, const char* name, const int32_t* host_data,
                                       const int64_t* shape, int32_t ndim);
/* rtenhip_graph_run / _plan with each input's element type (input_dtypes[i],
 * NULL = all float32); the plan infers every value's type (Cast, Gather,
 * Where, shape ops carry int32; the f32 kernels reject int32 inputs with
 * RTENHIP_INCORRECT_INPUT_TYPE).  output_dtypes (may be NULL) receives the
 * outputs' types.  A plan with a Gather on non-constant indices checks its
 * indices on the device (gather.rs:52-60): by default the run waits for that
 * check and returns an out-of-range index ("Entry in `indices` is out of
 * range", INVALID_VALUE) itself, as Model::run does.  With
 * rtenhip_graph_set_deferred_checks(g, 1) the run is queued without a host
 * round trip and the error is reported by rtenhip_graph_synchronize only. */
rtenhip_status rtenhip_graph_run_typed(rtenhip_graph* g, const int32_t* input_ids,
                                       const rtenhip_tensor* inputs, const int32_t* input_dtypes,
                                       int32_t n_inputs, const int32_t* output_ids,
                                       rtenhip_tensor* outputs, int32_t n_outputs);
rtenhip_status rtenhip_graph_plan_typed(rtenhip_graph* g, const int32_t* input_ids,
                                        const rtenhip_tensor* inputs, const int32_t* input_dtypes,
                                        int32_t n_inputs, const int32_t* output_ids,
                                        int32_t n_outputs, int64_t* shapes, int32_t* ndims,
                                        int32_t* output_dtypes);
/* Wait for every queued run of the graph and report the deferred Gather index
 * error of the earliest run that had one (see rtenhip_graph_run_typed); the
 * error is cleared once reported.  Stands in for the point where RTen's
 * synchronous Model::run returns (src/model.rs:580-592). */
rtenhip_status rtenhip_graph_synchronize(rtenhip_graph* g);
/* enabled = 1: Gather index checks of later runs are deferred to
 * rtenhip_graph_synchronize (runs queue back to back); 0 (default): every run
 * returns its own index error (gather.rs:52-60).  No counterpart in RTen, whose
 * Model::run is synchronous. */
rtenhip_status rtenhip_graph_set_deferred_checks(rtenhip_graph* g, int enabled);
/* Output shape of a value after the last run (or -1). */
int32_t rtenhip_graph_value_shape(rtenhip_graph* g, int32_t id, int64_t* shape);
/* Per-op timing table like RTEN_TIMING (graph.rs:1039-1055), when enabled. */
rtenhip_status rtenhip_graph_set_timing(rtenhip_graph* g, int enabled);
const char* rtenhip_graph_timing_report(rtenhip_graph* g);

/* .rten V2 model loader (src/model.rs:265-522): parses the file bytes (host),
 * uploads constants, builds the graph.  Returns NULL on error. */
rtenhip_graph* rtenhip_model_load(rtenhip_ctx* ctx, const uint8_t* bytes, size_t len);
/* Model::load with ModelOptions::with_optimize (src/model.rs:156-162, 190-199):
 * optimize = 0 keeps the graph as stored (no load-time fusion). */
rtenhip_graph* rtenhip_model_load_with_options(rtenhip_ctx* ctx, const uint8_t* bytes, size_t len,
                                               int optimize);
/* Parse a .rten file on the host only (no device) and return a text listing of
 * its nodes (index, kind, name, op type, decoded attributes, constant shape and
 * checksum), or NULL with the load error in rtenhip_last_error_message().
 * Errors use the reference's ModelLoadError texts (model.rs:677-689). */
const char* rtenhip_model_describe(const uint8_t* bytes, size_t len);
int32_t rtenhip_model_input_ids(rtenhip_graph* g, int32_t* ids, int32_t cap);
int32_t rtenhip_model_output_ids(rtenhip_graph* g, int32_t* ids, int32_t cap);
int32_t rtenhip_graph_node_id(rtenhip_graph* g, const char* name);
/* The graph as it stands (after rtenhip_graph_optimize): one line per node,
 * tab-separated -- "id\top\tname\tOperatorName\tin,ids\tout,ids" for each
 * operator still in the graph, with RTen's Operator::name() after its fusions
 * (optimize.rs:286-518: "Gelu", "LayerNormalization", "Silu",
 * "FusedTranspose(MatMul)"; device fusions as "FusedAttention" or the base
 * operator), "id\tconst\tname\tdims" (dims "AxB...", after constant
 * propagation too) and "id\tvalue\tname".  Host only. */
const char* rtenhip_graph_describe(rtenhip_graph* g);

/* ---- Index / select / convert (BERT embedding and mask path) ---- */

/* Gather (src/ops/gather.rs:21-76): y = x taken along `axis` at `indices`
 * (negative entries count from the end); y has shape x[:axis] + indices +
 * x[axis+1:].  Errors: "Axis is invalid", "Entry in `indices` is out of range".
 * The index check runs on the device, so rtenhip_gather_f32 synchronizes the
 * context's stream to report it. */
rtenhip_status rtenhip_gather_output_shape(const rtenhip_tensor* x,
                                           const rtenhip_tensor_i32* indices, int64_t axis,
                                           int64_t* out_shape, int32_t* out_ndim);
rtenhip_status rtenhip_gather_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x,
                                  const rtenhip_tensor_i32* indices, int64_t axis,
                                  rtenhip_tensor* y);
/* Where (src/ops/binary_elementwise.rs:850-929): out = cond != 0 ? x : y, all
 * three broadcast to one shape ("Cannot broadcast inputs"). */
rtenhip_status rtenhip_where_output_shape(const rtenhip_tensor_i32* cond, const rtenhip_tensor* x,
                                          const rtenhip_tensor* y, int64_t* out_shape,
                                          int32_t* out_ndim);
rtenhip_status rtenhip_where_f32(rtenhip_ctx* ctx, const rtenhip_tensor_i32* cond,
                                 const rtenhip_tensor* x, const rtenhip_tensor* y,
                                 rtenhip_tensor* out);
/* Cast (src/ops/convert.rs:6-17): f32 -> i32 as Rust `as` (truncation toward
 * zero, saturating, NaN -> 0); i32 -> f32 rounded to nearest even.  y has x's
 * shape and is contiguous. */
rtenhip_status rtenhip_cast_f32_to_i32(rtenhip_ctx* ctx, const rtenhip_tensor* x,
                                       rtenhip_tensor_i32* y);
rtenhip_status rtenhip_cast_i32_to_f32(rtenhip_ctx* ctx, const rtenhip_tensor_i32* x,
                                       rtenhip_tensor* y);

/* ---- host-resident runs (Model::run with host tensors) -------------------
 * RTen's Model::run takes and returns host tensors (src/model.rs:580-592) and
 * rten-cli times that call in a loop (rten-cli/src/main.rs:296-317).  These
 * entry points give a host caller the same surface without paying the PCIe
 * copies on top of every forward. */
/* Page-locked (pinned) host memory, the form the upload DMA reads directly
 * (hipHostMalloc).  Pageable memory works with rtenhip_graph_run_host too,
 * but its copies are staged and do not overlap the forward. */
void* rtenhip_host_alloc(rtenhip_ctx* ctx, size_t bytes);
void rtenhip_host_free(rtenhip_ctx* ctx, void* ptr);
/* Queue one Model::run over HOST tensors and return without waiting:
 * inputs[i].data / outputs[j].data are host pointers (contiguous; shapes and
 * element types as for rtenhip_graph_run_typed, input_dtypes NULL = all
 * float32).  Inside the library: the inputs are uploaded on a high-priority
 * copy stream into one of two device slots while the previous run computes;
 * the forward (hipGraph replay after the plan's first run) waits only for its
 * slot's upload; its outputs are downloaded behind the next run's upload.
 * The host buffers must stay untouched until the run is waited for.  *run_id
 * (may be NULL) receives the run's id for rtenhip_graph_wait.  Gather index
 * errors (gather.rs:52-60) of host runs are reported by rtenhip_graph_wait. */
rtenhip_status rtenhip_graph_run_host(rtenhip_graph* g, const int32_t* input_ids, const rtenhip_tensor* inputs,
                                      const int32_t* input_dtypes, int32_t n_inputs, const int32_t* output_ids,
                                      rtenhip_tensor* outputs, int32_t n_outputs, uint64_t* run_id);
/* Block until host run `run_id` has its outputs on the host (and every
 * earlier run too); run_id 0 waits for every queued run of the graph.  The
 * point where RTen's synchronous Model::run returns (src/model.rs:580-592). */
rtenhip_status rtenhip_graph_wait(rtenhip_graph* g, uint64_t run_id);

/* ---- batch-sharded runs over several GPUs ----------------
 * One replica of a .rten model (rtenhip_model_load_with_options) per device,
 * the batch split into contiguous slices (earlier shards take the remainder),
 * and one exchange: an RCCL all-gather of the per-shard outputs over xGMI
 * when the devices are distinct (RTENHIP_SHARDED_RCCL=0 disables it), else
 * device-to-host copies of each shard.  Batch items are independent
 * (src/ops/conv.rs:243-270), so each image's output is the reference's bits
 * for the shard its device ran (a one-image shard's FC takes RTen's gemv
 * order, gemm.rs:651-704).  Models with one input and one output. */
typedef struct rtenhip_sharded rtenhip_sharded;
rtenhip_sharded* rtenhip_sharded_create(const uint8_t* model_bytes, size_t len, const int32_t* devices,
                                        int32_t n_devices, int optimize);
void rtenhip_sharded_destroy(rtenhip_sharded* s);
/* 1 when the outputs are all-gathered with RCCL, 0 for host copies. */
int32_t rtenhip_sharded_gather_mode(rtenhip_sharded* s);
/* The replica of shard i (for its timing report / tuning knobs), or NULL. */
rtenhip_graph* rtenhip_sharded_graph(rtenhip_sharded* s, int32_t shard);
/* Model::run over a HOST batch: input [B, ...] -> output [B, ...], both host
 * buffers; returns when the output is on the host. */
rtenhip_status rtenhip_sharded_run_host(rtenhip_sharded* s, const rtenhip_tensor* input, rtenhip_tensor* output);
/* RCCL mode: the gathered outputs of the last run on shard i's device
 * ([n_shards][rows][...] with rows = ceil(B / n_shards), short shards
 * zero-padded), for a device-resident consumer; NULL otherwise. */
const float* rtenhip_sharded_gathered(rtenhip_sharded* s, int32_t shard);

#ifdef __cplusplus
}
#endif

#endif /* RTEN_HIP_H */
