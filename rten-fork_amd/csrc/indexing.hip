// Index / select / convert operators on int32 and f32 tensors (the BERT
// embedding and attention-mask path):
//  - Gather (src/ops/gather.rs:21-76): y = x taken along `axis` at `indices`,
//    negative indices counting from the end;
//  - Where (src/ops/binary_elementwise.rs:850-929): out = cond != 0 ? x : y
//    with three-way broadcasting;
//  - Cast (src/ops/convert.rs:6-17): f32 -> i32 as Rust `as` (truncation
//    toward zero, saturating, NaN -> 0), i32 -> f32 rounded to nearest even.
// Pure data movement, so results are exact.  One thread per output element;
// per-dimension strides map the output index to each operand (0 = broadcast).
#include <climits>

#include "common.h"
#include "ctx.h"

namespace rtenhip {

constexpr int IX_DIMS = 2 * RTENHIP_MAX_DIMS;
struct IdxDesc {
  int ndim;
  int64_t shape[IX_DIMS];
  int64_t s0[IX_DIMS], s1[IX_DIMS], s2[IX_DIMS];
};

__device__ __forceinline__ void ix_offsets(const IdxDesc& d, int64_t i, int64_t& o0, int64_t& o1,
                                           int64_t& o2) {
  o0 = o1 = o2 = 0;
  for (int k = d.ndim - 1; k >= 0; k--) {
    const int64_t c = i % d.shape[k];
    i /= d.shape[k];
    o0 += c * d.s0[k];
    o1 += c * d.s1[k];
    o2 += c * d.s2[k];
  }
}

__global__ void gather_kernel(const float* __restrict__ x, const int32_t* __restrict__ idx,
                              float* __restrict__ y, int64_t n, IdxDesc d, int64_t axis_len,
                              int64_t axis_stride, int* __restrict__ bad) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t xo, io, unused;
    ix_offsets(d, i, xo, io, unused);
    int64_t j = idx[io];
    if (j < 0) j += axis_len;
    float v = 0.f;
    if (j < 0 || j >= axis_len)
      atomicOr(bad, 1);
    else
      v = x[xo + j * axis_stride];
    y[i] = v;
  }
}

// Row gather (axis 0 of a contiguous [V, D] table, D % 4 == 0, contiguous
// indices and output): one wave per index copies its row as float4s -- the
// embedding lookups of BERT.  Same values and the same out-of-range flag as
// gather_kernel (an out-of-range row is zero-filled).
__global__ __launch_bounds__(256) void gather_rows_kernel(const float* __restrict__ x, const int32_t* __restrict__ idx,
                                                          float* __restrict__ y, int64_t rows, int64_t V, int D4,
                                                          int* __restrict__ bad) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int lane = threadIdx.x & 63;
  int64_t j = idx[r];
  if (j < 0) j += V;
  const bool ok = j >= 0 && j < V;
  if (!ok && lane == 0) atomicOr(bad, 1);
  const float4* src = reinterpret_cast<const float4*>(x) + (ok ? j : 0) * D4;
  float4* dst = reinterpret_cast<float4*>(y) + r * D4;
  for (int c = lane; c < D4; c += 64) dst[c] = ok ? src[c] : make_float4(0.f, 0.f, 0.f, 0.f);
}

__global__ void where_kernel(const int32_t* __restrict__ c, const float* __restrict__ x,
                             const float* __restrict__ y, float* __restrict__ out, int64_t n,
                             IdxDesc d) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t co, xo, yo;
    ix_offsets(d, i, co, xo, yo);
    out[i] = c[co] != 0 ? x[xo] : y[yo];
  }
}

__global__ void cast_f2i_kernel(const float* __restrict__ x, int32_t* __restrict__ y, int64_t n,
                                IdxDesc d) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t xo, a, b;
    ix_offsets(d, i, xo, a, b);
    const float v = x[xo];
    y[i] = v != v ? 0
                  : v >= 2147483648.f ? INT_MAX : v <= -2147483648.f ? INT_MIN : (int32_t)v;
  }
}

__global__ void cast_i2f_kernel(const int32_t* __restrict__ x, float* __restrict__ y, int64_t n,
                                IdxDesc d) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t xo, a, b;
    ix_offsets(d, i, xo, a, b);
    y[i] = __int2float_rn(x[xo]);
  }
}

static dim3 ix_grid(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b > 65536) b = 65536;
  return dim3((unsigned)(b < 1 ? 1 : b));
}

static const rtenhip_tensor* as_f(const rtenhip_tensor_i32* t) {
  return reinterpret_cast<const rtenhip_tensor*>(t);  // identical layout
}

// Gather geometry: output dims x[:ax] + indices + x[ax+1:]; s0 = x strides,
// s1 = index strides.
static rtenhip_status gather_plan(const rtenhip_tensor* x, const rtenhip_tensor_i32* idx,
                                  int64_t axis, IdxDesc& d, int64_t& ax) {
  if (!x || !idx) return fail(RTENHIP_INVALID_VALUE, "null argument");
  if (axis < -(int64_t)x->ndim || axis >= (int64_t)x->ndim)
    return fail(RTENHIP_INVALID_VALUE, "Axis is invalid");
  ax = axis < 0 ? axis + x->ndim : axis;
  const int nd = x->ndim - 1 + idx->ndim;
  if (nd > RTENHIP_MAX_DIMS) return fail(RTENHIP_UNSUPPORTED_VALUE, "Gather output has too many dims");
  d = IdxDesc{};
  d.ndim = nd;
  int k = 0;
  for (int i = 0; i < ax; i++, k++) {
    d.shape[k] = x->shape[i];
    d.s0[k] = x->strides[i];
  }
  for (int i = 0; i < idx->ndim; i++, k++) {
    d.shape[k] = idx->shape[i];
    d.s1[k] = idx->strides[i];
  }
  for (int i = (int)ax + 1; i < x->ndim; i++, k++) {
    d.shape[k] = x->shape[i];
    d.s0[k] = x->strides[i];
  }
  return RTENHIP_OK;
}

static bool ix_bcast(const int64_t* a, int na, const int64_t* b, int nb, int64_t* out, int* no) {
  const int n = na > nb ? na : nb;
  for (int i = 0; i < n; i++) {
    const int ia = i - (n - na), ib = i - (n - nb);
    const int64_t da = ia >= 0 ? a[ia] : 1, db = ib >= 0 ? b[ib] : 1;
    if (da != db && da != 1 && db != 1) return false;
    out[i] = da == 1 ? db : da;
  }
  *no = n;
  return true;
}

// Stride of operand t along output dim k of an nd-dim broadcast shape.
static int64_t ix_bstride(const rtenhip_tensor* t, int nd, int k) {
  const int i = k - (nd - t->ndim);
  return (i < 0 || t->shape[i] == 1) ? 0 : t->strides[i];
}

static rtenhip_status where_shape(const rtenhip_tensor_i32* c, const rtenhip_tensor* x,
                                  const rtenhip_tensor* y, int64_t* shape, int* nd) {
  if (!c || !x || !y) return fail(RTENHIP_INVALID_VALUE, "null argument");
  int64_t xy[RTENHIP_MAX_DIMS];
  int nxy;
  if (!ix_bcast(x->shape, x->ndim, y->shape, y->ndim, xy, &nxy) ||
      !ix_bcast(c->shape, c->ndim, xy, nxy, shape, nd))
    return fail(RTENHIP_INCOMPATIBLE_INPUT_SHAPES, "Cannot broadcast inputs");
  return RTENHIP_OK;
}

static bool out_matches(const rtenhip_tensor* y, const int64_t* shape, int nd) {
  if (!y || y->ndim != nd || !is_contiguous(*y)) return false;
  for (int i = 0; i < nd; i++)
    if (y->shape[i] != shape[i]) return false;
  return true;
}

// Gather for the graph executor: out-of-range indices are recorded in *flag
// (device int, zeroed by the caller) instead of synchronizing, so the launch
// can be captured in a hipGraph; the run checks the flag when it completes.
rtenhip_status launch_gather(const rtenhip_tensor* x, const rtenhip_tensor_i32* indices, int64_t axis,
                             rtenhip_tensor* y, int* flag, hipStream_t s) {
  IdxDesc d;
  int64_t ax;
  rtenhip_status st = gather_plan(x, indices, axis, d, ax);
  if (st) return st;
  if (!out_matches(y, d.shape, d.ndim))
    return fail(RTENHIP_INCOMPATIBLE_INPUT_SHAPES, "Output tensor has the wrong shape");
  const int64_t n = numel(*y);
  if (n == 0) return RTENHIP_OK;
  if (ax == 0 && x->ndim == 2 && is_contiguous(*x) && x->shape[1] % 4 == 0 && x->shape[1] / 4 < (1 << 30) &&
      is_contiguous(*reinterpret_cast<const rtenhip_tensor*>(indices)) && ((uintptr_t)x->data % 16) == 0 &&
      ((uintptr_t)y->data % 16) == 0) {
    const int64_t rows = n / x->shape[1];
    hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, x->data,
                       indices->data, y->data, rows, x->shape[0], (int)(x->shape[1] / 4), flag);
    RTENHIP_LAUNCH_CHECK();
    return RTENHIP_OK;
  }
  hipLaunchKernelGGL(gather_kernel, ix_grid(n), dim3(256), 0, s, x->data, indices->data, y->data, n,
                     d, x->shape[ax], x->strides[ax], flag);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

// The end of a run's Gather check (graph executor): the run's flag goes to
// word seq % nslots of a fine-grained (host-mapped) ring, the flag is
// cleared and seq advances -- one launch that a hipGraph capture holds, where
// a device-to-host copy and a fill after the replay each cost a dispatch and
// an inter-launch gap.
__global__ void gather_check_finish_kernel(int* flag, unsigned* seq, int* ring, int nslots) {
  if (threadIdx.x != 0) return;
  const unsigned q = *seq;
  ring[q % (unsigned)nslots] = *flag;
  __threadfence_system();
  *flag = 0;
  *seq = q + 1;
}

rtenhip_status launch_gather_check_finish(int* flag, unsigned* seq, int* ring, int nslots, hipStream_t s) {
  if (!flag || !seq || !ring || nslots <= 0) return fail(RTENHIP_INVALID_VALUE, "gather check ring");
  hipLaunchKernelGGL(gather_check_finish_kernel, dim3(1), dim3(64), 0, s, flag, seq, ring, nslots);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

}  // namespace rtenhip

using namespace rtenhip;

extern "C" rtenhip_status rtenhip_gather_output_shape(const rtenhip_tensor* x,
                                                      const rtenhip_tensor_i32* indices,
                                                      int64_t axis, int64_t* out_shape,
                                                      int32_t* out_ndim) {
  IdxDesc d;
  int64_t ax;
  rtenhip_status st = gather_plan(x, indices, axis, d, ax);
  if (st) return st;
  for (int i = 0; i < d.ndim; i++) out_shape[i] = d.shape[i];
  *out_ndim = d.ndim;
  return RTENHIP_OK;
}

extern "C" rtenhip_status rtenhip_gather_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x,
                                             const rtenhip_tensor_i32* indices, int64_t axis,
                                             rtenhip_tensor* y) {
  IdxDesc d;
  int64_t ax;
  rtenhip_status st = gather_plan(x, indices, axis, d, ax);
  if (st) return st;
  if (!out_matches(y, d.shape, d.ndim))
    return fail(RTENHIP_INCOMPATIBLE_INPUT_SHAPES, "Output tensor has the wrong shape");
  const int64_t n = numel(*y);
  if (n == 0) return RTENHIP_OK;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  int* flag = reinterpret_cast<int*>(c->scratch_floats(1, 0));
  if (!flag) return fail(RTENHIP_HIP_ERROR, "scratch allocation failed");
  RTENHIP_HIP_CHECK(hipMemsetAsync(flag, 0, sizeof(int), c->stream));
  hipLaunchKernelGGL(gather_kernel, ix_grid(n), dim3(256), 0, c->stream, x->data, indices->data,
                     y->data, n, d, x->shape[ax], x->strides[ax], flag);
  RTENHIP_LAUNCH_CHECK();
  int bad = 0;
  RTENHIP_HIP_CHECK(hipMemcpyAsync(&bad, flag, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  RTENHIP_HIP_CHECK(hipStreamSynchronize(c->stream));
  if (bad) return fail(RTENHIP_INVALID_VALUE, "Entry in `indices` is out of range");
  return RTENHIP_OK;
}

extern "C" rtenhip_status rtenhip_where_output_shape(const rtenhip_tensor_i32* cond,
                                                     const rtenhip_tensor* x,
                                                     const rtenhip_tensor* y, int64_t* out_shape,
                                                     int32_t* out_ndim) {
  int nd = 0;
  rtenhip_status st = where_shape(cond, x, y, out_shape, &nd);
  if (st) return st;
  *out_ndim = nd;
  return RTENHIP_OK;
}

extern "C" rtenhip_status rtenhip_where_f32(rtenhip_ctx* ctx, const rtenhip_tensor_i32* cond,
                                            const rtenhip_tensor* x, const rtenhip_tensor* y,
                                            rtenhip_tensor* out) {
  int64_t shape[RTENHIP_MAX_DIMS];
  int nd = 0;
  rtenhip_status st = where_shape(cond, x, y, shape, &nd);
  if (st) return st;
  if (!out_matches(out, shape, nd))
    return fail(RTENHIP_INCOMPATIBLE_INPUT_SHAPES, "Output tensor has the wrong shape");
  const int64_t n = numel(*out);
  if (n == 0) return RTENHIP_OK;
  IdxDesc d{};
  d.ndim = nd;
  for (int k = 0; k < nd; k++) {
    d.shape[k] = shape[k];
    d.s0[k] = ix_bstride(as_f(cond), nd, k);
    d.s1[k] = ix_bstride(x, nd, k);
    d.s2[k] = ix_bstride(y, nd, k);
  }
  hipStream_t s = stream_of(ctx);
  hipLaunchKernelGGL(where_kernel, ix_grid(n), dim3(256), 0, s, cond->data, x->data, y->data,
                     out->data, n, d);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

static rtenhip_status cast_desc(const rtenhip_tensor* x, const rtenhip_tensor* y, IdxDesc& d) {
  if (!x || !y) return fail(RTENHIP_INVALID_VALUE, "null argument");
  if (!out_matches(y, x->shape, x->ndim))
    return fail(RTENHIP_INCOMPATIBLE_INPUT_SHAPES, "Output tensor has the wrong shape");
  d = IdxDesc{};
  d.ndim = x->ndim;
  for (int k = 0; k < x->ndim; k++) {
    d.shape[k] = x->shape[k];
    d.s0[k] = x->strides[k];
  }
  return RTENHIP_OK;
}

extern "C" rtenhip_status rtenhip_cast_f32_to_i32(rtenhip_ctx* ctx, const rtenhip_tensor* x,
                                                  rtenhip_tensor_i32* y) {
  IdxDesc d;
  rtenhip_status st = cast_desc(x, as_f(y), d);
  if (st) return st;
  const int64_t n = numel(*x);
  if (n == 0) return RTENHIP_OK;
  hipLaunchKernelGGL(cast_f2i_kernel, ix_grid(n), dim3(256), 0, stream_of(ctx), x->data, y->data,
                     n, d);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

extern "C" rtenhip_status rtenhip_cast_i32_to_f32(rtenhip_ctx* ctx, const rtenhip_tensor_i32* x,
                                                  rtenhip_tensor* y) {
  IdxDesc d;
  rtenhip_status st = cast_desc(as_f(x), y, d);
  if (st) return st;
  const int64_t n = numel(*y);
  if (n == 0) return RTENHIP_OK;
  hipLaunchKernelGGL(cast_i2f_kernel, ix_grid(n), dim3(256), 0, stream_of(ctx), x->data, y->data,
                     n, d);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}
