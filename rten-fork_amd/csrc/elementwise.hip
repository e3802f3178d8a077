// Elementwise kernels: unary activations (src/ops/unary_elementwise.rs with
// rten-vecmath numerics), broadcasting binary ops
// (src/ops/binary_elementwise.rs:158-439), BatchNormalization
// (src/ops/norm.rs:18-54) and strided copies (make-contiguous).
//
// All are HBM-bound streaming kernels: 16-byte vector loads/stores where the
// layout allows, grid capped at ~2048 blocks and grid-strided.
#include "common.h"
#include "vecmath.h"

namespace rtenhip {

template <int OP>
__device__ __forceinline__ float unary_apply(float v, float p0, float p1) {
  if constexpr (OP == RTENHIP_UNARY_RELU) return rust_max(v, 0.f);
  if constexpr (OP == RTENHIP_UNARY_CLIP) return rust_clamp(v, p0, p1);
  if constexpr (OP == RTENHIP_UNARY_GELU) return vm_gelu(v);
  if constexpr (OP == RTENHIP_UNARY_ERF) return vm_erf(v);
  if constexpr (OP == RTENHIP_UNARY_SIGMOID) return vm_sigmoid(v);
  if constexpr (OP == RTENHIP_UNARY_TANH) return vm_tanh(v);
  if constexpr (OP == RTENHIP_UNARY_EXP) return vm_exp(v);
  if constexpr (OP == RTENHIP_UNARY_SILU) return __fmul_rn(v, vm_sigmoid(v));
  if constexpr (OP == RTENHIP_UNARY_SQRT) return sqrt_rn(v);
  return v;
}

template <int OP>
__global__ void unary_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n,
                             float p0, float p1) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool vec = ((((uintptr_t)x) | ((uintptr_t)y)) & 15) == 0;
  if (vec) {
    const int64_t n4 = n / 4;
    for (int64_t v = i; v < n4; v += stride) {
      float4 a = reinterpret_cast<const float4*>(x)[v];
      a.x = unary_apply<OP>(a.x, p0, p1);
      a.y = unary_apply<OP>(a.y, p0, p1);
      a.z = unary_apply<OP>(a.z, p0, p1);
      a.w = unary_apply<OP>(a.w, p0, p1);
      reinterpret_cast<float4*>(y)[v] = a;
    }
    for (int64_t t = n4 * 4 + i; t < n; t += stride) y[t] = unary_apply<OP>(x[t], p0, p1);
  } else {
    for (int64_t t = i; t < n; t += stride) y[t] = unary_apply<OP>(x[t], p0, p1);
  }
}

static dim3 stream_grid(int64_t n, int per_thread = 4) {
  int64_t blocks = (n / per_thread + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 4096) blocks = 4096;
  return dim3((unsigned)blocks);
}

rtenhip_status launch_unary(int op, const float* x, float* y, int64_t n, float p0, float p1,
                            hipStream_t s) {
  if (n == 0) return RTENHIP_OK;
  dim3 g = stream_grid(n), b(256);
  switch (op) {
#define CASE(OPV)                                                              \
  case OPV:                                                                    \
    hipLaunchKernelGGL(unary_kernel<OPV>, g, b, 0, s, x, y, n, p0, p1);        \
    break;
    CASE(RTENHIP_UNARY_RELU)
    CASE(RTENHIP_UNARY_CLIP)
    CASE(RTENHIP_UNARY_GELU)
    CASE(RTENHIP_UNARY_ERF)
    CASE(RTENHIP_UNARY_SIGMOID)
    CASE(RTENHIP_UNARY_TANH)
    CASE(RTENHIP_UNARY_EXP)
    CASE(RTENHIP_UNARY_SILU)
    CASE(RTENHIP_UNARY_SQRT)
#undef CASE
    default:
      return fail(RTENHIP_UNSUPPORTED_VALUE, "Unsupported unary op");
  }
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

template <int OP>
__device__ __forceinline__ float binary_apply(float a, float b) {
  if constexpr (OP == RTENHIP_BINARY_ADD) return __fadd_rn(a, b);
  if constexpr (OP == RTENHIP_BINARY_SUB) return __fsub_rn(a, b);
  if constexpr (OP == RTENHIP_BINARY_MUL) return __fmul_rn(a, b);
  if constexpr (OP == RTENHIP_BINARY_POW) {
    // powf with the reference's fast paths (binary_elementwise.rs:742-751)
    if (b == 2.f) return __fmul_rn(a, a);
    if (b == 3.f) return __fmul_rn(__fmul_rn(a, a), a);
    return (float)pow((double)a, (double)b);
  }
  return __fdiv_rn(a, b);
}

// mode 0: same shape, contiguous.  mode 1: b repeats every `inner` elements
// of a (row broadcast, e.g. bias [C] over [..., C]).  mode 2: b constant per
// run of `inner` elements cycling (e.g. [C,1,1] over [N,C,H,W]): b index =
// (i / inner) % nb.  mode 3: general strided broadcast.
template <int OP>
__global__ void binary_kernel(const float* __restrict__ a, const float* __restrict__ b,
                              float* __restrict__ y, int64_t n, BcastDesc d, int mode,
                              int64_t inner, int64_t nb) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float av, bv;
    if (mode == 0) {
      av = a[i];
      bv = b[i];
    } else if (mode == 1) {
      av = a[i];
      bv = b[i % inner];
    } else if (mode == 2) {
      av = a[i];
      bv = b[(i / inner) % nb];
    } else {
      int64_t rem = i, oa = 0, ob = 0;
      for (int k = d.ndim - 1; k >= 0; k--) {
        int64_t idx = rem % d.shape[k];
        rem /= d.shape[k];
        oa += idx * d.sa[k];
        ob += idx * d.sb[k];
      }
      av = a[oa];
      bv = b[ob];
    }
    y[i] = binary_apply<OP>(av, bv);
  }
}

rtenhip_status launch_binary(int op, const float* a, const float* b, float* y, int64_t n,
                             const BcastDesc& d, int mode, int64_t inner, int64_t nb,
                             hipStream_t s) {
  if (n == 0) return RTENHIP_OK;
  dim3 g = stream_grid(n, 1), bl(256);
  switch (op) {
    case RTENHIP_BINARY_ADD:
      hipLaunchKernelGGL(binary_kernel<RTENHIP_BINARY_ADD>, g, bl, 0, s, a, b, y, n, d, mode, inner, nb);
      break;
    case RTENHIP_BINARY_SUB:
      hipLaunchKernelGGL(binary_kernel<RTENHIP_BINARY_SUB>, g, bl, 0, s, a, b, y, n, d, mode, inner, nb);
      break;
    case RTENHIP_BINARY_MUL:
      hipLaunchKernelGGL(binary_kernel<RTENHIP_BINARY_MUL>, g, bl, 0, s, a, b, y, n, d, mode, inner, nb);
      break;
    case RTENHIP_BINARY_DIV:
      hipLaunchKernelGGL(binary_kernel<RTENHIP_BINARY_DIV>, g, bl, 0, s, a, b, y, n, d, mode, inner, nb);
      break;
    case RTENHIP_BINARY_POW:
      hipLaunchKernelGGL(binary_kernel<RTENHIP_BINARY_POW>, g, bl, 0, s, a, b, y, n, d, mode, inner, nb);
      break;
    default:
      return fail(RTENHIP_UNSUPPORTED_VALUE, "Unsupported binary op");
  }
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

// batch_norm_in_place (norm.rs:18-54): per (n, c) plane,
// y = (x - mean) * (scale / sqrt(var + eps)) + bias, separate roundings.
__global__ void batch_norm_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t C,
                                  int64_t inner, const float* __restrict__ scale,
                                  const float* __restrict__ bias, const float* __restrict__ mean,
                                  const float* __restrict__ var, float eps) {
  const int64_t plane = blockIdx.y;  // n*C + c
  const int64_t c = plane % C;
  const float sc = __fdiv_rn(scale[c], sqrt_rn(__fadd_rn(var[c], eps)));
  const float mu = mean[c], bi = bias[c];
  const float* xp = x + plane * inner;
  float* yp = y + plane * inner;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < inner;
       i += (int64_t)gridDim.x * blockDim.x)
    yp[i] = __fadd_rn(__fmul_rn(__fsub_rn(xp[i], mu), sc), bi);
}

rtenhip_status launch_batch_norm(const float* x, float* y, int64_t N, int64_t C, int64_t inner,
                                 const float* scale, const float* bias, const float* mean,
                                 const float* var, float eps, hipStream_t s) {
  if (N * C * inner == 0) return RTENHIP_OK;
  int64_t bx = (inner + 255) / 256;
  if (bx > 64) bx = 64;
  hipLaunchKernelGGL(batch_norm_kernel, dim3((unsigned)bx, (unsigned)(N * C)), dim3(256), 0, s, x,
                     y, C, inner, scale, bias, mean, var, eps);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

// Zero-bordered copy of an NCHW tensor: out [N, C, H+pt+pb, W+pl+pr].  Gives
// the DMA GEMM a conv input that needs no bounds checks (the border holds the
// zeros the reference's im2col would insert, im2col.rs:236-248).
// One padded row per wave, lanes over its columns (coalesced); the row's
// source and validity are computed once per row, no per-element division.
__global__ __launch_bounds__(256) void pad_nchw_kernel(const float* __restrict__ x,
                                                       float* __restrict__ y, int rows, int H,
                                                       int W, int Hp, int Wp, int pt, int pl) {
  const int r = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (r >= rows) return;
  const int plane = r / Hp;
  const int yh = r - plane * Hp - pt;
  const bool in = (unsigned)yh < (unsigned)H;
  const float* xr = x + ((int64_t)plane * H + (in ? yh : 0)) * W;
  float* yr = y + (int64_t)r * Wp;
  const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(yr, 0, Wp * 4, 0x00020000);
  // Up to 4 * 64 columns per pass with every load issued before the stores
  // (a store-then-load loop would wait for each store: vmcnt is in order).
  for (int c0 = 0; c0 < Wp; c0 += 256) {
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int c = c0 + j * 64 + (threadIdx.x & 63);
      const int xw = c - pl;
      const bool ok = in && c < Wp && (unsigned)xw < (unsigned)W;
      v[j] = ok ? xr[xw] : 0.f;
    }
    // Columns past the row end get an out-of-range buffer offset: the store
    // is dropped by the hardware, so no lane-divergent branch (and no
    // conservative wait) around the stores.
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int c = c0 + j * 64 + (threadIdx.x & 63);
      const uint32_t off = c < Wp ? (uint32_t)(c * 4) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[j]), yrs, off, 0, 0);
    }
  }
}

rtenhip_status launch_pad_nchw(const float* x, float* y, int64_t planes, int H, int W, int pt,
                               int pl, int pb, int pr, hipStream_t s) {
  const int Hp = H + pt + pb, Wp = W + pl + pr;
  const int64_t rows = planes * Hp;
  if (rows == 0 || Wp == 0) return RTENHIP_OK;
  if (rows >= (int64_t(1) << 31)) return fail(RTENHIP_UNSUPPORTED_VALUE, "padded input too large");
  hipLaunchKernelGGL(pad_nchw_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, x, y,
                     (int)rows, H, W, Hp, Wp, pt, pl);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

// Strided -> contiguous copy (to_contiguous_in).
struct CopyDesc {
  int ndim;
  int64_t shape[RTENHIP_MAX_DIMS];
  int64_t strides[RTENHIP_MAX_DIMS];
};
__global__ void copy_strided_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n,
                                    CopyDesc d) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    int64_t rem = i, off = 0;
    for (int k = d.ndim - 1; k >= 0; k--) {
      off += (rem % d.shape[k]) * d.strides[k];
      rem /= d.shape[k];
    }
    y[i] = x[off];
  }
}

rtenhip_status launch_copy_strided(const rtenhip_tensor& src, float* dst, hipStream_t s) {
  int64_t n = numel(src);
  if (n == 0) return RTENHIP_OK;
  CopyDesc d{};
  d.ndim = src.ndim;
  for (int i = 0; i < src.ndim; i++) {
    d.shape[i] = src.shape[i];
    d.strides[i] = src.strides[i];
  }
  hipLaunchKernelGGL(copy_strided_kernel, stream_grid(n, 1), dim3(256), 0, s, src.data, dst, n, d);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

// Strided view -> strided view copy of 4-byte elements (Concat's blocks,
// Slice / Expand views into a strided destination).
struct ViewDesc {
  int ndim;
  int64_t shape[RTENHIP_MAX_DIMS];
  int64_t src[RTENHIP_MAX_DIMS];
  int64_t dst[RTENHIP_MAX_DIMS];
};
__global__ void copy_view_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n, ViewDesc d) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    int64_t rem = i, so = 0, dof = 0;
    for (int k = d.ndim - 1; k >= 0; k--) {
      const int64_t idx = rem % d.shape[k];
      rem /= d.shape[k];
      so += idx * d.src[k];
      dof += idx * d.dst[k];
    }
    y[dof] = x[so];
  }
}

rtenhip_status launch_copy_view(const float* src, const int64_t* shape, const int64_t* src_strides, int ndim,
                                float* dst, const int64_t* dst_strides, hipStream_t s) {
  int64_t n = 1;
  for (int i = 0; i < ndim; i++) n *= shape[i];
  if (n == 0) return RTENHIP_OK;
  if (ndim > RTENHIP_MAX_DIMS) return fail(RTENHIP_UNSUPPORTED_VALUE, "too many dims");
  ViewDesc d{};
  d.ndim = ndim;
  for (int i = 0; i < ndim; i++) {
    d.shape[i] = shape[i];
    d.src[i] = src_strides[i];
    d.dst[i] = dst_strides[i];
  }
  hipLaunchKernelGGL(copy_view_kernel, stream_grid(n, 1), dim3(256), 0, s, src, dst, n, d);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

// ConstantOfShape on the device (generate.rs:28-42): every element = v.
__global__ void fill_kernel(uint32_t* __restrict__ y, int64_t n, uint32_t v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = v;
}

rtenhip_status launch_fill(void* y, int64_t n, uint32_t bits, hipStream_t s) {
  if (n == 0) return RTENHIP_OK;
  hipLaunchKernelGGL(fill_kernel, stream_grid(n, 1), dim3(256), 0, s, static_cast<uint32_t*>(y), n, bits);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

// Timing runs only (Graph::run with timing on): one wave that holds the
// stream until the host has queued the whole eager plan, so the per-op event
// pairs time the kernels back to back instead of the host's launch pace.  It
// polls word[0] of pinned, uncached host memory the host sets after queueing
// (a load over PCIe each time, so never stale) and gives up after max_ticks
// of s_memrealtime (100 MHz) whatever happens: it cannot hang the queue.  On
// giving up it sets word[1] (a vector store from lane 0), so the host can tell
// that the events of that run include host time (Graph::run's report).
__global__ void hold_kernel(int* word, uint64_t max_ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  bool released = false;
  while (__builtin_amdgcn_s_memrealtime() - t0 < max_ticks) {
    if (__hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
      released = true;
      break;
    }
    __builtin_amdgcn_s_sleep(64);
  }
  if (!released && threadIdx.x == 0) __hip_atomic_store(word + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

rtenhip_status launch_hold(int* word, double max_ms, hipStream_t s) {
  const uint64_t ticks = (uint64_t)(max_ms * 1e5);  // s_memrealtime runs at 100 MHz
  hipLaunchKernelGGL(hold_kernel, dim3(1), dim3(64), 0, s, word, ticks);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

// col2im (src/ops/conv.rs:329-375), one thread per output element: the
// reference fills the plane with the bias and adds each (ky, kx) column image
// in turn, so an output receives bias + its columns in (ky, kx) order.
__global__ void col2im_kernel(const float* __restrict__ col, const float* __restrict__ bias,
                              float* __restrict__ y, int64_t total, int O, int OH, int OW, int H,
                              int W, int kh, int kw, int sh, int sw, int pt, int pl) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int ox = (int)(i % OW);
    const int oy = (int)((i / OW) % OH);
    const int64_t nc = i / ((int64_t)OW * OH);
    const int c = (int)(nc % O);
    const int64_t n = nc / O;
    float acc = bias ? bias[c] : 0.f;
    const float* cb = col + ((n * O + c) * kh * kw) * (int64_t)H * W;
    for (int ky = 0; ky < kh; ky++) {
      const int yy = oy + pt - ky;
      if (yy < 0 || yy % sh) continue;
      const int yi = yy / sh;
      if (yi >= H) continue;
      for (int kx = 0; kx < kw; kx++) {
        const int xx = ox + pl - kx;
        if (xx < 0 || xx % sw) continue;
        const int xi = xx / sw;
        if (xi >= W) continue;
        acc = __fadd_rn(acc, cb[((int64_t)(ky * kw + kx) * H + yi) * W + xi]);
      }
    }
    y[i] = acc;
  }
}

rtenhip_status launch_col2im(const float* col, const float* bias, float* y, int64_t N, int64_t O,
                             int64_t OH, int64_t OW, int64_t H, int64_t W, int64_t kh,
                             int64_t kw, int64_t sh, int64_t sw, int64_t pt, int64_t pl,
                             hipStream_t s) {
  const int64_t total = N * O * OH * OW;
  if (total == 0) return RTENHIP_OK;
  const int64_t blocks = std::min<int64_t>((total + 255) / 256, 16384);
  hipLaunchKernelGGL(col2im_kernel, dim3((unsigned)blocks), dim3(256), 0, s, col, bias, y, total,
                     (int)O, (int)OH, (int)OW, (int)H, (int)W, (int)kh, (int)kw, (int)sh, (int)sw,
                     (int)pt, (int)pl);
  RTENHIP_LAUNCH_CHECK();
  return RTENHIP_OK;
}

}  // namespace rtenhip
