// Context object behind rtenhip_ctx.
#pragma once

#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <tuple>

#include "common.h"

namespace rtenhip {

struct Ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  // Thread count RTen would run with (RTEN_NUM_THREADS semantics,
  // src/threading.rs:41-62).  It only changes numerics in the gemv path,
  // where the reference's column blocking depends on it (gemm.rs:673).
  int ref_threads = 0;
  std::mutex mu;
  std::map<std::tuple<int, int, int, int, int, int, int>, int2*> ktabs;
  void* scratch = nullptr;
  size_t scratch_cap[2] = {0, 0};

  explicit Ctx(int dev);
  ~Ctx();
  // Grow-only device scratch (two independent slots).  Synchronizes the
  // stream when it has to grow, so callers must not be capturing.
  float* scratch_floats(size_t n, size_t slot);
  // Device table of VirtualIm2Col row offsets for one conv geometry.
  const int2* ktab(int C, int H, int W, int kh, int kw, int dh, int dw);
};

rtenhip_status output_size_and_padding(int64_t in_h, int64_t in_w, int64_t k_h, int64_t k_w,
                                       int64_t stride_h, int64_t stride_w, int pad_mode,
                                       const int64_t* pads_in, int64_t dil_y, int64_t dil_x,
                                       int64_t out_hw[2], int64_t pads[4]);
rtenhip_status conv_impl(Ctx* c, const rtenhip_tensor* x, const rtenhip_tensor* w,
                         const float* bias, int pad_mode, const int64_t* pads,
                         const int64_t* strides, const int64_t* dilations, int64_t groups,
                         const float* residual, int act, float lo, float hi, rtenhip_tensor* y);
rtenhip_status gemm_impl(Ctx* c, int64_t m, int64_t n, int64_t k, const float* a, int64_t a_rs,
                         int64_t a_cs, const float* b, int64_t b_rs, int64_t b_cs, float* out,
                         int64_t out_rs, float alpha, float beta, const float* bias, int act);

// broadcast_shapes (src/ops/binary_elementwise.rs:23-45).
bool broadcast_shapes(const int64_t* a, int an, const int64_t* b, int bn, int64_t* out, int* on);

}  // namespace rtenhip
