// Shared helpers for the CPU oracle (test infrastructure; see rten_oracle.h).
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../rten_oracle.h"

namespace orc {

void set_error(int code, const std::string& msg);
int fail(int code, const char* msg);

int threads();

// Strided matrix view (rten_tensor::Matrix).
struct Mat {
  const float* data;
  int64_t rows, cols;
  int64_t rs, cs;  // element strides
  float at(int64_t r, int64_t c) const { return data[r * rs + c * cs]; }
};

// Virtual B operand (VirtualMatrix, src/gemm.rs:133-161): packs rows
// [k0,k1) x cols [c0,c1) into NR-wide row-major panels, zero padded.
struct VirtualB {
  virtual ~VirtualB() {}
  virtual int64_t rows() const = 0;
  virtual int64_t cols() const = 0;
  virtual void pack_b(float* out, int64_t nr, int64_t k0, int64_t k1, int64_t c0,
                      int64_t c1) const = 0;
};

// GemmExecutor::gemm_bias with Unpacked A and Unpacked/Virtual B.
// `force_serial` runs on the calling thread only (used inside per-image
// parallel loops, mirroring rayon's nested scheduling without changing the
// per-element summation order, which is thread-count independent).
void gemm_impl(float* out, int64_t out_rs, const Mat& a, const Mat* b, const VirtualB* vb,
               float alpha, float beta, const float* bias, bool force_serial);

// Helpers shared by ops.
int64_t numel(const int64_t* shape, int ndim);

}  // namespace orc
