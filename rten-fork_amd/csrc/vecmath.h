// Device restatement of rten-vecmath's f32 approximations, bit-compatible
// with the reference's SIMD code: every mul_add is an explicit fma and every
// other operation rounds separately (__f*_rn intrinsics; the library is also
// compiled with -ffp-contract=off).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace rtenhip {

// simd_exp (rten-vecmath/src/exp.rs:73-133): Cody-Waite reduction + degree-6
// polynomial, exponent scaling split into two factors, +-104 clamps.
__device__ __forceinline__ float vm_exp(float x) {
  const float INV_LOG2 = 1.44269504088896340736f, MAGIC = 12582912.f;
  const float LN2_HI = -6.93145752e-1f, LN2_LO = -1.42860677e-6f;
  float j = __fmaf_rn(x, INV_LOG2, MAGIC);
  j = __fsub_rn(j, MAGIC);
  float r = __fmaf_rn(j, LN2_HI, x);
  r = __fmaf_rn(j, LN2_LO, r);
  // _mm256_cvttps_epi32: NaN / out of range -> INT_MIN.
  int32_t k = (j != j || j >= 2147483648.f || j < -2147483648.f) ? INT32_MIN : (int32_t)j;
  float t = 1.37805939e-3f;
  t = __fmaf_rn(t, r, 8.37312452e-3f);
  t = __fmaf_rn(t, r, 4.16695364e-2f);
  t = __fmaf_rn(t, r, 1.66664720e-1f);
  t = __fmaf_rn(t, r, 4.99999851e-1f);
  t = __fmaf_rn(t, r, 1.0f);
  r = __fmaf_rn(t, r, 1.0f);
  uint32_t ia = k > 0 ? 0u : 0x83000000u;
  uint32_t is = ia + 0x7f000000u;
  uint32_t it = ((uint32_t)k << 23) - ia;
  r = __fmul_rn(r, __uint_as_float(is));
  r = __fmul_rn(r, __uint_as_float(it));
  if (x >= 104.f) r = __builtin_huge_valf();
  if (x <= -104.f) r = 0.f;
  return r;
}

// simd_sigmoid (exp.rs:144-148): 1 / (1 + exp(0 - x)).
__device__ __forceinline__ float vm_sigmoid(float x) {
  return __fdiv_rn(1.f, __fadd_rn(1.f, vm_exp(__fsub_rn(0.f, x))));
}

// simd_erf (erf.rs:29-58): Abramowitz & Stegun 7.1.26.
__device__ __forceinline__ float vm_erf(float x) {
  const bool neg = x < 0.f;
  const float ax = neg ? __fsub_rn(0.f, x) : x;
  const float t = __fdiv_rn(1.f, __fmaf_rn(ax, 0.3275911f, 1.f));
  float y = 1.061405429f;
  y = __fmaf_rn(y, t, -1.453152027f);
  y = __fmaf_rn(y, t, 1.421413741f);
  y = __fmaf_rn(y, t, -0.284496736f);
  y = __fmaf_rn(y, t, 0.254829592f);
  const float at = __fmul_rn(y, t);
  const float e = vm_exp(__fsub_rn(0.f, __fmul_rn(ax, ax)));
  const float r = __fsub_rn(1.f, __fmul_rn(at, e));
  return neg ? __fsub_rn(0.f, r) : r;
}

// simd_gelu (erf.rs:85-91): 0.5x * (1 + erf(x / sqrt 2)).
__device__ __forceinline__ float vm_gelu(float x) {
  const float half_x = __fmul_rn(x, 0.5f);
  const float y = __fadd_rn(vm_erf(__fmul_rn(x, 0.70710678118654752440f)), 1.f);
  return __fmul_rn(half_x, y);
}

// simd_tanh (tanh.rs:14-65).
__device__ __forceinline__ float vm_tanh(float x) {
  const bool x_neg = x <= 0.f;
  const float ax = fabsf(x);
  const bool cutoff = ax >= 9.02f, tiny = ax <= 0.0004f, small = ax <= 0.55f;
  const float xs = __fmul_rn(x, x);
  float ys = __fmaf_rn(1.5497927553951740264892578125e-2f, xs, -5.21197654306888580322265625e-2f);
  ys = __fmaf_rn(ys, xs, 0.13310669362545013427734375f);
  ys = __fmaf_rn(ys, xs, -0.33332359790802001953125f);
  ys = __fmaf_rn(ys, xs, 0.999999940395355224609375f);
  ys = __fmul_rn(ys, ax);
  const float e = vm_exp(__fmul_rn(ax, 2.f));
  const float ym = __fdiv_rn(__fsub_rn(e, 1.f), __fadd_rn(e, 1.f));
  float y = cutoff ? 1.f : ym;
  y = small ? ys : y;
  y = tiny ? ax : y;
  return x_neg ? __fsub_rn(0.f, y) : y;
}

// Correctly rounded f32 sqrt (Rust's f32::sqrt is IEEE).  v_sqrt_f32 is
// accurate to ~1 ulp only, so the result is corrected by one ulp in either
// direction from the sign of the fma residuals (the expansion LLVM uses for
// correctly rounded sqrt); tiny inputs are pre-scaled by 2^32.
__device__ __forceinline__ float sqrt_rn(float x) {
  const bool tiny = x < 1.0e-28f;  // ~2^-93: keep the scaled value normal
  const float xs = tiny ? __fmul_rn(x, 4294967296.f) : x;
  float s = __builtin_amdgcn_sqrtf(xs);
  const int si = __float_as_int(s);
  const float sdn = __int_as_float(si - 1), sup = __int_as_float(si + 1);
  const float rdn = __fmaf_rn(-sdn, s, xs);
  const float rup = __fmaf_rn(-sup, s, xs);
  if (rdn <= 0.f) s = sdn;
  if (rup > 0.f) s = sup;
  if (xs == 0.f || xs == __builtin_huge_valf() || !(xs >= 0.f)) s = __builtin_amdgcn_sqrtf(xs);
  return tiny ? __fmul_rn(s, 1.52587890625e-05f) : s;
}

// f32::max (NaN operand -> the other operand), as Relu uses it.
__device__ __forceinline__ float rust_max(float a, float b) { return fmaxf(a, b); }

// f32::clamp(lo, hi): NaN stays NaN.
__device__ __forceinline__ float rust_clamp(float x, float lo, float hi) {
  return x < lo ? lo : (x > hi ? hi : x);
}

}  // namespace rtenhip
