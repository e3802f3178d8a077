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

// vm_exp on two values at once: the same operations in the same order, the
// fma / mul / add steps as packed f32 instructions (v_pk_fma_f32 etc., one
// IEEE-rounded operation per component), so each lane equals vm_exp bit for bit.
typedef float vm_f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ vm_f32x2 vm_exp2(vm_f32x2 x) {
  const vm_f32x2 INV_LOG2 = {1.44269504088896340736f, 1.44269504088896340736f};
  const vm_f32x2 MAGIC = {12582912.f, 12582912.f};
  const vm_f32x2 LN2_HI = {-6.93145752e-1f, -6.93145752e-1f}, LN2_LO = {-1.42860677e-6f, -1.42860677e-6f};
  vm_f32x2 j = __builtin_elementwise_fma(x, INV_LOG2, MAGIC);
  j = j - MAGIC;
  vm_f32x2 r = __builtin_elementwise_fma(j, LN2_HI, x);
  r = __builtin_elementwise_fma(j, LN2_LO, r);
  vm_f32x2 t = {1.37805939e-3f, 1.37805939e-3f};
  t = __builtin_elementwise_fma(t, r, (vm_f32x2){8.37312452e-3f, 8.37312452e-3f});
  t = __builtin_elementwise_fma(t, r, (vm_f32x2){4.16695364e-2f, 4.16695364e-2f});
  t = __builtin_elementwise_fma(t, r, (vm_f32x2){1.66664720e-1f, 1.66664720e-1f});
  t = __builtin_elementwise_fma(t, r, (vm_f32x2){4.99999851e-1f, 4.99999851e-1f});
  t = __builtin_elementwise_fma(t, r, (vm_f32x2){1.0f, 1.0f});
  r = __builtin_elementwise_fma(t, r, (vm_f32x2){1.0f, 1.0f});
  vm_f32x2 s1, s2;
#pragma unroll
  for (int c = 0; c < 2; c++) {
    const float jc = j[c];
    const int32_t k = (jc != jc || jc >= 2147483648.f || jc < -2147483648.f) ? INT32_MIN : (int32_t)jc;
    const uint32_t ia = k > 0 ? 0u : 0x83000000u;
    s1[c] = __uint_as_float(ia + 0x7f000000u);
    s2[c] = __uint_as_float(((uint32_t)k << 23) - ia);
  }
  r = r * s1;
  r = r * s2;
#pragma unroll
  for (int c = 0; c < 2; c++) {
    if (x[c] >= 104.f) r[c] = __builtin_huge_valf();
    if (x[c] <= -104.f) r[c] = 0.f;
  }
  return r;
}

// vm_exp2 for arguments that are <= 0 or NaN (softmax's x - max, GELU's
// -z^2), bit for bit.  There k = j <= 0 (or the value is replaced), so the
// scale split is fixed: s1 = 2^-123 and s2 = (k << 23) - 0x83000000, and k
// comes straight from the magic-number sum's low mantissa bits (j + MAGIC =
// 1.5 * 2^23 + k exactly while |k| < 2^22; 0x4B400000 << 23 wraps to 0), so
// the conversion and its NaN / range guards drop out.  Values where that
// does not hold (x <= -104, -inf) are replaced by the 0 clamp as in vm_exp;
// x >= 104 cannot occur; a NaN stays the same NaN through the fmas and the
// finite scales.
__device__ __forceinline__ vm_f32x2 vm_exp2_nonpos(vm_f32x2 x) {
  const vm_f32x2 INV_LOG2 = {1.44269504088896340736f, 1.44269504088896340736f};
  const vm_f32x2 MAGIC = {12582912.f, 12582912.f};
  const vm_f32x2 LN2_HI = {-6.93145752e-1f, -6.93145752e-1f}, LN2_LO = {-1.42860677e-6f, -1.42860677e-6f};
  const vm_f32x2 jm = __builtin_elementwise_fma(x, INV_LOG2, MAGIC);
  const vm_f32x2 j = jm - MAGIC;
  vm_f32x2 r = __builtin_elementwise_fma(j, LN2_HI, x);
  r = __builtin_elementwise_fma(j, LN2_LO, r);
  vm_f32x2 t = {1.37805939e-3f, 1.37805939e-3f};
  t = __builtin_elementwise_fma(t, r, (vm_f32x2){8.37312452e-3f, 8.37312452e-3f});
  t = __builtin_elementwise_fma(t, r, (vm_f32x2){4.16695364e-2f, 4.16695364e-2f});
  t = __builtin_elementwise_fma(t, r, (vm_f32x2){1.66664720e-1f, 1.66664720e-1f});
  t = __builtin_elementwise_fma(t, r, (vm_f32x2){4.99999851e-1f, 4.99999851e-1f});
  t = __builtin_elementwise_fma(t, r, (vm_f32x2){1.0f, 1.0f});
  r = __builtin_elementwise_fma(t, r, (vm_f32x2){1.0f, 1.0f});
  vm_f32x2 s2;
#pragma unroll
  for (int c = 0; c < 2; c++) s2[c] = __uint_as_float((__float_as_uint(jm[c]) << 23) + 0x7D000000u);
  r = r * (vm_f32x2){__uint_as_float(0x02000000u), __uint_as_float(0x02000000u)};
  r = r * s2;
#pragma unroll
  for (int c = 0; c < 2; c++)
    if (x[c] <= -104.f) r[c] = 0.f;
  return r;
}

// a / b for many a over one b (softmax's normalisation).  The compiler's f32
// division is v_div_scale (both operands), v_rcp, two fma refinements of the
// reciprocal, three fma quotient steps, v_div_fmas and v_div_fixup; with the
// divisor in [1, 256] and a == +0 or a in [2^-60, 2] div_scale scales neither
// operand (VCC = 0, so div_fmas is a plain fma) and div_fixup has nothing to
// fix, so the same steps without them, the divisor-only ones done once, give
// __fdiv_rn(a, b) bit for bit (checked on random operands by
// tests/test_vecmath_gpu.py through rtenhip_debug_div_check).  Other a take
// __fdiv_rn.
struct DivBy {
  float b, nb, r;
  bool ok;
};
__device__ __forceinline__ DivBy div_by_init(float b) {
  DivBy d;
  d.b = b;
  d.nb = -b;
  const float r0 = __builtin_amdgcn_rcpf(b);
  d.r = __fmaf_rn(__fmaf_rn(d.nb, r0, 1.f), r0, r0);
  d.ok = b >= 1.f && b <= 256.f;
  return d;
}
// Whether div_by_fast(d, a) is exact for this a.
__device__ __forceinline__ bool div_by_ok(const DivBy& d, float a) {
  return d.ok && (__float_as_uint(a) == 0u || (a >= 0x1p-60f && a <= 2.f));
}
// The shortcut alone (callers check div_by_ok first, e.g. once per wave).
__device__ __forceinline__ float div_by_fast(const DivBy& d, float a) {
  const float q = __fmul_rn(a, d.r);
  const float f2 = __fmaf_rn(d.nb, q, a);
  const float f3 = __fmaf_rn(f2, d.r, q);
  const float f4 = __fmaf_rn(d.nb, f3, a);
  return __fmaf_rn(f4, d.r, f3);
}
// div_by_fast on two values (packed f32 operations, the same steps).
__device__ __forceinline__ vm_f32x2 div_by_fast2(const DivBy& d, vm_f32x2 a) {
  const vm_f32x2 r = {d.r, d.r}, nb = {d.nb, d.nb};
  const vm_f32x2 q = a * r;
  const vm_f32x2 f2 = __builtin_elementwise_fma(nb, q, a);
  const vm_f32x2 f3 = __builtin_elementwise_fma(f2, r, q);
  const vm_f32x2 f4 = __builtin_elementwise_fma(nb, f3, a);
  return __builtin_elementwise_fma(f4, r, f3);
}
__device__ __forceinline__ float div_by(const DivBy& d, float a) {
  return div_by_ok(d, a) ? div_by_fast(d, a) : __fdiv_rn(a, d.b);
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

// vm_gelu on two values at once (vm_erf inlined): the same operations in the
// same order, packed where both components take the same one, so each lane
// equals vm_gelu bit for bit.
__device__ __forceinline__ vm_f32x2 vm_gelu2(vm_f32x2 x) {
  const vm_f32x2 zero = {0.f, 0.f}, one = {1.f, 1.f};
  const vm_f32x2 half_x = x * (vm_f32x2){0.5f, 0.5f};
  const vm_f32x2 z = x * (vm_f32x2){0.70710678118654752440f, 0.70710678118654752440f};
  const vm_f32x2 nz = zero - z;
  vm_f32x2 az;
  az[0] = z[0] < 0.f ? nz[0] : z[0];
  az[1] = z[1] < 0.f ? nz[1] : z[1];
  const vm_f32x2 den = __builtin_elementwise_fma(az, (vm_f32x2){0.3275911f, 0.3275911f}, one);
  vm_f32x2 t;
  t[0] = __fdiv_rn(1.f, den[0]);
  t[1] = __fdiv_rn(1.f, den[1]);
  vm_f32x2 y = {1.061405429f, 1.061405429f};
  y = __builtin_elementwise_fma(y, t, (vm_f32x2){-1.453152027f, -1.453152027f});
  y = __builtin_elementwise_fma(y, t, (vm_f32x2){1.421413741f, 1.421413741f});
  y = __builtin_elementwise_fma(y, t, (vm_f32x2){-0.284496736f, -0.284496736f});
  y = __builtin_elementwise_fma(y, t, (vm_f32x2){0.254829592f, 0.254829592f});
  const vm_f32x2 at = y * t;
  const vm_f32x2 e = vm_exp2_nonpos(zero - az * az);
  const vm_f32x2 r = one - at * e;
  const vm_f32x2 nr = zero - r;
  vm_f32x2 erf;
  erf[0] = z[0] < 0.f ? nr[0] : r[0];
  erf[1] = z[1] < 0.f ? nr[1] : r[1];
  return half_x * (erf + one);
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

// Clip: RTen's Clamp::clamp (src/ops/unary_elementwise.rs:263-291), i.e.
// self.max(lo).min(hi) with the trait's own max (self > val ? self : val) and
// min (self < val ? self : val) -- not f32::clamp: NaN becomes lo (then
// min(lo, hi)), and a zero equal to a bound becomes that bound's zero
// (Clip(0, 6) maps -0 to +0).
__host__ __device__ __forceinline__ float rust_clamp(float x, float lo, float hi) {
  const float m = x > lo ? x : lo;
  return m < hi ? m : hi;
}

}  // namespace rtenhip
