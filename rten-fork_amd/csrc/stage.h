// Batched global -> LDS staging shared by the pooling, depthwise and fused
// MobileNetV2 kernels.
#pragma once

#include <hip/hip_runtime.h>

namespace rtenhip {

// Staging copy into LDS: element e (0 <= e < n) goes from ld(e) to st(e, v).
// Each thread issues U loads before any store -- unconditional, at a clamped
// index, with an empty asm use so the compiler cannot sink them into the
// guarded stores -- so a block pays one memory round trip per U elements
// per thread, not one per element.
template <int U, typename T, typename Ld, typename St>
__device__ __forceinline__ void stage_batched(int n, Ld ld, St st) {
  for (int t = threadIdx.x; t < n; t += U * (int)blockDim.x) {
    T v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = ld(min(t + u * (int)blockDim.x, n - 1));
#pragma unroll
    for (int u = 0; u < U; u++) {
      if constexpr (sizeof(T) == 16) {
        const float4 f = *reinterpret_cast<const float4*>(&v[u]);
        asm volatile("" ::"v"(f.x), "v"(f.y), "v"(f.z), "v"(f.w));
      } else {
        asm volatile("" ::"v"(v[u]));
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++)
      if (t + u * (int)blockDim.x < n) st(t + u * (int)blockDim.x, v[u]);
  }
}

}  // namespace rtenhip
