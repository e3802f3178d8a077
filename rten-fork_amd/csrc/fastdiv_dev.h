// Device side of FastDiv (common.h): n / d for 0 <= n < 2^31.
#pragma once

#include "common.h"

namespace rtenhip {

__device__ __forceinline__ int fdiv(int n, FastDiv f) {
  return (int)(((uint64_t)(uint32_t)n * f.mul) >> f.shift);
}

}  // namespace rtenhip
