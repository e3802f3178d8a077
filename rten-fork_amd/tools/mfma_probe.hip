// Micro-probe of the f32 MFMA issue rate on gfx950 (tuning aid, not product).
// Build: hipcc -O3 --offload-arch=gfx950 mfma_probe.hip -o mfma_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// CHAINS independent 32x32x2 accumulators, ITERS rounds, operands in VGPRs.
template <int CHAINS>
__global__ __launch_bounds__(256) void mfma32_loop(float* out, int iters, float a0, float b0) {
  f32x16 acc[CHAINS];
  for (int c = 0; c < CHAINS; c++) acc[c] = (f32x16){0};
  float a = a0 + threadIdx.x * 1e-7f, b = b0 - threadIdx.x * 1e-7f;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int c = 0; c < CHAINS; c++) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[c], 0, 0, 0);
  }
  float s = 0;
  for (int c = 0; c < CHAINS; c++)
    for (int j = 0; j < 16; j++) s += acc[c][j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int CHAINS>
__global__ __launch_bounds__(256) void mfma16_loop(float* out, int iters, float a0, float b0) {
  f32x4 acc[CHAINS];
  for (int c = 0; c < CHAINS; c++) acc[c] = (f32x4){0};
  float a = a0 + threadIdx.x * 1e-7f, b = b0 - threadIdx.x * 1e-7f;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int c = 0; c < CHAINS; c++) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[c], 0, 0, 0);
  }
  float s = 0;
  for (int c = 0; c < CHAINS; c++)
    for (int j = 0; j < 4; j++) s += acc[c][j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// MFMA interleaved with VALU fmas on a second value (does VALU co-issue?).
template <int CHAINS, int NVALU>
__global__ __launch_bounds__(256) void mfma32_valu(float* out, int iters, float a0, float b0) {
  f32x16 acc[CHAINS];
  for (int c = 0; c < CHAINS; c++) acc[c] = (f32x16){0};
  float a = a0 + threadIdx.x * 1e-7f, b = b0 - threadIdx.x * 1e-7f;
  float v[NVALU > 0 ? NVALU : 1];
  for (int j = 0; j < NVALU; j++) v[j] = a * (j + 1);
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int c = 0; c < CHAINS; c++) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[c], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < NVALU; j++) v[j] = __builtin_fmaf(v[j], b, a);
  }
  float s = 0;
  for (int c = 0; c < CHAINS; c++)
    for (int j = 0; j < 16; j++) s += acc[c][j];
  for (int j = 0; j < NVALU; j++) s += v[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename F>
static void run(const char* name, F launch, double flops) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  launch();
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; r++) launch();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  printf("%-40s %8.3f ms  %7.1f TFLOP/s\n", name, ms / 5, flops / (ms / 5 * 1e-3) / 1e12);
}

int main() {
  float* out;
  hipMalloc(&out, 1 << 26);
  const int iters = 4000;
  for (int blocks_per_cu : {1, 2, 4}) {
    const int grid = 256 * blocks_per_cu;
    char name[128];
    const double f32 = 2.0 * 32 * 32 * 2;
    const double f16 = 2.0 * 16 * 16 * 4;
#define RUN32(C)                                                                            \
    snprintf(name, sizeof name, "32x32x2 chains=%d blocks/CU=%d", C, blocks_per_cu);        \
    run(name, [&] { hipLaunchKernelGGL(mfma32_loop<C>, dim3(grid), dim3(256), 0, 0, out, iters, 1.f, 1.f); }, \
        f32 * C * iters * 4.0 * grid);
    RUN32(1) RUN32(2) RUN32(4)
#define RUN16(C)                                                                            \
    snprintf(name, sizeof name, "16x16x4 chains=%d blocks/CU=%d", C, blocks_per_cu);        \
    run(name, [&] { hipLaunchKernelGGL(mfma16_loop<C>, dim3(grid), dim3(256), 0, 0, out, iters, 1.f, 1.f); }, \
        f16 * C * iters * 4.0 * grid);
    RUN16(1) RUN16(2) RUN16(4)
#define RUNV(C, V)                                                                          \
    snprintf(name, sizeof name, "32x32x2 c=%d +%d VALU fma, b/CU=%d", C, V, blocks_per_cu); \
    run(name, [&] { hipLaunchKernelGGL((mfma32_valu<C, V>), dim3(grid), dim3(256), 0, 0, out, iters, 1.f, 1.f); }, \
        f32 * C * iters * 4.0 * grid);
    RUNV(2, 2) RUNV(2, 8) RUNV(2, 16)
  }
  return 0;
}
