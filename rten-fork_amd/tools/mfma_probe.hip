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

// Cross-wave co-execution: in a 512-thread block waves 0-3 run an MFMA chain
// and waves 4-7 (one per SIMD as well) run NVALU dependent-free VALU fmas per
// MFMA-equivalent step.  Time vs MFMA alone tells whether another wave's VALU
// work takes MFMA time away.
template <int NVALU>
__global__ __launch_bounds__(512) void mfma_vs_valu_waves(float* out, int iters, float a0, float b0) {
  const int wave = threadIdx.x >> 6;
  float a = a0 + threadIdx.x * 1e-7f, b = b0 - threadIdx.x * 1e-7f;
  float s = 0;
  if (wave < 4) {
    f32x16 acc = (f32x16){0};
    for (int i = 0; i < iters; i++) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    for (int j = 0; j < 16; j++) s += acc[j];
  } else {
    float v[8];
    for (int j = 0; j < 8; j++) v[j] = a * (j + 1);
    for (int i = 0; i < iters; i++)
#pragma unroll
      for (int j = 0; j < NVALU; j++) v[j & 7] = __builtin_fmaf(v[j & 7], b, a);
    for (int j = 0; j < 8; j++) s += v[j];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// Same, with the second wave per SIMD issuing NLDS ds_read_b64 per MFMA step
// (results folded with one VALU op per 8 reads so they are not dead).
template <int NLDS>
__global__ __launch_bounds__(512) void mfma_vs_lds_waves(float* out, int iters, float a0, float b0) {
  __shared__ float2 sh[4096];
  const int wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 4096; i += 512) sh[i] = make_float2(i * 1e-3f, i);
  __syncthreads();
  float a = a0 + threadIdx.x * 1e-7f, b = b0 - threadIdx.x * 1e-7f;
  float s = 0;
  if (wave < 4) {
    f32x16 acc = (f32x16){0};
    for (int i = 0; i < iters; i++) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    for (int j = 0; j < 16; j++) s += acc[j];
  } else if (NLDS > 0) {
    float2 v = make_float2(0, 0);
    int idx = threadIdx.x & 63;
    for (int i = 0; i < iters; i++) {
#pragma unroll
      for (int j = 0; j < NLDS; j++) {
        const volatile float2* pp = &sh[(idx + j * 64 + i) & 4095];
        float tx = pp->x;
        v.x += tx;
      }
    }
    s = v.x;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// One wave per SIMD: an MFMA chain with NLDS ds_read_b64 per MFMA in the same
// wave feeding the next MFMA's operand (the conv loop's pattern).
template <int CH, int NLDS>
__global__ __launch_bounds__(256) void mfma_with_lds(float* out, int iters, float a0, float b0) {
  __shared__ float sh[8192];
  for (int i = threadIdx.x; i < 8192; i += 256) sh[i] = 1e-3f * (i & 127);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  f32x16 acc[CH];
  for (int c = 0; c < CH; c++) acc[c] = (f32x16){0};
  float av[8], bv[8];
  for (int j = 0; j < 8; j++) { av[j] = sh[lane + 64 * j]; bv[j] = sh[4096 + lane + 64 * j]; }
  for (int i = 0; i < iters; i += 8) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
#pragma unroll
      for (int c = 0; c < CH; c++) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j], bv[j], acc[c], 0, 0, 0);
      if (NLDS > 0) {
        av[j] = sh[(lane + 64 * j + 8 * i) & 4095];
        bv[j] = sh[4096 + ((lane + 64 * j + 8 * i) & 4095)];
      }
    }
  }
  float s = 0;
  for (int c = 0; c < CH; c++) for (int j = 0; j < 16; j++) s += acc[c][j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// LDS read width experiment: one chain per wave, each MFMA step consumes one A
// and one B float; they are read from LDS 1 (W=1: ds_read_b32 x2 per step),
// 2 (W=2: ds_read_b64 x2 per 2 steps) or 4 (W=4: ds_read_b128 x2 per 4 steps)
// steps at a time.
template <int W>
__global__ __launch_bounds__(256) void mfma_lds_width(float* out, int iters, float a0, float b0) {
  __shared__ float sh[8192];
  for (int i = threadIdx.x; i < 8192; i += 256) sh[i] = 1e-3f * (i & 127);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  typedef float vw __attribute__((ext_vector_type(W)));
  f32x16 acc = (f32x16){0};
  vw av[2], bv[2];
  av[0] = *(const vw*)&sh[lane * W];
  bv[0] = *(const vw*)&sh[4096 + lane * W];
  for (int i = 0; i < iters; i += 2 * W) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int nx = h ^ 1;
      const int off = ((i + h * W) * 64 + lane * W) & 4095;
      av[nx] = *(const vw*)&sh[off];
      bv[nx] = *(const vw*)&sh[4096 + off];
#pragma unroll
      for (int j = 0; j < W; j++) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[h][j], bv[h][j], acc, 0, 0, 0);
    }
  }
  float s = 0;
  for (int j = 0; j < 16; j++) s += acc[j];
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
    RUNV(1, 4) RUNV(1, 8)
  }
#define RUNX(V)                                                                             \
  run("mfma wave + other wave " #V " VALU/step", [&] {                                     \
    hipLaunchKernelGGL((mfma_vs_valu_waves<V>), dim3(256), dim3(512), 0, 0, out, iters, 1.f, 1.f); \
  }, 2.0 * 32 * 32 * 2 * iters * 4.0 * 256);
  RUNX(0) RUNX(4) RUNX(8) RUNX(16) RUNX(32)
#define RUNL(V)                                                                             \
  run("mfma wave + other wave " #V " ds_read_b64/step", [&] {                              \
    hipLaunchKernelGGL((mfma_vs_lds_waves<V>), dim3(256), dim3(512), 0, 0, out, iters, 1.f, 1.f); \
  }, 2.0 * 32 * 32 * 2 * iters * 4.0 * 256);
  RUNL(0) RUNL(1) RUNL(2) RUNL(4) RUNL(8)
#define RUNW(C, V, B)                                                                       \
  run("mfma chains=" #C " + own 2 ds_read_b32 per step(" #V "), blocks/CU=" #B, [&] {      \
    hipLaunchKernelGGL((mfma_with_lds<C, V>), dim3(256 * B), dim3(256), 0, 0, out, iters, 1.f, 1.f); \
  }, 2.0 * 32 * 32 * 2 * iters * 4.0 * 256 * B * C);
#define RUNLW(W, B)                                                                         \
  run("1 chain, LDS reads " #W " floats wide, blocks/CU=" #B, [&] {                        \
    hipLaunchKernelGGL((mfma_lds_width<W>), dim3(256 * B), dim3(256), 0, 0, out, iters, 1.f, 1.f); \
  }, 2.0 * 32 * 32 * 2 * iters * 4.0 * 256 * B);
  RUNLW(1, 1) RUNLW(2, 1) RUNLW(4, 1) RUNLW(1, 3) RUNLW(2, 3) RUNLW(4, 3) RUNLW(1, 4) RUNLW(4, 4)
  RUNW(1, 0, 1) RUNW(1, 1, 1) RUNW(1, 0, 3) RUNW(1, 1, 3) RUNW(2, 1, 2) RUNW(4, 1, 1) RUNW(4, 1, 2)
  return 0;
}
