// Probe (tuning aid, not product): is v_mfma_f32_16x16x4_f32 bitwise the
// k-ordered fmaf chain that v_mfma_f32_32x32x2_f32 is, and what FLOP/s do the
// two shapes sustain on RANDOM operands (the clock the chip holds depends on
// operand toggling, MI355X_MICROARCH.md "DVFS give-back")?
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off mfma_shape_probe.hip -o mfma_shape_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// One wave: D = A[16x4] B[4x16] + C via 16x16x4 (block 0 of the instruction).
// Operand layout (cdna_hip_programming.md §3): lane l supplies A[l%16][l/16]
// and B[l/16][l%16]; accumulator element j of lane l is row 4*(l/16)+j, col l%16.
__global__ void one16(const float* A, const float* B, const float* C, float* D) {
  const int l = threadIdx.x;
  const float a = A[(l % 16) * 4 + l / 16];
  const float b = B[(l / 16) * 16 + l % 16];
  f32x4 c;
  for (int j = 0; j < 4; j++) c[j] = C[(4 * (l / 16) + j) * 16 + l % 16];
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  for (int j = 0; j < 4; j++) D[(4 * (l / 16) + j) * 16 + l % 16] = c[j];
}

// One wave: D = A[32x2] B[2x32] + C via 32x32x2.  lane l supplies A[l%32][l/32],
// B[l/32][l%32]; element j of lane l is row (j&3) + 8*(j>>2) + 4*(l/32), col l%32.
__global__ void one32(const float* A, const float* B, const float* C, float* D) {
  const int l = threadIdx.x;
  const float a = A[(l % 32) * 2 + l / 32];
  const float b = B[(l / 32) * 32 + l % 32];
  f32x16 c;
  for (int j = 0; j < 16; j++) c[j] = C[((j & 3) + 8 * (j >> 2) + 4 * (l / 32)) * 32 + l % 32];
  c = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  for (int j = 0; j < 16; j++) D[((j & 3) + 8 * (j >> 2) + 4 * (l / 32)) * 32 + l % 32] = c[j];
}

// Throughput on random operands: each lane cycles through 16 random A and B
// values held in registers, CH independent accumulators.
template <int CH>
__global__ __launch_bounds__(256) void loop32(const float* rnd, float* out, int iters) {
  float a[16], b[16];
  for (int j = 0; j < 16; j++) {
    a[j] = rnd[(threadIdx.x * 37 + j * 11 + blockIdx.x) & 4095];
    b[j] = rnd[(threadIdx.x * 53 + j * 7 + blockIdx.x * 3) & 4095];
  }
  f32x16 acc[CH];
  for (int c = 0; c < CH; c++) acc[c] = (f32x16){0};
  for (int i = 0; i < iters; i++)
#pragma unroll
    for (int j = 0; j < 16; j++)
#pragma unroll
      for (int c = 0; c < CH; c++) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j], b[(j + c) & 15], acc[c], 0, 0, 0);
  float s = 0;
  for (int c = 0; c < CH; c++)
    for (int j = 0; j < 16; j++) s += acc[c][j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int CH>
__global__ __launch_bounds__(256) void loop16(const float* rnd, float* out, int iters) {
  float a[16], b[16];
  for (int j = 0; j < 16; j++) {
    a[j] = rnd[(threadIdx.x * 37 + j * 11 + blockIdx.x) & 4095];
    b[j] = rnd[(threadIdx.x * 53 + j * 7 + blockIdx.x * 3) & 4095];
  }
  f32x4 acc[CH];
  for (int c = 0; c < CH; c++) acc[c] = (f32x4){0};
  for (int i = 0; i < iters; i++)
#pragma unroll
    for (int j = 0; j < 16; j++)
#pragma unroll
      for (int c = 0; c < CH; c++) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[(j + c) & 15], acc[c], 0, 0, 0);
  float s = 0;
  for (int c = 0; c < CH; c++)
    for (int j = 0; j < 4; j++) s += acc[c][j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static uint32_t rng_state = 12345;
static float frand() {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 17;
  rng_state ^= rng_state << 5;
  return ((rng_state >> 8) * (1.0f / 16777216.0f)) * 2.f - 1.f;
}

template <typename F>
static double timeit(F launch) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int r = 0; r < 20; r++) launch();  // >= 1 s of warm load for the clock
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 10; r++) launch();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 10;
}

int main() {
  float *dA, *dB, *dC, *dD;
  hipMalloc(&dA, 4096 * 4);
  hipMalloc(&dB, 4096 * 4);
  hipMalloc(&dC, 4096 * 4);
  hipMalloc(&dD, 4096 * 4);
  std::vector<float> A(64), B(64), C(256), D(1024);
  // --- bit-exactness of 16x16x4 vs the fmaf chain k = 0..3 (and 3..0, and a
  //     single-rounding dot product), over many random trials incl. cancellation.
  long mism_fwd = 0, mism_rev = 0, mism_dot = 0, total = 0;
  for (int t = 0; t < 200; t++) {
    for (auto& v : A) v = frand() * (t % 3 == 0 ? 1e3f : 1.f);
    for (auto& v : B) v = frand();
    for (auto& v : C) v = frand() * (t % 2 ? 1e-3f : 10.f);
    hipMemcpy(dA, A.data(), 64 * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), 64 * 4, hipMemcpyHostToDevice);
    hipMemcpy(dC, C.data(), 256 * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(one16, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD);
    hipMemcpy(D.data(), dD, 256 * 4, hipMemcpyDeviceToHost);
    for (int i = 0; i < 16; i++)
      for (int j = 0; j < 16; j++) {
        float f = C[i * 16 + j], r = C[i * 16 + j];
        for (int k = 0; k < 4; k++) f = std::fmaf(A[i * 4 + k], B[k * 16 + j], f);
        for (int k = 3; k >= 0; k--) r = std::fmaf(A[i * 4 + k], B[k * 16 + j], r);
        double dd = C[i * 16 + j];
        for (int k = 0; k < 4; k++) dd += (double)A[i * 4 + k] * B[k * 16 + j];
        const float dot = (float)dd;
        uint32_t g, e1, e2, e3;
        memcpy(&g, &D[i * 16 + j], 4);
        memcpy(&e1, &f, 4);
        memcpy(&e2, &r, 4);
        memcpy(&e3, &dot, 4);
        mism_fwd += g != e1;
        mism_rev += g != e2;
        mism_dot += g != e3;
        total++;
      }
  }
  printf("16x16x4: %ld elements; mismatches vs fmaf chain k=0..3: %ld, k=3..0: %ld, one-rounding dot: %ld\n",
         total, mism_fwd, mism_rev, mism_dot);
  // --- same for 32x32x2
  mism_fwd = mism_rev = total = 0;
  for (int t = 0; t < 100; t++) {
    for (auto& v : A) v = frand() * (t % 3 == 0 ? 1e3f : 1.f);
    for (auto& v : B) v = frand();
    std::vector<float> C32(1024);
    for (auto& v : C32) v = frand() * (t % 2 ? 1e-3f : 10.f);
    hipMemcpy(dA, A.data(), 64 * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), 64 * 4, hipMemcpyHostToDevice);
    hipMemcpy(dC, C32.data(), 1024 * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(one32, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD);
    hipMemcpy(D.data(), dD, 1024 * 4, hipMemcpyDeviceToHost);
    for (int i = 0; i < 32; i++)
      for (int j = 0; j < 32; j++) {
        float f = C32[i * 32 + j], r = C32[i * 32 + j];
        for (int k = 0; k < 2; k++) f = std::fmaf(A[i * 2 + k], B[k * 32 + j], f);
        for (int k = 1; k >= 0; k--) r = std::fmaf(A[i * 2 + k], B[k * 32 + j], r);
        uint32_t g, e1, e2;
        memcpy(&g, &D[i * 32 + j], 4);
        memcpy(&e1, &f, 4);
        memcpy(&e2, &r, 4);
        mism_fwd += g != e1;
        mism_rev += g != e2;
        total++;
      }
  }
  printf("32x32x2: %ld elements; mismatches vs fmaf chain k=0..1: %ld, k=1..0: %ld\n", total, mism_fwd,
         mism_rev);

  // --- throughput on random operands
  std::vector<float> R(4096);
  for (auto& v : R) v = frand();
  float* dR;
  hipMalloc(&dR, 4096 * 4);
  hipMemcpy(dR, R.data(), 4096 * 4, hipMemcpyHostToDevice);
  float* out;
  hipMalloc(&out, 1 << 24);
  const int iters = 400;
  for (int bpc : {1, 2}) {
    const int grid = 256 * bpc;
    double ms;
    ms = timeit([&] { hipLaunchKernelGGL(loop32<2>, dim3(grid), dim3(256), 0, 0, dR, out, iters); });
    printf("32x32x2 random, 2 chains, %d blk/CU: %.3f ms %.1f TFLOP/s\n", bpc, ms,
           2.0 * 32 * 32 * 2 * 16 * 2 * iters * 4.0 * grid / (ms * 1e-3) / 1e12);
    ms = timeit([&] { hipLaunchKernelGGL(loop16<4>, dim3(grid), dim3(256), 0, 0, dR, out, iters); });
    printf("16x16x4 random, 4 chains, %d blk/CU: %.3f ms %.1f TFLOP/s\n", bpc, ms,
           2.0 * 16 * 16 * 4 * 16 * 4 * iters * 4.0 * grid / (ms * 1e-3) / 1e12);
    ms = timeit([&] { hipLaunchKernelGGL(loop16<8>, dim3(grid), dim3(256), 0, 0, dR, out, iters); });
    printf("16x16x4 random, 8 chains, %d blk/CU: %.3f ms %.1f TFLOP/s\n", bpc, ms,
           2.0 * 16 * 16 * 4 * 16 * 8 * iters * 4.0 * grid / (ms * 1e-3) / 1e12);
  }
  return 0;
}
