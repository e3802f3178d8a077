// HBM streaming probe (tuning aid): what write / read+write rates the
// pointwise-conv output pattern can reach on this box.
//   copy    : y[i] = x[i], float4, grid-stride
//   fill    : y[i] = c, float4 stores only
//   planes  : the pointwise-conv pattern: lane owns 4 pixels of one image,
//             reads K planes, writes M planes (plane stride P floats)
// usage: stream_probe [M K P N]   (default 96 16 12544 128 = MobileNetV2 features.2.expand)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      printf("%s failed: %s\n", #x, hipGetErrorString(e));                    \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

__global__ void copy_k(const float4* __restrict__ x, float4* __restrict__ y, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) y[i] = x[i];
}
__global__ void fill_k(float4* __restrict__ y, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    y[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}
template <int KMAX>
__global__ void planes_k(const float* __restrict__ x, float* __restrict__ y, int M, int K, int P4,
                         int groups4) {
  const int gi = blockIdx.x * 256 + threadIdx.x;
  if (gi >= groups4) return;
  const int img = gi / P4;
  const int p = (gi - img * P4) * 4;
  const long P = (long)P4 * 4;
  const float* xp = x + (long)img * K * P + p;
  float4 s = make_float4(0, 0, 0, 0);
#pragma unroll
  for (int k = 0; k < KMAX; k++) {
    if (k < K) {
      const float4 v = *(const float4*)(xp + k * P);
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
  }
  float* yp = y + (long)img * M * P + p;
  for (int o = 0; o < M; o++) {
    *(float4*)(yp + o * P) = s;
    s.x += 1.f;
  }
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 96, K = argc > 2 ? atoi(argv[2]) : 16;
  const int P = argc > 3 ? atoi(argv[3]) : 12544, N = argc > 4 ? atoi(argv[4]) : 128;
  const long nx = (long)N * K * P, ny = (long)N * M * P;
  float *x, *y;
  CK(hipMalloc(&x, nx * 4));
  CK(hipMalloc(&y, ny * 4));
  CK(hipMemset(x, 0, nx * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, double bytes, auto launch) {
    for (int i = 0; i < 3; i++) launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 10; r++) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    printf("%-28s %8.1f us  %6.2f TB/s\n", name, best * 1e3, bytes / (best * 1e-3) / 1e12);
  };
  const long n4 = ny / 4;
  for (int g : {1024, 2048, 4096, 8192}) {
    char nm[64];
    snprintf(nm, sizeof nm, "fill grid %d", g);
    timeit(nm, ny * 4.0, [&] { fill_k<<<g, 256>>>((float4*)y, n4); });
  }
  const long c4 = nx / 4;
  timeit("copy x->y (x bytes each way)", 2.0 * nx * 4, [&] { copy_k<<<4096, 256>>>((const float4*)x, (float4*)y, c4); });
  const int groups4 = (int)((long)N * P / 4);
  timeit("planes (read K, write M)", (nx + ny) * 4.0,
         [&] { planes_k<32><<<(groups4 + 255) / 256, 256>>>(x, y, M, K, P / 4, groups4); });
  CK(hipFree(x));
  CK(hipFree(y));
  return 0;
}
