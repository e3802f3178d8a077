// Probe: v_mfma_f32_4x4x1_16b_f32 operand / result layout and whether a chain
// of them is bitwise the k-ordered fmaf chain (for an MFMA stem with 4
// output channels per block).  Hypothesis H1: A lane l = (block l/4, row l%4),
// B lane l = (block l/4, col l%4), D reg r of lane l = (block l/4, row r,
// col l%4).  H2: D reg r of lane l = (block l/4, row l%4, col r).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int K = 27;
__global__ void probe(const float* a, const float* b, float* d) {
  const int l = threadIdx.x;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < K; k++) acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a[k * 64 + l], b[k * 64 + l], acc, 0, 0, 0);
  for (int r = 0; r < 4; r++) d[l * 4 + r] = acc[r];
}
int main() {
  float ha[K * 64], hb[K * 64], hd[256];
  srand(7);
  for (int i = 0; i < K * 64; i++) {
    ha[i] = (float)rand() / RAND_MAX * 2.f - 1.f;
    hb[i] = ((float)rand() / RAND_MAX * 2.f - 1.f) * (i % 7 == 0 ? 1e-3f : 1.f);
  }
  float *da, *db, *dd;
  hipMalloc(&da, sizeof ha); hipMalloc(&db, sizeof hb); hipMalloc(&dd, sizeof hd);
  hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
  hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, da, db, dd);
  hipMemcpy(hd, dd, sizeof hd, hipMemcpyDeviceToHost);
  int bad1 = 0, bad2 = 0, near1 = 0;
  for (int l = 0; l < 64; l++)
    for (int r = 0; r < 4; r++) {
      const int blk = l / 4;
      // H1: row r, col l%4 -> A lane (blk, r), B lane (blk, l%4)
      float e1 = 0.f, e2 = 0.f;
      for (int k = 0; k < K; k++) {
        e1 = fmaf(ha[k * 64 + blk * 4 + r], hb[k * 64 + blk * 4 + (l % 4)], e1);
        e2 = fmaf(ha[k * 64 + blk * 4 + (l % 4)], hb[k * 64 + blk * 4 + r], e2);
      }
      uint32_t g, x1, x2;
      memcpy(&g, &hd[l * 4 + r], 4); memcpy(&x1, &e1, 4); memcpy(&x2, &e2, 4);
      bad1 += g != x1; bad2 += g != x2;
      near1 += fabsf(hd[l * 4 + r] - e1) < 1e-4f;
    }
  printf("H1 (D reg r = row r, lane col) mismatches %d / 256 (near %d); H2 mismatches %d / 256\n", bad1, near1, bad2);
  return 0;
}
