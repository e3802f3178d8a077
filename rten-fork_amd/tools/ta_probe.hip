// Vector-memory throughput probe (tuning aid for the batch-1 latency GEMM):
// every wave streams ITERS x 16 dwordx4 / dword loads from its own slot of a
// buffer; reports bytes per CU per microsecond.  argv: waves_per_cu,
// slot stride in floats, slots (distinct slots, round-robin over waves).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int P>
__global__ __launch_bounds__(256) void probe(const float* __restrict__ buf, int iters, long stride, int slots,
                                             float* out) {
  const int lane = threadIdx.x & 63;
  const int w = (blockIdx.x * 4 + (threadIdx.x >> 6)) % slots;
  const float* base = buf + (size_t)w * stride;
  float acc = 0.f;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < 16; j++) {
      if (P == 0) {
        const float4 v = *(const float4*)(base + (it % 4) * 4096 + j * 256 + lane * 4);
        acc += (v.x + v.y) + (v.z + v.w);
      } else if (P == 1) {
        acc += base[(it % 16) * 1024 + j * 64 + lane];
      } else {
        acc += base[(it % 16) * 1024 + j * 16 + (lane & 15) + (lane >> 4) * 3136];
      }
    }
  }
  if (acc == 1234.5f) out[0] = acc;
}

int main(int argc, char** argv) {
  const int waves_per_cu = argc > 1 ? atoi(argv[1]) : 8;
  const long stride = argc > 2 ? atol(argv[2]) : 16384;
  const int slots = argc > 3 ? atoi(argv[3]) : 2048;
  const int iters = 64;
  const size_t n = (size_t)slots * stride + 16384 + 4 * 3136 + 64;
  float* buf;
  float* out;
  hipMalloc(&buf, n * 4);
  hipMemset(buf, 0, n * 4);
  hipMalloc(&out, 4);
  const int blocks = 256 * waves_per_cu / 4;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"dwordx4 contiguous (16KB/it)", "dword contiguous (4KB/it)", "dword lat-gather (4 rows)"};
  const int bytes[] = {1024, 256, 256};
  for (int p = 0; p < 3; p++) {
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(e0);
      if (p == 0) probe<0><<<blocks, 256>>>(buf, iters, stride, slots, out);
      else if (p == 1) probe<1><<<blocks, 256>>>(buf, iters, stride, slots, out);
      else probe<2><<<blocks, 256>>>(buf, iters, stride, slots, out);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep) {
        const double instr_per_cu = (double)waves_per_cu * iters * 16;
        const double us = ms * 1e3;
        printf("%-30s w/CU %2d stride %6ld slots %5d: %7.1f us, %5.1f ns/instr/CU, %6.1f GB/s/CU\n", names[p],
               waves_per_cu, stride, slots, us, us * 1e3 / instr_per_cu, instr_per_cu * bytes[p] / us / 1e3);
      }
    }
  }
  return 0;
}
