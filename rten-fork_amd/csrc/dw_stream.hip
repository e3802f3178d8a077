// Streaming depthwise 3x3 for small planes (MobileNetV2's 14x14 and 7x7
// stages, and the 14 -> 7 stride-2 layer): HBM-bound layers where the
// whole-plane LDS kernel (pool.hip depthwise_lds_kernel) runs one staging
// round trip per block and leaves the memory pipe idle while it computes.
//
// Persistent blocks, each owning one chunk of PB consecutive channels and
// walking the batch: group i of a block is image n0 + i*step, channels
// chunk*PB .. chunk*PB + PB - 1 -- PB whole planes, one contiguous range of
// the input and of the output.  Groups are copied into an NBUF-deep LDS ring
// by LDS DMA (buffer_load_dwordx4 ... lds, no VGPR round trip), NBUF - 1
// groups ahead of the one being computed, so the copies of later groups are
// in flight while a group computes and stores.  A thread owns one output row
// of one plane of the chunk, so its channel -- weights and bias in registers
// -- is fixed for the whole kernel.
//
// Arithmetic: depthwise_lds_kernel's (conv_2d_depthwise_block,
// src/ops/conv/depthwise.rs:49-203): per output the bias, then + v * w over
// the taps in (ky, kx) order, each product and sum rounded, taps outside the
// image skipped (a row outside the image by a select of the unchanged sum,
// columns at compile time), then the activation.
//
// Waits: the DMAs are inline asm (invisible to the compiler's waitcnt pass),
// the stores are raw buffer stores with a fixed count per wave and group
// (idle lanes store to an out-of-range offset, which the hardware drops), and
// vmcnt retires in issue order, so the wait for group i's copies is a
// compile-time count of the younger operations: see wait_group.
#include "common.h"
#include "vecmath.h"

namespace rtenhip {

namespace {

typedef uint32_t dws_u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t dws_u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ dws_u32x4 dws_rsrc(const void* base, uint32_t num_records) {
  const uint64_t a = (uint64_t)base;
  return (dws_u32x4){(uint32_t)a, (uint32_t)(a >> 32) & 0xffffu, num_records, 0x00020000u};
}

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void dws_dma16(dws_u32x4 r, uint32_t lds_dst, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               ::"s"(__builtin_amdgcn_readfirstlane(lds_dst)), "v"(voff), "s"(r)
               : "memory", "m0");
}
#pragma clang diagnostic pop

constexpr uint32_t DWS_OOB = 0x80000000u;
constexpr int DWS_NT = 256, DWS_NW = DWS_NT / 64;

template <int H, int S>
struct DwsShape {
  static constexpr int W = H;
  static constexpr int OH = (H + 2 - 3) / S + 1;  // pads 1, kernel 3
  static constexpr int OW = OH;
};

struct DwsDesc {
  const float* x;
  const float* w;
  const float* bias;
  float* y;
  int N, C;
  int nch;    // C / PB
  int step;   // images between a block's consecutive groups (gridDim.x / nch)
  int act;
  float lo, hi;
};

// NSEG: output row segments per row (a thread owns SEG = OW / NSEG outputs).
template <int H, int S, int PB, int NSEG, int NBUF>
__global__ __launch_bounds__(DWS_NT) void dw_stream_kernel(DwsDesc d) {
  using Sh = DwsShape<H, S>;
  constexpr int W = Sh::W, OH = Sh::OH, OW = Sh::OW;
  constexpr int HW = H * W, OHW = OH * OW;
  constexpr int GF = PB * HW;                        // floats per group (input)
  constexpr int NI = (GF + 255) / 256;               // 1 KB DMA instructions per group
  constexpr int NDMA = (NI + DWS_NW - 1) / DWS_NW;   // per wave
  constexpr int BUF = NDMA * DWS_NW * 256;           // floats per ring slot
  constexpr int GO4 = PB * OHW / 4;                  // output float4s per group
  constexpr int NST = (GO4 + DWS_NT - 1) / DWS_NT;   // 16-byte stores per lane and group
  static_assert(OW % NSEG == 0 && PB * OH * NSEG <= DWS_NT, "one row segment per thread");
  static_assert(NSEG == 1 || S == 1, "segmented rows at stride 1");
  constexpr int SEG = OW / NSEG;
  constexpr int WC = (SEG - 1) * S + 3;  // input columns of a segment's window
  static_assert(NBUF == 3, "wait counts below assume a ring of 3");
  static_assert((GF * 4) % 16 == 0 && (PB * OHW) % 4 == 0, "whole float4s per group");
  static_assert(PB * OHW <= BUF, "outputs staged in the slot");
  __shared__ float ring[NBUF * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int chunk = blockIdx.x % d.nch;
  const int n0 = blockIdx.x / d.nch;
  const int ng = n0 < d.N ? (d.N - n0 + d.step - 1) / d.step : 0;
  const int pp = tid / (OH * NSEG), rem = tid - pp * (OH * NSEG);
  const int oy = rem / NSEG, sg = rem - oy * NSEG;
  const bool active = pp < PB;
  const int c = chunk * PB + (active ? pp : 0);

  auto group_in = [&](int i) {
    const int n = n0 + i * d.step;
    return d.x + ((int64_t)n * d.C + (int64_t)chunk * PB) * HW;
  };
  // Wave `wave` copies instructions q = j * NW + wave of the group's GF floats
  // into ring slot `slot`; lanes past the group read out of range (0, and land
  // in the slot's padding).
  auto issue = [&](int i, int slot) __attribute__((always_inline)) {
    const dws_u32x4 r = dws_rsrc(group_in(i), (uint32_t)(GF * 4));
    const uint32_t base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)ring +
                          (uint32_t)(slot * BUF * 4);
#pragma unroll
    for (int j = 0; j < NDMA; j++) {
      const int q = j * DWS_NW + wave;
      const int f = q * 256 + lane * 4;
      dws_dma16(r, base + (uint32_t)(q * 1024), f < GF ? (uint32_t)(f * 4) : DWS_OOB);
    }
  };
  // Group i's copies are complete once at most the operations issued after
  // them are outstanding (vmcnt retires in order): for i >= 2 the stores of
  // groups i-2 and i-1 and, unless i is the last, group i+1's copies; i = 1
  // and i = 0 have fewer predecessors in the stream (see the loop order).
  auto wait_group = [&](int i) __attribute__((always_inline)) {
    const bool next = i + 1 < ng;
    if (i >= 2) {
      if (next) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NST + NDMA) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NST) : "memory");
    } else if (i == 1) {
      if (next) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST + NDMA) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST) : "memory");
    } else {
      if (next) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NDMA) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  };

  if (ng > 0) issue(0, 0);
  if (ng > 1) issue(1, 1);
  // Weights and bias (compiler-tracked loads, issued after the first two
  // groups' copies: their wait before the first use also covers those).
  float wk[9];
#pragma unroll
  for (int t = 0; t < 9; t++) wk[t] = d.w[c * 9 + t];
  const float b0 = d.bias ? d.bias[c] : 0.f;
  const int act = d.act;
  const float lo = d.lo, hi = d.hi;

  // Rows of this thread's window: input rows oy*S - 1 + ky; row ky = 0 is
  // outside the image for oy = 0, row 2 past the bottom for stride 1's last
  // output row (stride 2 on an even H never reaches past it).
  const bool row0_ok = oy > 0;
  const bool row2_ok = oy * S + 1 < H;
  const int iy0 = row0_ok ? oy * S - 1 : 0;
  const int iy2 = row2_ok ? oy * S + 1 : 0;
  // Window columns ix = x0 + j, j < WC; only the first and the last can fall
  // outside the image (compile-time with whole rows, per segment otherwise).
  const int x0 = sg * SEG * S - 1;
  const bool colL_ok = x0 >= 0;
  const bool colR_ok = x0 + WC - 1 < W;

  for (int i = 0; i < ng; i++) {
    const int slot = i % NBUF;
    wait_group(i);
    __builtin_amdgcn_s_barrier();  // every wave's copies landed; slot (i+2)%3 read by no one
    asm volatile("" ::: "memory");  // no LDS read moves above the barrier
    if (i + 2 < ng) issue(i + 2, (i + 2) % NBUF);
    const float* tp = ring + slot * BUF + (active ? pp : 0) * HW;
    float rw[3][WC];
#pragma unroll
    for (int j = 0; j < WC; j++) {
      const int ix = NSEG == 1 ? min(max(j - 1, 0), W - 1) : min(max(x0 + j, 0), W - 1);
      rw[0][j] = tp[iy0 * W + ix];
      rw[1][j] = tp[oy * S * W + ix];
      rw[2][j] = tp[iy2 * W + ix];
    }
    float out[SEG];
#pragma unroll
    for (int ox = 0; ox < SEG; ox++) {
      float acc = b0;
#pragma unroll
      for (int ky = 0; ky < 3; ky++) {
        float t = acc;
#pragma unroll
        for (int kx = 0; kx < 3; kx++) {
          const int j = ox * S + kx;
          const float v = __fadd_rn(t, __fmul_rn(rw[ky][j], wk[ky * 3 + kx]));
          if constexpr (NSEG == 1) {
            if (j - 1 >= 0 && j - 1 < W) t = v;  // whole rows: x0 = -1
          } else if (j == 0) {
            t = colL_ok ? v : t;
          } else if (j == WC - 1) {
            t = colR_ok ? v : t;
          } else {
            t = v;
          }
        }
        acc = ky == 0 ? (row0_ok ? t : acc) : ky == 2 ? (row2_ok ? t : acc) : t;
      }
      if (act == RTENHIP_ACT_RELU) acc = rust_max(acc, 0.f);
      else if (act == RTENHIP_ACT_CLIP) acc = rust_clamp(acc, lo, hi);
      out[ox] = acc;
    }
    // The group's outputs are one contiguous range (planes of OH x OW): they
    // go through the slot just read (every wave done with it first) and out
    // as 16-byte stores, 1 KB per wave instruction.
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    float* op = ring + slot * BUF;
    if (active) {
#pragma unroll
      for (int ox = 0; ox < SEG; ox++) op[pp * OHW + oy * OW + sg * SEG + ox] = out[ox];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int n = n0 + i * d.step;
    const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(
        d.y + ((int64_t)n * d.C + (int64_t)chunk * PB) * OHW, 0, PB * OHW * 4, 0x00020000);
#pragma unroll
    for (int j = 0; j < NST; j++) {
      const int f4 = j * DWS_NT + tid;
      const float4 v = *reinterpret_cast<const float4*>(op + 4 * (f4 < GO4 ? f4 : 0));
      const dws_u32x4 u = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
      __builtin_amdgcn_raw_buffer_store_b128(u, yr, f4 < GO4 ? 16 * f4 : (int)DWS_OOB, 0, 0);
    }
  }
}

long long g_dws_launches = 0;  // host-side count (tests: the kernel ran, not the fallback)

template <int H, int S, int PB, int NSEG>
bool launch_dws(const float* x, const float* w, const float* bias, float* y, int N, int C, int act, float lo,
                float hi, hipStream_t s, rtenhip_status& st) {
  if (C % PB != 0) return false;
  auto kern = dw_stream_kernel<H, S, PB, NSEG, 3>;
  static int cus = 0, occ = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, DWS_NT, 0) != hipSuccess || occ <= 0) occ = 1;
  }
  DwsDesc d{x, w, bias, y, N, C, C / PB, 0, act, lo, hi};
  // Blocks: a multiple of the chunk count (every block keeps one chunk),
  // at most one resident wave of blocks, and no more images per chunk than
  // the batch holds.
  int per_chunk = std::max(1, (cus * occ) / d.nch);
  per_chunk = std::min(per_chunk, N);
  // Equal group counts per block: the fewest images per chunk column that
  // still gives every block ceil(N / per_chunk) groups.
  const int groups_per_block = (N + per_chunk - 1) / per_chunk;
  per_chunk = (N + groups_per_block - 1) / groups_per_block;
  d.step = per_chunk;
  const int grid = d.nch * per_chunk;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(DWS_NT), 0, s, d);
  const hipError_t e = hipGetLastError();
  st = e == hipSuccess ? RTENHIP_OK : hip_fail(e, "dw_stream_kernel launch");
  g_dws_launches++;
  return true;
}

}  // namespace

// Streaming depthwise for 3x3 / pads 1 / dilation 1 on square 14x14 (stride 1
// or 2) and 7x7 (stride 1) planes without a residual; false when the shape is
// not one of those (the caller runs depthwise_lds_kernel).  RTENHIP_DW_STREAM=0
// disables it (A/B experiments).
bool launch_depthwise_stream(const float* x, const float* w, const float* bias, float* y, int N, int C, int H,
                             int W, int OH, int OW, int kh, int kw, int sh, int sw, int dh, int dw, int pt, int pl,
                             const int* omin, const int* omax, const float* residual, int act, float lo, float hi,
                             hipStream_t s, rtenhip_status& st) {
  static const bool on = [] {
    const char* e = getenv("RTENHIP_DW_STREAM");
    return !(e && atoi(e) == 0);
  }();
  if (!on || residual || kh != 3 || kw != 3 || dh != 1 || dw != 1 || sh != sw || pt != 1 || pl != 1 || H != W ||
      N <= 0 || C <= 0)
    return false;
  static const bool dws28 = [] {
    const char* e = getenv("RTENHIP_DW_STREAM28");  // A/B: 0 leaves 28x28 to depthwise_lds4_kernel
    return !(e && atoi(e) == 0);
  }();
  const int S = sh, OE = (H + 2 - 3) / S + 1;
  if (OH != OE || OW != OE) return false;
  // The kernel skips exactly the columns outside the image; the caller's
  // x-range bounds (the reference's min/max_out_x) must say the same.
  for (int kx = 0; kx < 3; kx++) {
    int lo_x = 0, hi_x = 0;
    while (lo_x < OW && lo_x * S - 1 + kx < 0) lo_x++;
    while (hi_x < OW && hi_x * S - 1 + kx < W) hi_x++;
    if (omin[kx] != lo_x || omax[kx] != hi_x) return false;
  }
  if ((uintptr_t)x % 16 != 0 || (uintptr_t)y % 16 != 0) return false;
  if ((int64_t)N * C * H * W >= (int64_t(1) << 29)) return false;
  if (H == 14 && S == 1) return launch_dws<14, 1, 16, 1>(x, w, bias, y, N, C, act, lo, hi, s, st);
  if (H == 7 && S == 1) return launch_dws<7, 1, 32, 1>(x, w, bias, y, N, C, act, lo, hi, s, st);
  if (H == 14 && S == 2) return launch_dws<14, 2, 16, 1>(x, w, bias, y, N, C, act, lo, hi, s, st);
  if (H == 28 && S == 1 && dws28) return launch_dws<28, 1, 4, 2>(x, w, bias, y, N, C, act, lo, hi, s, st);
  return false;
}

}  // namespace rtenhip

extern "C" long long rtenhip_debug_dw_stream_launches() { return rtenhip::g_dws_launches; }
