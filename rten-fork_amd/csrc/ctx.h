// Context object behind rtenhip_ctx.
#pragma once

#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <tuple>

#include "common.h"
#include "gemm_dma.h"

namespace rtenhip {

struct Ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  // The graphs' executor stream (Graph::run), one per context and shared by
  // its graphs: a process gets few hardware queues (GPU_MAX_HW_QUEUES, 4 by
  // default), and streams beyond that share them, serialising copies or
  // kernels queued behind another graph's work.
  hipStream_t exec_stream = nullptr;
  // exec_stream was created by the library (else the caller's, set through
  // rtenhip_set_exec_stream, and not destroyed here).
  bool owns_exec = false;
  // Thread count RTen would run with (RTEN_NUM_THREADS semantics,
  // src/threading.rs:41-62).  It only changes numerics in the gemv path,
  // where the reference's column blocking depends on it (gemm.rs:673).
  int ref_threads = 0;
  std::mutex mu;
  std::map<std::tuple<int, int, int, int, int, int, int>, int2*> ktabs;
  std::map<std::tuple<int, int, int, int, int, int, int>, int*> dtabs;
  static constexpr int NSLOTS = 6;
  void* slots[NSLOTS] = {};
  size_t slot_cap[NSLOTS] = {};
  bool use_dma = true;
  // Packed-weight cache keyed by (weights pointer, M, K, bm, bk, il).  Only valid
  // when the caller guarantees weights are immutable (graph constants); the
  // public per-op API packs on every call unless a tuning tool opts in.
  bool trust_weight_cache = false;
  std::map<std::tuple<const void*, int64_t, int64_t, int, int, int>, float*> packed_cache;

  explicit Ctx(int dev);
  ~Ctx();
  // Grow-only device scratch (independent slots: 0 contiguous copies,
  // 1 softmax / padded inputs, 2 packed weights, 3 split workspaces, 4 and 5
  // the unfused attention sequence's scores and output).  Synchronizes the
  // stream when it has to grow, so callers must not be capturing.
  float* scratch_floats(size_t n, size_t slot);
  // Grow-only zeroed int buffer for DMA split arrival counters (the kernel
  // leaves them zero).  Synchronizes when it grows, like scratch_floats.
  int* split_counters(size_t n);
  int* counters = nullptr;
  size_t counters_cap = 0;
  // Bumped whenever scratch_floats / split_counters reallocate: a captured
  // hipGraph that baked in an older scratch pointer must be re-captured
  // (Graph::run compares it with the generation stored at capture).
  uint64_t scratch_gen = 0;
  // While set, every scratch request is recorded as (slot -> max floats);
  // slot NSLOTS stands for the split counters.  Graph::run records a plan's
  // needs during its eager runs and reserves them before capturing, so no
  // scratch buffer grows (and synchronizes) inside a capture.
  std::map<size_t, size_t>* scratch_log = nullptr;
  // Grow scratch slots (and the split counters) to the recorded needs.
  // Returns false on an allocation failure.
  bool reserve_scratch(const std::map<size_t, size_t>& need);
  // Device table of VirtualIm2Col row offsets for one conv geometry.
  const int2* ktab(int C, int H, int W, int kh, int kw, int dh, int dw);
  // Device table of per-k input offsets c*H*W + ky*dh*W + kx*dw (DMA GEMM).
  const int* dtab(int C, int H, int W, int kh, int kw, int dh, int dw);
};

// Conv through the DMA GEMM with caller-managed inputs: xin is the (padded)
// input [N, C, Hp, Wp]; packed_w the weights packed for (bm, bk) per group.
struct ConvDmaArgs {
  const float* xin;
  int64_t N, C, Hp, Wp, O, kh, kw, sh, sw, dh, dw, oh, ow, groups;
  const float* packed_w;  // groups * packed_a_floats(opg, K)
  const float* bias;
  const float* bn;  // fused BatchNormalization: [3][bn_c] mean, scale / sqrt(var + eps), beta (DmaDesc::bn)
  int64_t bn_c;
  const float* residual;
  int act;
  float lo, hi;
  float* y;
  int64_t y_img, y_row, y_off;  // output addressing (padded outputs allowed)
  int cfg;                      // DMA kernel configuration, -1 = default
  // KC split of the remainder tiles (dma_split_plan): enabled when split is
  // set and the caller's workspace / zeroed counters are large enough.
  bool split;
  float* ws;
  int64_t ws_cap;
  int* counters;
  int64_t cnt_cap;
  int persist_k;  // persistent launch: resident blocks per CU (0: one block per item)
  // The unpadded input and its geometry (direct VALU conv: padding in place).
  const float* x_unpadded;
  int64_t H, W, pad_t, pad_l;
};
rtenhip_status conv_dma(Ctx* c, const ConvDmaArgs& a);
// Two ungrouped 1x1 latency-GEMM convs (cfg = kLatCfgBase + 71 / 72 / 74, packed
// weights and K-block workspaces bound) in one launch; a0 pointwise stride 1.
bool conv_lat_pair_ok(const ConvDmaArgs& a0, const ConvDmaArgs& a1);
rtenhip_status conv_lat_pair(Ctx* c, const ConvDmaArgs& a0, const ConvDmaArgs& a1);
// conv3 + downsample as one dual DMA GEMM (see capi.cpp); cfg = a3.cfg, both
// packed for it.
bool conv_dual_ok(const ConvDmaArgs& a3, const ConvDmaArgs& ad, int cfg);
rtenhip_status conv_dma_dual(Ctx* c, const ConvDmaArgs& a3, const ConvDmaArgs& ad);

// Pointwise convs on the vector ALUs (conv_pointwise.hip): 1x1 / stride 1 /
// unpadded / ungrouped, K <= 256, P % 4 == 0, unpadded output; mc = output
// channels per pass (8, 16 or 32).  Weights transposed to [K][M rounded to 32].
struct ConvPlan;
bool conv_pw_valu_eligible(const ConvPlan& g, int64_t Hp, int64_t Wp, bool padded_out);
int64_t pw_weight_floats(int64_t M, int64_t K);
rtenhip_status pack_pw_weights(const float* w, int64_t M, int64_t K, float* wt, hipStream_t s);
// variant = mc + 100 * (KX / 16): mc in {8, 16, 32} output channels per pass;
// KX = 0 streams x per pass, KX = 16 / 32 holds a K <= KX column in VGPRs.
bool pw_variant_ok(int variant, int64_t K);
// Direct VALU conv (3-wide kernels, stride 1 or 2, K = C*kh*kw <= 64, OW % 4 == 0,
// unpadded output), variant kPwDirect + mc, mc in {16, 32}; mc + 100 stages
// the block's input rows in LDS (kh <= 3, dh = 1, sh = sw, pad_l <= 1).
bool conv_direct_valu_eligible(const ConvPlan& g, bool padded_out);
bool conv_direct_lds_eligible(const ConvPlan& g, bool padded_out);
rtenhip_status conv_direct_valu(const ConvDmaArgs& a, int mc, hipStream_t s);
constexpr int kPwDirect = 300;
// Network stems on MFMA with the im2col in LDS (conv_stem.hip): C = 3, 7x7 or
// 3x3, stride 2, ungrouped, M <= 64, no residual / BN, unpadded input and
// output; variant kPwStem.  Weights packed [K pair][2][M rounded to 32].
constexpr int kPwStem = 800;
bool conv_stem_eligible(const ConvPlan& g, bool padded_out);
int64_t stem_weight_floats(int64_t M, int64_t K);
rtenhip_status pack_stem_weights(const float* w, int64_t M, int64_t K, float* out, hipStream_t s);
rtenhip_status conv_stem(const ConvDmaArgs& a, hipStream_t s);
// ResNet stem + its MaxPool 3x3 / 2 / pads 1 (requires the fused Relu):
// pooled [N, 64, oh / 2, ow / 2]; halo: stem_pool_halo_floats scratch.
bool conv_stem_pool_eligible(const ConvPlan& g);
int64_t stem_pool_halo_floats(const ConvPlan& g);
rtenhip_status conv_stem_pool(const ConvDmaArgs& a, float* pooled, float* halo, hipStream_t s);
rtenhip_status conv_pw_valu(const ConvDmaArgs& a, int variant, hipStream_t s);
// DMA-config numbers at and above this select the pointwise VALU kernel,
// variant cfg - kPwCfgBase (graph tuner).
constexpr int kPwCfgBase = 1000;
// Config numbers in [kLatCfgBase, kPwCfgBase) select the latency GEMM
// (gemm_lat.hip), variant cfg - kLatCfgBase; like the DMA configurations they
// read the zero-bordered input and use the plan's split workspace.
constexpr int kLatCfgBase = 500;
inline bool is_lat_cfg(int cfg) { return cfg >= kLatCfgBase && cfg < kPwCfgBase; }
bool conv_dma_eligible(int64_t N, int64_t C, int64_t Hp, int64_t Wp, int64_t O, int64_t groups,
                       int64_t K);

// Resolved conv geometry shared by shape inference and execution.
struct ConvPlan {
  int64_t N, C, H, W, O, KC, kh, kw, sh, sw, dh, dw, oh, ow, groups;
  int64_t pads[4];
  bool one_d;
};
rtenhip_status plan_conv(const rtenhip_tensor* x, const rtenhip_tensor* w, int pad_mode,
                         const int64_t* pads, const int64_t* strides, const int64_t* dilations,
                         int64_t groups, ConvPlan& p);
// Whether the conv runs on the LDS-DMA GEMM (vs depthwise / gemv / general).
bool conv_takes_dma(const ConvPlan& p);
// Weights packed for DMA configuration cfg (all groups).
int64_t packed_conv_weight_floats(const ConvPlan& p, int cfg);
rtenhip_status pack_conv_weights(Ctx* c, const float* w, const ConvPlan& p, int cfg, float* out);

rtenhip_status output_size_and_padding(int64_t in_h, int64_t in_w, int64_t k_h, int64_t k_w,
                                       int64_t stride_h, int64_t stride_w, int pad_mode,
                                       const int64_t* pads_in, int64_t dil_y, int64_t dil_x,
                                       int64_t out_hw[2], int64_t pads[4]);
rtenhip_status conv_impl(Ctx* c, const rtenhip_tensor* x, const rtenhip_tensor* w,
                         const float* bias, int pad_mode, const int64_t* pads,
                         const int64_t* strides, const int64_t* dilations, int64_t groups,
                         const float* residual, int act, float lo, float hi, rtenhip_tensor* y);
rtenhip_status gemm_impl(Ctx* c, int64_t m, int64_t n, int64_t k, const float* a, int64_t a_rs,
                         int64_t a_cs, const float* b, int64_t b_rs, int64_t b_cs, float* out,
                         int64_t out_rs, float alpha, float beta, const float* bias, int act);

// Dense GEMM on the LDS-DMA kernel (MatMul / Gemm with a row-major A and B):
//   out[m, n] = act(fold(A @ B) (+ bias[m]) (+ colbias[n]) (+ residual[m, n]))
// A: [M, K] row stride a_rs, unit column stride; packed per call into pk
// (packed_a_floats(M, K, dma_cfg_tile(cfg)) floats).  B: [K, N] row stride
// b_rs, unit column stride, read in place through the K table koff(k) = k*b_rs.
// out / residual: row strides out_rs / res_rs.  Same KC = 256 block order as
// gemm_impl, so the result is bit-identical to the general kernel.
struct DenseDmaArgs {
  int64_t M, N, K;
  const float* a;
  int64_t a_rs;
  const float* b;
  int64_t b_rs;
  float* out;
  int64_t out_rs;
  const float* bias;
  const float* colbias;
  const float* residual;
  int64_t res_rs;
  int act;
  float lo, hi;
  int cfg;         // -1 = dma_default_cfg
  float* pk;       // packed-A buffer (nullptr: ctx scratch slot 2)
  bool pack;       // pack A into pk first (false: pk already holds it)
  bool split;      // KC split of the remainder tiles
  float* ws;       // split workspace / zeroed counters (nullptr: ctx scratch)
  int64_t ws_cap;
  int* counters;
  int64_t cnt_cap;
  int persist_k;   // persistent launch (see ConvDmaArgs::persist_k)
  float* pk_out;   // store C as the next MatMul's packed A (DmaDesc::pk_out) ...
  DmaTile pk_tile; // ... for this tile shape,
  int64_t pk_K;    // ... whose K is this GEMM's N
  // n_seg > 1: N = n_seg segments of N / n_seg columns, segment s reading B
  // at b + s * K * b_rs, writing out + s * M * out_rs, colbias[n] over all N.
  int64_t n_seg;
};
// Whether gemm_dense_dma with these operands and cfg can store its output as
// a packed A (DenseDmaArgs::pk_out): the vectorised epilogue runs.
bool dense_dma_pk_out_ok(const DenseDmaArgs& a, int cfg);
bool dense_dma_eligible(int64_t M, int64_t N, int64_t K, int64_t a_cs, int64_t b_rs, int64_t b_cs);
rtenhip_status gemm_dense_dma(Ctx* c, const DenseDmaArgs& a);

// ConvTranspose (conv_transpose.cpp).
rtenhip_status conv_transpose_impl(Ctx* c, const rtenhip_tensor* x, const rtenhip_tensor* w,
                                   const float* bias, int pad_mode, const int64_t* pads,
                                   const int64_t* strides, rtenhip_tensor* y);
rtenhip_status conv_transpose_output_shape(const rtenhip_tensor* x, const rtenhip_tensor* w,
                                           int pad_mode, const int64_t* pads,
                                           const int64_t* strides, int64_t* out_shape,
                                           int32_t* out_ndim);

// broadcast_shapes (src/ops/binary_elementwise.rs:23-45).
bool broadcast_shapes(const int64_t* a, int an, const int64_t* b, int bn, int64_t* out, int* on);

// Gather launch for the graph executor (indexing.hip): out-of-range indices
// set *flag (device int) instead of synchronizing.
rtenhip_status launch_gather(const rtenhip_tensor* x, const rtenhip_tensor_i32* indices, int64_t axis,
                             rtenhip_tensor* y, int* flag, hipStream_t s);
// Moves the run's Gather flag to ring[seq % nslots] (host-mapped), clears it
// and advances seq (indexing.hip).
rtenhip_status launch_gather_check_finish(int* flag, unsigned* seq, int* ring, int nslots, hipStream_t s);

}  // namespace rtenhip
