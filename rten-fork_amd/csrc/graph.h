// Graph IR and executor state behind rtenhip_graph (restates the semantics of
// src/graph.rs: value/constant/operator nodes, DFS execution plan, refcount
// frees, in-place reuse, timing).
#pragma once

#include <hip/hip_runtime.h>

#include <map>
#include <set>
#include <memory>
#include <string>
#include <vector>

#include "common.h"
#include "ctx.h"
#include "gemm_dma.h"
#include "packed_a.h"

namespace rtenhip {

using Shape = std::vector<int64_t>;

inline int64_t prod(const Shape& s, size_t from = 0, size_t to = SIZE_MAX) {
  int64_t n = 1;
  for (size_t i = from; i < std::min(to, s.size()); i++) n *= s[i];
  return n;
}


struct Attrs {
  std::map<std::string, std::vector<double>> nums;
  std::map<std::string, std::string> strs;
  bool has(const std::string& k) const { return nums.count(k) || strs.count(k); }
  double num(const std::string& k, double dflt) const {
    auto it = nums.find(k);
    return it == nums.end() || it->second.empty() ? dflt : it->second[0];
  }
  std::vector<int64_t> ints(const std::string& k, std::vector<int64_t> dflt) const {
    auto it = nums.find(k);
    if (it == nums.end()) return dflt;
    std::vector<int64_t> r;
    for (double v : it->second) r.push_back((int64_t)v);
    return r;
  }
  std::string str(const std::string& k, const std::string& dflt) const {
    auto it = strs.find(k);
    return it == strs.end() ? dflt : it->second;
  }
};

// Parse "key=v1,v2;key2=text".
bool parse_attrs(const char* s, Attrs& out);

enum class NodeKind { Value, Constant, Operator };

// A value whose contents are known on the host when a plan is made: an int32
// or small f32 constant, or the output of the shape subgraph of an ONNX export
// (Shape -> Gather -> Unsqueeze -> Concat -> Reshape, position-id Slices ...),
// which RTen runs as tiny CPU ops on every Model::run.  A plan is specialised
// to its input shapes, so these are evaluated once, at plan time
// (graph_host.cpp), and never launched.
struct HostVal {
  int dtype = RTENHIP_DTYPE_INT32;
  Shape shape;
  std::vector<uint32_t> raw;  // 4-byte elements: int32 values or f32 bit patterns
  int64_t numel() const {
    int64_t n = 1;
    for (int64_t d : shape) n *= d;
    return n;
  }
  int64_t i(size_t k) const {  // element k as an integer
    return dtype == RTENHIP_DTYPE_INT32 ? (int64_t)(int32_t)raw[k] : (int64_t)u2f(raw[k]);
  }
  static float u2f(uint32_t u) {
    float f;
    __builtin_memcpy(&f, &u, 4);
    return f;
  }
};

struct Node {
  NodeKind kind = NodeKind::Value;
  std::string name;
  // Constant: device data + host copy for small tensors (scalar attrs).
  float* dev = nullptr;
  Shape shape;
  std::vector<float> host_small;   // values of small constants (int32 ones converted, exact)
  // Host copy of a constant's elements (all int32 constants, f32 ones up to
  // kHostConstMax elements) for plan-time evaluation of the shape subgraph.
  std::vector<uint32_t> host_raw;
  bool has_host = false;
  int dtype = RTENHIP_DTYPE_FLOAT32;  // constants: element type
  bool owns_dev = true;
  // Operator
  std::string op_type;
  Attrs attrs;
  std::vector<int> inputs;   // -1 = absent optional input
  std::vector<int> outputs;
  // Load-time fusion (rtenhip_graph_optimize): Conv epilogue.
  // Conv -> BatchNormalization: the BN node (kept, removed from the plan) and
  // its per-channel [3][O] device table {mean, scale / sqrt(var + eps), beta}
  // (owned), applied to the rounded conv output before the residual.
  int fused_bn = -1;
  float* bn_dev = nullptr;
  int fused_residual = -1;   // value id added after the bias
  int fused_act = 0;         // RTENHIP_ACT_*
  float act_lo = 0.f, act_hi = 0.f;
  // MobileNetV2's expand -> depthwise pair (Graph::optimize): the 1x1 expand
  // Conv whose only consumer is this depthwise Conv.  A plan whose shapes the
  // fused kernel takes (mbconv.hip) drops that op and runs both here, reading
  // the expand's input; otherwise both run as they are.
  int fe_op = -1;
  // The mirror pair: a 1x1 projection Conv whose input is a depthwise 3x3
  // Conv's output read by nothing else (MobileNetV2's features.1).  A plan
  // whose shapes dw_project.hip takes drops the depthwise op and runs both
  // here, reading the depthwise conv's input.
  int fd_op = -1;
  // MatMul epilogue: constant [N] added per column after the K fold
  // (MatMul -> Add(bias)), before the residual and the activation.
  int fused_colbias = -1;
  // FusedTranspose (src/ops/fused.rs:45-80): input index -> permutation of
  // that input's view (empty = reversed axes, Transpose without perm).
  std::map<int, std::vector<int64_t>> input_perm;
  bool removed = false;      // op folded into another
  // Operator::name() of the node after RTen's fusions (optimize.rs), when it
  // differs from op_type: "FusedTranspose(MatMul)".
  std::string fused_name;
  bool alias_input0 = false; // output is a view of input 0 (Flatten/Reshape)
};

struct Slot {
  size_t offset = 0;  // bytes into the arena, or external pointer when ext
  float* ext = nullptr;
  Shape shape;
};

// A Conv the plan runs on the LDS-DMA GEMM (see exec_op).
struct ConvExec {
  ConvPlan g;
  int cfg = -1;             // kernel configuration (chosen on the first run)
  float* packed = nullptr;  // weights packed for cfg, owned by the plan
  bool split = false;       // KC split of the remainder tiles (dma_split_plan)
  float* ws = nullptr;      // its workspace and arrival counters, plan-owned
  int* counters = nullptr;
  int64_t ws_floats = 0, n_counters = 0;
  int persist = 0;          // persistent launch, blocks per CU (0: one block per item); tuned
  // A VALU configuration (cfg >= kPwCfgBase) needs 16-byte aligned operands;
  // a later run bound to a misaligned graph input / output view takes this
  // DMA configuration instead (weights packed for it when the VALU one is chosen).
  int fb_cfg = -1;
  float* fb_packed = nullptr;
  // A Gemm (FC layer) run as this conv: x [B, K] as B images of [K, 1, 1],
  // W [O, K] (transB) as O pointwise filters, C [O] as the bias.
  bool fc = false;
};

// A MatMul the plan runs on the dense LDS-DMA GEMM: [batch.., M, K] @ [K, N]
// with the batch folded into M (matmul.rs:162-169), A contiguous.
struct MatMulExec {
  int64_t M, N, K, b_rs;
  int cfg = -1;          // kernel configuration (chosen on the first run)
  bool split = false;
  float* ws = nullptr;   // split workspace and arrival counters, plan-owned
  int* counters = nullptr;
  int64_t ws_floats = 0, n_counters = 0;
  int persist = 0;       // persistent launch, blocks per CU (0: one block per item); tuned
  // Grouped MatMuls (Plan::mm_group): this leader runs nseg MatMuls that
  // share A, as one GEMM with N = nseg * seg_n over stacked B / bias /
  // output segments (BERT's Q, K and V projections).
  int nseg = 1;
  int64_t seg_n = 0;
  float* b_cat = nullptr;   // [nseg][K][seg_n]
  float* cb_cat = nullptr;  // [nseg][seg_n] or null
};

// A value stored with a zero border so the DMA convs reading it need no
// per-run padding copy: physical [N, C, H + pt + pb, W + pl + pr], written by
// its producer (a DMA conv) into the interior.  Persistent, outside the arena,
// so the border stays zero.
struct PaddedValue {
  float* base = nullptr;
  int64_t pads[4] = {0, 0, 0, 0};
  Shape phys;
};

struct Plan {
  ~Plan();
  // Kernel knobs the plan was made under (Graph::find_plan matches them):
  // Ctx::use_dma, and use_dma with no forced GEMM configuration (dense
  // MatMuls on the DMA GEMM; only then are Q/K/V groups and packed-A
  // producers formed, since only that kernel writes them).
  bool dma = true, dma_mm = true;
  std::vector<int> ops;               // topological order
  std::map<int, ConvExec> convs;      // op id -> DMA conv state
  std::map<int, PaddedValue> padded;  // value id -> zero-bordered storage
  std::map<int, MatMulExec> matmuls;  // op id -> dense DMA MatMul state
  // Conv -> Add fusions whose Add broadcasts (the other input is not the conv
  // output's shape): the conv runs into this plan-owned buffer, then the Add
  // and the activation run as the unfused graph would.  op id -> (buffer, shape).
  std::map<int, std::pair<float*, Shape>> conv_unfused;
  // Depthwise convs running their expand conv too (see Node::fe_op): op id ->
  // the expand's input value, which the depthwise op then reads.
  std::map<int, int> expand_fused;
  // A bottleneck's conv3 and the next block's conv1 as one conv_pair.hip
  // launch at conv3's position (conv1's op then skips): conv3 op -> conv1 op;
  // conv1 op -> the conv3 inputs it keeps allocated until then (x, residual);
  // conv3 op -> its packed weights.
  std::map<int, int> conv_pair;
  std::map<int, std::pair<int, int>> pair_hold;
  struct PairExec {
    float* w3p = nullptr;
    float* w1p = nullptr;
  };
  std::map<int, PairExec> pair_exec;
  // Projection convs running their depthwise conv too (see Node::fd_op): op id
  // -> the depthwise conv's input value, which the projection op then reads.
  std::map<int, int> dwpw_fused;
  // ... of which those running the stem conv producing the depthwise input
  // too (dw_project.hip stem_dw_project_kernel): projection op -> the stem
  // conv op (out of the plan; dwpw_fused then names the stem's input).
  std::map<int, int> stem_dwpw;
  // MaxPool ops running their stem conv too (conv_stem.hip POOL): pool op ->
  // the conv op (out of the plan; its output never exists); the weights
  // packed for the stem kernel and the halo rows between bands.
  std::map<int, int> stem_pool;
  struct StemPoolExec {
    float* packed = nullptr;
    float* halo = nullptr;
  };
  std::map<int, StemPoolExec> stem_pool_exec;
  // Grouped MatMuls (MatMulExec::nseg): leader op -> members (leader first),
  // members run by their leader; the members' outputs are segments of one
  // arena block of [nseg][M][N].
  std::map<int, std::vector<int>> mm_group;
  std::set<int> mm_group_skip;
  // FusedAttention op -> the value (its output's Reshape) a dense MatMul
  // reads as A: the attention kernel also stores it packed (Plan::pk_cons).
  std::map<int, int> attn_pk;
  std::set<int> attn_pk_only;  // ... and nothing reads its row-major output
  // ResNet's conv3 + downsample pairs: conv3 op -> downsample op (its fused
  // residual's producer, read by nothing else).  On the first run conv3 times
  // the dual GEMM (gemm_dma_kernel DUAL, both convs in one launch) against
  // the two launches as tuned; when it wins (dual_on) the downsample op is
  // skipped and conv3 computes both.
  std::map<int, int> conv_dual;
  struct DualExec {
    int cfg = -1;
    float* pk3 = nullptr;  // conv3 / downsample weights packed for cfg
    float* pkd = nullptr;
    int persist = 0;
  };
  std::map<int, DualExec> dual_on;   // conv3 op -> its dual launch
  std::set<int> dual_skip;           // downsample ops computed by their conv3
  // Batch-1 bottleneck conv1 + downsample (both 1x1, reading the block
  // input) in one latency-GEMM launch (gemm_lat2_pair_kernel): conv1 op ->
  // downsample op, which the plan moves right after conv1.  On the first run,
  // once both are tuned onto latency GEMMs, the pair variants are timed
  // against the two launches; when one wins (on) conv1's op runs both.
  std::map<int, int> lat_pair;
  std::map<int, int> lat_pair_of;  // downsample op -> its conv1 op
  struct LatPairExec {
    bool decided = false, on = false;
    int v0 = 0, v1 = 0;              // the pair's variants (conv1, downsample)
    float* ws[2] = {nullptr, nullptr};
    int* cnt[2] = {nullptr, nullptr};
    int64_t ws_floats[2] = {0, 0}, n_cnt[2] = {0, 0};
  };
  std::map<int, LatPairExec> lat_pair_exec;  // conv1 op ->
  float* mm_pack = nullptr;           // packed-A buffer shared by the plan's MatMuls
  int64_t mm_pack_floats = 0;
  // What mm_pack holds during a run: the A value it was packed from (value
  // ids are single-assignment, so MatMuls reading the same A -- Q/K/V
  // projections -- pack it once) and the tile shape; -1 = nothing.
  int mm_pack_value = -1;
  DmaTile mm_pack_tile{0, 0, 0};
  // A operands stored packed by their producer (packed_a.h), so the dense
  // MatMuls reading them skip pack_a: value -> its first dense-MatMul reader
  // (whose tile, chosen on the first run, fixes the layout).  Producers: a
  // dense MatMul whose output nothing else reads (BERT's FFN1 -> FFN2; it then
  // stores only the packed layout, pk_only) or a LayerNormalization over the
  // rows (row-major for its other readers, and packed: BERT's LN -> Q/K/V and
  // FFN1).  pk_buf: value -> buffer, floats (zeroed once, so the tile padding
  // stays zero); pk_ready: value -> tile stored during this run.
  std::map<int, int> pk_cons;
  std::set<int> pk_only;
  std::map<int, std::pair<float*, int64_t>> pk_buf;
  std::map<int, DmaTile> pk_ready;
  std::map<int, Slot> slots;          // value id -> storage
  size_t arena_bytes = 0;
  std::vector<int> input_ids, output_ids;
  std::vector<Shape> input_shapes;
  std::vector<int> input_dtypes;
  std::map<int, int> dtypes;          // value id -> element type (RTENHIP_DTYPE_*)
  // Plan-time values (see HostVal) and the device copies of those a kernel
  // or a graph output reads (uploaded once, plan-owned).
  std::map<int, HostVal> host;
  std::map<int, float*> host_dev;
  // Gathers with non-constant indices record an out-of-range index here
  // (graph-capturable: no sync inside the ops).  The end of each run copies
  // the flag into a pinned host word of a check slot, clears it and records
  // an event.  By default the run then waits for that event and returns the
  // error itself, as the reference's Model::run does (gather.rs:52-60).
  // With Graph::deferred_checks the slots form a ring of kGatherChecks, so
  // several runs can be queued; each slot carries its run's sequence number
  // and its error is reported only by Graph::synchronize
  // (rtenhip_graph_synchronize), never by a later, unrelated run.
  // (Round 6: the flag's move and clear are one launch at the end of the run,
  // inside the captured graph -- launch_gather_check_finish -- into the
  // check ring gring, a fine-grained host-mapped array of kGatherChecks
  // words; the run's slot is gseq % kGatherChecks, gseq counting the finish
  // launches on the host as gseq_dev does on the device.)
  int* gather_flag = nullptr;
  static constexpr int kGatherChecks = 4;
  int* gring_host = nullptr;
  int* gring_dev = nullptr;
  unsigned* gseq_dev = nullptr;
  uint64_t gseq = 0;
  struct GatherCheck {
    int* host = nullptr;       // the slot's word of gring_host
    hipEvent_t ev = nullptr;
    bool pending = false;
    uint64_t run = 0;          // Graph::run_seq of the run that queued it
  } gchk[kGatherChecks];
  int gchk_next = 0;
  // hipGraph replay state: each capture is valid for its exact input / output
  // pointers (and the ctx scratch generation it baked in).  Up to
  // kMaxCaptures bindings are kept (least recently used replaced), so a
  // caller that alternates between staging buffers (double-buffered host
  // input, rten_hip/staging.py) replays without re-capturing.
  struct Capture {
    hipGraphExec_t exec = nullptr;
    std::vector<float*> in, out;
    uint64_t scratch_gen = 0;   // Ctx::scratch_gen when captured
    uint64_t last_use = 0;      // Graph::run_seq
  };
  static constexpr int kMaxCaptures = 4;
  std::vector<Capture> captures;
  void drop_captures() {
    for (auto& c : captures)
      if (c.exec) (void)hipGraphExecDestroy(c.exec);
    captures.clear();
  }
  std::vector<float*> bound_in, bound_out;  // this run's binding (ptr_of)
  std::map<size_t, size_t> scratch_need;   // ctx scratch slot -> floats (eager runs)
  int eager_runs = 0;
};

struct HostPipe;
void destroy_host_pipe(HostPipe* p);

struct Graph {
  Ctx* ctx = nullptr;
  rtenhip_ctx* cptr = nullptr;
  std::vector<Node> nodes;
  std::map<std::string, int> by_name;
  std::vector<int> model_inputs, model_outputs;
  std::vector<std::unique_ptr<Plan>> plans;
  // Grouped MatMuls' stacked weights and column biases ([nseg][K][N],
  // [nseg][N]), keyed by the members' (weight, bias) node ids; shared by
  // every plan of the graph.
  std::map<std::vector<int>, std::pair<float*, float*>> mm_cat;
  void* arena = nullptr;
  size_t arena_cap = 0;
  hipStream_t exec_stream = nullptr;
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  bool timing = false;
  int* hold_word = nullptr;  // pinned coherent host words: [0] releases launch_hold, [1] set when it timed out
  bool use_hip_graph = true;
  // Gather index checks (Plan::gchk): false = each run waits for its own
  // check and returns its error; true = checks are queued and reported by
  // synchronize() only (rtenhip_graph_set_deferred_checks).
  bool deferred_checks = false;
  uint64_t run_seq = 0;             // runs started
  uint64_t deferred_error_run = 0;  // earliest run with an unreported index error (0: none)
  bool autotune = true;  // time DMA conv configurations on a plan's first run
  int persist_mode = -1; // DMA GEMM launches: -1 tuned, 0 never persistent, k: always, k blocks/CU
  int lat_mode = -1;     // latency GEMM convs (gemm_lat.hip): -1 tuned, 0 never, v > 0 forced variant
  int pw_valu_mode = -1; // pointwise convs on the VALU kernel: -1 tuned, 0 never, v > 0 forced variant (pw_variant_ok)
  std::string timing_report;
  std::map<std::string, std::pair<double, int>> timing_totals;  // op type -> (ms, count)
  // Host-resident runs (graph_io.cpp, rtenhip_graph_run_host): the staging
  // pipeline, and while ext_order is set run() orders the executor stream
  // after ext_waits and records ext_records at its end instead of syncing with
  // the caller's stream.
  HostPipe* host_pipe = nullptr;
  bool ext_order = false;
  std::vector<hipEvent_t> ext_waits, ext_records;

  ~Graph();
  int add_node(Node n);
  // in_dt: element type per input (RTENHIP_DTYPE_*), nullptr = all float32.
  rtenhip_status run(const int32_t* in_ids, const rtenhip_tensor* ins, int n_in,
                     const int32_t* out_ids, rtenhip_tensor* outs, int n_out,
                     const int32_t* in_dt = nullptr);
  rtenhip_status optimize();
  // Waits for the queued runs and reports a Gather index error any of them
  // recorded (see Plan::gchk).
  rtenhip_status synchronize();
  // Reads the completed Gather checks of p (all pending ones when wait) into
  // deferred_error_run.
  rtenhip_status collect_gather_checks(Plan& p, bool wait);
  // RTen's own passes (src/optimize.rs:286-518, graph_optimize.cpp), run
  // first by optimize(): constant propagation, Silu / Gelu / LayerNorm fusion.
  rtenhip_status rten_optimize();
  rtenhip_status propagate_constants();
  int fuse_rten_patterns();
  // Host value of `id` (a constant with a host copy, or a plan-time value of
  // the plan being made / run), or nullptr.
  const HostVal* host_value(int id, HostVal& tmp) const;
  const std::map<int, HostVal>* planning_host = nullptr;
  rtenhip_status plan_shapes(const int32_t* in_ids, const rtenhip_tensor* ins, int n_in,
                             const int32_t* out_ids, int n_out, int64_t* shapes, int32_t* ndims,
                             const int32_t* in_dt = nullptr, int32_t* out_dt = nullptr);

 private:
  rtenhip_status find_plan(const int32_t* in_ids, const rtenhip_tensor* ins, int n_in,
                           const int32_t* in_dt, const int32_t* out_ids, int n_out, Plan** out);
  rtenhip_status make_plan(const std::vector<int>& in_ids, const std::vector<Shape>& in_shapes,
                           const std::vector<int>& in_dtypes, const std::vector<int>& out_ids,
                           Plan& p);
  rtenhip_status infer_shapes(int op_id, const std::vector<const Shape*>& ins,
                              std::vector<Shape>& outs);
  rtenhip_status infer_dtypes(int op_id, const std::vector<int>& ins, std::vector<int>& outs);
  rtenhip_status exec_op(Plan& p, int op_id);
  // Plan-time evaluation of op_id from host values (graph_host.cpp): returns
  // true with out filled, false when an input is not known on the host or the
  // op is not one the host evaluates; st is set on an operator error.
  bool host_eval(int op_id, const std::vector<const Shape*>& in_shapes, const Shape& out_shape,
                 int out_dtype, HostVal& out, rtenhip_status& st);
  rtenhip_status exec_data_op(Plan& p, int op_id, bool& handled);
  rtenhip_status exec_conv_dma(Plan& p, int op_id, ConvExec& ce);
  // conv3 of a Plan::conv_dual pair: the dual launch, or (first run) the
  // choice between it and the unfused pair.
  rtenhip_status exec_conv_dual(Plan& p, int op_id, bool& handled);
  // conv1 + downsample of a Plan::lat_pair: the pair launch, and (first run,
  // at the downsample op) the choice between it and the two launches.
  rtenhip_status exec_lat_pair(Plan& p, int c_op);
  rtenhip_status tune_lat_pair(Plan& p, int c_op);
  void conv_io_args(Plan& p, int op_id, ConvDmaArgs& a);
  rtenhip_status exec_expand_dw(Plan& p, int op_id);
  rtenhip_status exec_dw_project(Plan& p, int op_id);
  rtenhip_status exec_conv_pair(Plan& p, int op_id);
  rtenhip_status exec_stem_pool(Plan& p, int op_id);
  rtenhip_status exec_matmul(Plan& p, int op_id, rtenhip_tensor a, rtenhip_tensor b, rtenhip_tensor y);
  rtenhip_status exec_attention(Plan& p, int op_id, rtenhip_tensor y);
  // The packed-A store a producer of value v makes this run, or false.
  bool packed_out_for(Plan& p, int v, int64_t M, int64_t K, PackedOut& po, DmaTile& tile);
  rtenhip_status exec_matmul_dma(Plan& p, int op_id, const rtenhip_tensor& a,
                                 const rtenhip_tensor& b, const rtenhip_tensor& y, MatMulExec& me);
  float* ptr_of(Plan& p, int value_id);
};

// Slice (slice.rs:18-65) as a strided view of an input of shape xs: base
// element offset, output dims and per-dim source strides (negative for
// negative steps).  False when starts / ends / axes / steps are not known on
// the host (st stays OK) or on an operator error (st set).
bool slice_view(const Graph& g, const Node& op, const Shape& xs, int64_t& base, std::vector<int64_t>& out_dims,
                std::vector<int64_t>& sst, rtenhip_status& st);

constexpr int64_t kHostConstMax = 4096;     // f32 constants kept on the host
constexpr int64_t kHostEvalMax = 1 << 16;    // plan-time evaluation output cap

}  // namespace rtenhip
