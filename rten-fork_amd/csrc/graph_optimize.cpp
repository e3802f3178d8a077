// RTen's load-time graph optimizer on the device graph (GraphOptimizer::
// optimize, src/optimize.rs:286-297), run first by Graph::optimize:
//
//  - propagate_constants (optimize.rs:301-327 via Graph::partial_run /
//    prune_plan, graph.rs:1147-1234): every operator reachable from the
//    outputs whose inputs are all constants is evaluated once -- on the device,
//    through an ordinary plan with no inputs -- and its leaf values (read by an
//    operator that is not evaluable, or a model output) become constants;
//  - fuse_silu / fuse_gelu / fuse_layer_norm (optimize.rs:380-518) with the
//    pattern matcher of src/optimize/pattern_matcher.rs: commutative Add / Mul
//    match either way round, constants within 1e-4, symbols bind one node, an
//    operator pattern needs exactly its input count.  A fused operator
//    replaces the subgraph's final node in place (same name, same output
//    value, as Fusion::apply + replace_value); the intermediate operators stay
//    and are simply not planned when nothing live reads them.
//
// (fuse_transpose, optimize.rs:333-377, is the FusedTranspose pass of
// Graph::optimize: a MatMul reads the Transpose's input as a permuted view.)
#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>

#include "graph.h"

namespace rtenhip {
namespace {

struct Pat {
  enum Kind { Sym, Const, Op } kind = Sym;
  std::string name;  // symbol or operator name
  bool const_only = false;
  float value = 0.f;
  std::vector<Pat> in;
  std::string key;  // unary_op_key
};

Pat sym(const char* n, bool c = false) {
  Pat p;
  p.kind = Pat::Sym;
  p.name = n;
  p.const_only = c;
  return p;
}
Pat cst(float v) {
  Pat p;
  p.kind = Pat::Const;
  p.value = v;
  return p;
}
Pat op(const char* n, std::vector<Pat> in, const char* key = "") {
  Pat p;
  p.kind = Pat::Op;
  p.name = n;
  p.in = std::move(in);
  p.key = key;
  return p;
}

constexpr float kConstTolerance = 1e-4f;  // pattern_matcher.rs:70

bool commutative(const std::string& t) {  // Operator::is_commutative
  return t == "Add" || t == "Mul" || t == "And" || t == "Or" || t == "Xor" || t == "Equal";
}

struct Matcher {
  const Graph& g;
  const std::map<int, int>& producer;  // value -> live operator
  std::vector<std::pair<std::string, int>> syms;

  int find(const std::string& n) const {
    for (auto& s : syms)
      if (s.first == n) return s.second;
    return -1;
  }

  bool op_matches(const Pat& p, int op_id) {
    const Node& n = g.nodes[op_id];
    if (n.op_type != p.name || p.in.size() != n.inputs.size()) return false;
    if (commutative(n.op_type) && p.in.size() == 2 && n.inputs[0] >= 0 && n.inputs[1] >= 0) {
      const size_t mark = syms.size();
      if (test(p.in[0], n.inputs[0]) && test(p.in[1], n.inputs[1])) return true;
      syms.resize(mark);
      return test(p.in[1], n.inputs[0]) && test(p.in[0], n.inputs[1]);
    }
    for (size_t i = 0; i < p.in.size(); i++)
      if (n.inputs[i] < 0 || !test(p.in[i], n.inputs[i])) return false;
    return true;
  }

  // Pattern::test_impl (pattern_matcher.rs:188-238)
  bool test(const Pat& p, int id) {
    if (id < 0 || id >= (int)g.nodes.size()) return false;
    const Node& n = g.nodes[id];
    if (p.kind == Pat::Op) {
      if (n.kind == NodeKind::Constant) return false;
      int op_id = id;
      if (n.kind == NodeKind::Value) {
        auto it = producer.find(id);
        if (it == producer.end()) return false;
        op_id = it->second;
      }
      if (!op_matches(p, op_id)) return false;
      if (!p.key.empty()) syms.push_back({p.key, op_id});
      return true;
    }
    if (p.kind == Pat::Const) {
      // ConstantPattern::matches: a float tensor with one element (item())
      if (n.kind != NodeKind::Constant || n.dtype != RTENHIP_DTYPE_FLOAT32 || prod(n.shape) != 1 ||
          n.host_small.empty())
        return false;
      return std::fabs(n.host_small[0] - p.value) <= kConstTolerance;
    }
    if (n.kind == NodeKind::Operator) return false;
    if (p.const_only && n.kind != NodeKind::Constant) return false;
    const int bound = find(p.name);
    if (bound >= 0) return bound == id;
    syms.push_back({p.name, id});
    return true;
  }
};

}  // namespace

// Operators reachable from the model outputs (all operators when the graph
// declares none), in dependency order.
static std::vector<int> live_ops_topo(const Graph& g, const std::map<int, int>& producer) {
  std::vector<int> order;
  std::set<int> seen;
  std::function<void(int)> visit = [&](int v) {
    auto it = producer.find(v);
    if (it == producer.end() || seen.count(it->second)) return;
    seen.insert(it->second);
    const Node& n = g.nodes[it->second];
    for (int i : n.inputs)
      if (i >= 0) visit(i);
    if (n.fused_residual >= 0) visit(n.fused_residual);
    order.push_back(it->second);
  };
  if (!g.model_outputs.empty()) {
    for (int o : g.model_outputs) visit(o);
  } else {
    for (auto& kv : producer) visit(kv.first);
  }
  return order;
}

static std::map<int, int> live_producers(const Graph& g) {
  std::map<int, int> producer;
  for (int i = 0; i < (int)g.nodes.size(); i++)
    if (g.nodes[i].kind == NodeKind::Operator && !g.nodes[i].removed)
      for (int o : g.nodes[i].outputs) producer[o] = i;
  return producer;
}

rtenhip_status Graph::propagate_constants() {
  const std::map<int, int> producer = live_producers(*this);
  const std::vector<int> order = live_ops_topo(*this, producer);
  std::set<int> resolved;  // values computable from constants
  std::set<int> evaluable_ops;
  std::set<int> leaf_inputs;  // resolved inputs of operators that are not evaluable
  auto is_resolved = [&](int v) { return nodes[v].kind == NodeKind::Constant || resolved.count(v); };
  for (int op : order) {
    const Node& n = nodes[op];
    bool all = n.fused_residual < 0;
    for (int i : n.inputs)
      if (i >= 0 && !is_resolved(i)) all = false;
    if (!all) {
      for (int i : n.inputs)
        if (i >= 0 && resolved.count(i)) leaf_inputs.insert(i);
      continue;
    }
    evaluable_ops.insert(op);
    for (int o : n.outputs) resolved.insert(o);
  }
  std::vector<int> leaves;
  for (int v : resolved)
    if (leaf_inputs.count(v) || std::count(model_outputs.begin(), model_outputs.end(), v)) leaves.push_back(v);
  if (leaves.empty()) return RTENHIP_OK;

  // Evaluate the leaves with a plan that has no inputs.
  std::vector<int64_t> shp(leaves.size() * RTENHIP_MAX_DIMS);
  std::vector<int32_t> nds(leaves.size()), dts(leaves.size());
  rtenhip_status st = plan_shapes(nullptr, nullptr, 0, leaves.data(), (int)leaves.size(), shp.data(), nds.data(),
                                  nullptr, dts.data());
  if (st) return st;
  std::vector<rtenhip_tensor> outs(leaves.size());
  std::vector<float*> bufs(leaves.size(), nullptr);
  auto free_bufs = [&]() {
    for (float* b : bufs)
      if (b) (void)hipFree(b);
  };
  for (size_t k = 0; k < leaves.size(); k++) {
    Shape s(shp.begin() + k * RTENHIP_MAX_DIMS, shp.begin() + k * RTENHIP_MAX_DIMS + nds[k]);
    if (hipMalloc(&bufs[k], (size_t)std::max<int64_t>(1, prod(s)) * 4) != hipSuccess) {
      free_bufs();
      return fail(RTENHIP_HIP_ERROR, "hipMalloc failed for a propagated constant");
    }
    outs[k] = make_tensor(bufs[k], s.data(), (int)s.size());
  }
  const bool timing_was = timing;
  timing = false;
  hipStream_t caller = ctx->stream;
  st = run(nullptr, nullptr, 0, leaves.data(), outs.data(), (int)leaves.size());
  timing = timing_was;
  if (!st && hipStreamSynchronize(caller) != hipSuccess) st = fail(RTENHIP_HIP_ERROR, "constant propagation sync");
  if (st) {
    free_bufs();
    std::string msg = std::string("partial evaluation failed: ") + rtenhip_last_error_message();
    return fail(st, msg.c_str());
  }
  // The leaf values become constants (RTen adds constant nodes and replaces
  // every use; here the value node itself turns into the constant, which
  // keeps the ids that inputs, outputs and consumers hold).
  for (size_t k = 0; k < leaves.size(); k++) {
    Node& n = nodes[leaves[k]];
    n.kind = NodeKind::Constant;
    n.dev = bufs[k];
    n.owns_dev = true;
    n.shape.assign(outs[k].shape, outs[k].shape + outs[k].ndim);
    n.dtype = dts[k];
    const int64_t cnt = prod(n.shape);
    if (cnt <= (n.dtype == RTENHIP_DTYPE_INT32 ? ((int64_t)1 << 22) : kHostConstMax)) {
      n.host_raw.resize((size_t)cnt);
      if (cnt && hipMemcpy(n.host_raw.data(), bufs[k], (size_t)cnt * 4, hipMemcpyDeviceToHost) != hipSuccess)
        return fail(RTENHIP_HIP_ERROR, "hipMemcpy failed");
      n.has_host = true;
      if (cnt <= 64) {
        n.host_small.resize((size_t)cnt);
        for (int64_t i = 0; i < cnt; i++)
          n.host_small[i] = n.dtype == RTENHIP_DTYPE_INT32 ? (float)(int32_t)n.host_raw[i] : HostVal::u2f(n.host_raw[i]);
      }
    }
  }
  for (int op : evaluable_ops) nodes[op].removed = true;
  for (auto& pl : plans) pl->drop_captures();
  plans.clear();
  return RTENHIP_OK;
}

int Graph::fuse_rten_patterns() {
  int fused = 0;
  struct Fusion {
    int op;
    std::string type;
    std::vector<int> inputs;
    Attrs attrs;
  };
  // GraphMutator::apply_fusion (optimize.rs:128-143): every fusion of a pass is
  // found on the graph as it is, then all are applied.
  auto apply_pass = [&](const std::function<bool(Matcher&, int, Fusion&)>& try_fuse) {
    const std::map<int, int> producer = live_producers(*this);
    std::vector<Fusion> found;
    for (int i = 0; i < (int)nodes.size(); i++) {
      const Node& n = nodes[i];
      if (n.kind != NodeKind::Operator || n.removed || n.outputs.size() != 1) continue;
      Matcher m{*this, producer, {}};
      Fusion f;
      f.op = i;
      if (try_fuse(m, i, f)) found.push_back(std::move(f));
    }
    for (Fusion& f : found) {
      Node& n = nodes[f.op];
      n.op_type = f.type;
      n.inputs = f.inputs;
      n.attrs = f.attrs;
      n.input_perm.clear();
      fused++;
    }
  };

  // fuse_silu (optimize.rs:380-398): x * Sigmoid(x)
  {
    const Pat pat = op("Mul", {sym("x"), op("Sigmoid", {sym("x")})});
    apply_pass([&](Matcher& m, int i, Fusion& f) {
      if (!m.test(pat, nodes[i].outputs[0])) return false;
      f.type = "Silu";
      f.inputs = {m.find("x")};
      return true;
    });
  }
  // fuse_gelu (optimize.rs:401-424): x * (Erf(x / sqrt(2)) + 1.0) * 0.5
  {
    const Pat pat = op("Mul", {op("Mul", {sym("x"), op("Add", {op("Erf", {op("Div", {sym("x"), cst(std::sqrt(2.0f))})}),
                                                               cst(1.0f)})}),
                               cst(0.5f)});
    apply_pass([&](Matcher& m, int i, Fusion& f) {
      if (!m.test(pat, nodes[i].outputs[0])) return false;
      f.type = "Gelu";
      f.inputs = {m.find("x")};
      return true;
    });
  }
  // fuse_layer_norm (optimize.rs:427-518): three patterns matched from the
  // final step backwards; both ReduceMeans must reduce axis -1 only.
  {
    const Pat center = op("Sub", {sym("x"), op("ReduceMean", {sym("x")}, "center_mean")});
    const Pat norm = op("Div", {sym("x"), op("Sqrt", {op("Add", {sym("epsilon", true),
                                                               op("ReduceMean", {op("Pow", {sym("x"), cst(2.0f)})},
                                                                  "norm_mean")})})});
    const Pat shift_scale = op("Add", {op("Mul", {sym("x"), sym("scale", true)}), sym("bias", true)});
    auto reduces_last_axis = [&](int op_id) {
      const Node& n = nodes[op_id];
      if (n.op_type != "ReduceMean") return false;
      auto it = n.attrs.nums.find("axes");
      if (it != n.attrs.nums.end() && it->second.size() == 1 && it->second[0] == -1) return true;
      if (n.inputs.size() > 1 && n.inputs[1] >= 0) {
        const Node& a = nodes[n.inputs[1]];
        return a.kind == NodeKind::Constant && a.dtype == RTENHIP_DTYPE_INT32 && a.shape.size() == 1 &&
               a.has_host && a.host_raw.size() == 1 && (int32_t)a.host_raw[0] == -1;
      }
      return false;
    };
    apply_pass([&](Matcher& m, int i, Fusion& f) {
      if (!m.test(shift_scale, nodes[i].outputs[0])) return false;
      const int x1 = m.find("x"), scale = m.find("scale"), bias = m.find("bias");
      Matcher m2{*this, m.producer, {}};
      if (!m2.test(norm, x1) || !reduces_last_axis(m2.find("norm_mean"))) return false;
      const int x2 = m2.find("x"), eps = m2.find("epsilon");
      Matcher m3{*this, m.producer, {}};
      if (!m3.test(center, x2) || !reduces_last_axis(m3.find("center_mean"))) return false;
      // Constant::as_scalar for f32: a float tensor with one element
      const Node& e = nodes[eps];
      if (e.dtype != RTENHIP_DTYPE_FLOAT32 || prod(e.shape) != 1 || e.host_small.empty()) return false;
      f.type = "LayerNormalization";
      f.inputs = {m3.find("x"), scale, bias};
      f.attrs.nums["axis"] = {-1};
      f.attrs.nums["epsilon"] = {(double)e.host_small[0]};
      return true;
    });
  }
  return fused;
}

rtenhip_status Graph::rten_optimize() {
  rtenhip_status st = propagate_constants();
  if (st) return st;
  (void)fuse_rten_patterns();
  return RTENHIP_OK;
}

}  // namespace rtenhip
