// .rten model loader (Model::load, src/model.rs:265-522; header: src/header.rs:57-146;
// FlatBuffers schema: src/schema.fbs; attribute decoding: src/op_registry.rs:239-820).
//
// The file is parsed on the host with a small bounds-checked FlatBuffers
// reader (no flatc / flatbuffers library in this image), into the same node
// list the reference builds (values, constants, operators in file order, so a
// file node index is the graph node id).  Constants are uploaded once; the
// graph is then optimized unless the caller opts out (ModelOptions::
// with_optimize, model.rs:156-162).
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "graph.h"

namespace rtenhip {
namespace {

// sg::OperatorType names in enum order (schema.fbs:12-121).
const char* const kOpTypes[] = {
    "Add", "ArgMin", "ArgMax", "AveragePool", "BatchNormalization", "Cast", "Clip", "Concat",
    "ConstantOfShape", "Conv", "ConvTranspose", "Cos", "CumSum", "Div", "Equal", "Erf", "Expand",
    "Flatten", "Gather", "Gemm", "GlobalAveragePool", "Greater", "GRU", "Identity", "LeakyRelu",
    "Less", "LessOrEqual", "Log", "LogSoftmax", "LSTM", "MatMul", "MaxPool", "Mod", "Mul", "Pad",
    "Pow", "Range", "ReduceMean", "ReduceL2", "Relu", "Reshape", "Resize", "Shape", "Sigmoid",
    "Sin", "Slice", "Split", "Sqrt", "Squeeze", "Softmax", "Sub", "Tanh", "Transpose", "Unsqueeze",
    "Where", "ReduceProd", "ReduceSum", "ReduceMin", "ReduceMax", "NonZero", "ScatterElements",
    "Tile", "Not", "Abs", "Max", "Mean", "Min", "Sum", "OneHot", "Round", "Floor", "Ceil",
    "Reciprocal", "TopK", "Neg", "Exp", "GreaterOrEqual", "Size", "Tan", "Acos", "Asin", "Atan",
    "InstanceNormalization", "HardSigmoid", "HardSwish", "And", "Or", "Xor", "Trilu", "ScatterND",
    "NonMaxSuppression", "Sign", "GatherElements", "LayerNormalization", "ReduceSumSquare",
    "RandomUniform", "Elu", "RandomUniformLike", "RandomNormal", "RandomNormalLike", "Softplus",
    "GatherND", "Gelu", "Einsum", "If"};
constexpr int kNumOpTypes = sizeof(kOpTypes) / sizeof(kOpTypes[0]);

// sg::OperatorAttrs union member ids used by the supported operators.
enum AttrsType : uint8_t {
  kAveragePoolAttrs = 2,
  kBatchNormalizationAttrs = 3,
  kCastAttrs = 4,
  kConcatAttrs = 5,
  kConstantOfShapeAttrs = 6,
  kConvAttrs = 7,
  kConvTransposeAttrs = 8,
  kFlattenAttrs = 9,
  kGatherAttrs = 10,
  kGemmAttrs = 11,
  kMaxPoolAttrs = 15,
  kReduceMeanAttrs = 16,
  kReshapeAttrs = 17,
  kSoftmaxAttrs = 20,
  kTransposeAttrs = 21,
  kLayerNormalizationAttrs = 30,
  kGeluAttrs = 37,
};
enum NodeKindType : uint8_t { kOperatorNode = 1, kConstantNode = 2, kValueNode = 3 };
enum ConstantDataType : uint8_t { kFloatData = 1, kIntData = 2 };

struct LoadError {
  int code;
  std::string msg;
};

// Bounds-checked FlatBuffers access (the checks a verifier would make).
struct Fb {
  const uint8_t* p;
  size_t n;
  bool in(size_t off, size_t len) const { return off <= n && len <= n - off; }
  template <typename T>
  T rd(size_t off) const {
    if (!in(off, sizeof(T))) throw LoadError{RTENHIP_INVALID_VALUE, "parse error: range out of bounds"};
    T v;
    std::memcpy(&v, p + off, sizeof(T));
    return v;
  }
};

struct Table {
  const Fb* fb = nullptr;
  size_t pos = 0;
  size_t vt = 0;
  uint16_t vsize = 0;
  explicit operator bool() const { return fb != nullptr; }
  static Table at(const Fb& fb, size_t pos) {
    Table t;
    t.fb = &fb;
    t.pos = pos;
    const int64_t vt = (int64_t)pos - (int64_t)fb.rd<int32_t>(pos);
    if (vt < 0) throw LoadError{RTENHIP_INVALID_VALUE, "parse error: invalid vtable offset"};
    t.vt = (size_t)vt;
    t.vsize = fb.rd<uint16_t>(t.vt);
    if (t.vsize < 4 || t.vsize % 2) throw LoadError{RTENHIP_INVALID_VALUE, "parse error: invalid vtable"};
    (void)fb.rd<uint8_t>(t.vt + t.vsize - 1);
    return t;
  }
  // Absolute position of a field, 0 when absent.
  size_t field(int slot) const {
    const size_t vo = 4 + 2 * (size_t)slot;
    if (vo + 2 > vsize) return 0;
    const uint16_t off = fb->rd<uint16_t>(vt + vo);
    return off ? pos + off : 0;
  }
  template <typename T>
  T scalar(int slot, T dflt) const {
    const size_t f = field(slot);
    return f ? fb->rd<T>(f) : dflt;
  }
  bool has(int slot) const { return field(slot) != 0; }
  size_t ref(int slot) const {  // target of a uoffset field, 0 when absent
    const size_t f = field(slot);
    return f ? f + fb->rd<uint32_t>(f) : 0;
  }
  Table table(int slot) const {
    const size_t r = ref(slot);
    return r ? Table::at(*fb, r) : Table();
  }
  // Vector field: element count and position of element 0.
  bool vec(int slot, uint32_t& len, size_t& data, size_t elem) const {
    const size_t r = ref(slot);
    if (!r) return false;
    len = fb->rd<uint32_t>(r);
    data = r + 4;
    if (!fb->in(data, (size_t)len * elem)) throw LoadError{RTENHIP_INVALID_VALUE, "parse error: range out of bounds"};
    return true;
  }
  template <typename T>
  bool vec_of(int slot, std::vector<T>& out) const {
    uint32_t len;
    size_t data;
    if (!vec(slot, len, data, sizeof(T))) return false;
    out.resize(len);
    if (len) std::memcpy(out.data(), fb->p + data, (size_t)len * sizeof(T));
    return true;
  }
  bool str(int slot, std::string& out) const {
    uint32_t len;
    size_t data;
    if (!vec(slot, len, data, 1)) return false;
    out.assign(reinterpret_cast<const char*>(fb->p + data), len);
    return true;
  }
  Table vec_table(size_t data, uint32_t i) const {
    const size_t e = data + 4 * (size_t)i;
    return Table::at(*fb, e + fb->rd<uint32_t>(e));
  }
};

struct PNode {
  NodeKind kind = NodeKind::Value;
  std::string name;
  std::string op_type;
  Attrs attrs;
  std::vector<int> inputs, outputs;
  Shape shape;
  std::vector<float> data;      // Float32 constants
  std::vector<int32_t> idata;   // Int32 constants
  int dtype = RTENHIP_DTYPE_FLOAT32;
};

struct PModel {
  std::vector<PNode> nodes;
  std::vector<int> inputs, outputs;
};

std::vector<double> to_d(const std::vector<uint32_t>& v) { return std::vector<double>(v.begin(), v.end()); }

[[noreturn]] void attr_error() {
  throw LoadError{RTENHIP_INVALID_VALUE, "operator error: invalid attributes for operator"};
}

// Padding attrs (padding_from_attrs, op_registry.rs:239-245): auto_pad Same ->
// "same"; NotSet with pads -> those pads; otherwise four zeros.
void read_padding(const Table& a, int auto_pad_slot, int pads_slot, Attrs& out) {
  const uint8_t auto_pad = a.scalar<uint8_t>(auto_pad_slot, 0);  // AutoPad default Same
  std::vector<uint32_t> pads;
  if (auto_pad == 0) {
    out.strs["auto_pad"] = "same";
  } else if (a.vec_of(pads_slot, pads)) {
    out.nums["pads"] = to_d(pads);
  } else {
    out.nums["pads"] = {0, 0, 0, 0};
  }
}

// ReadOp::read for the operators this backend registers (op_registry.rs:296-820).
void read_op(const std::string& type, uint8_t attrs_type, const Table& a, Attrs& out) {
  auto need = [&](uint8_t t) {
    if (attrs_type != t || !a) attr_error();
  };
  std::vector<uint32_t> u;
  if (type == "Conv") {
    need(kConvAttrs);
    read_padding(a, 0, 1, out);
    out.nums["groups"] = {(double)a.scalar<uint32_t>(2, 0)};
    out.nums["strides"] = a.vec_of(3, u) ? to_d(u) : std::vector<double>{1, 1};
    out.nums["dilations"] = a.vec_of(4, u) ? to_d(u) : std::vector<double>{1, 1};
  } else if (type == "ConvTranspose") {
    // ConvTransposeAttrs: strides (default [1, 1]), auto_pad (default NotSet), pads.
    need(kConvTransposeAttrs);
    out.nums["strides"] = a.vec_of(0, u) ? to_d(u) : std::vector<double>{1, 1};
    const uint8_t auto_pad = a.scalar<uint8_t>(1, 1);
    if (auto_pad == 0)
      out.strs["auto_pad"] = "same";
    else
      out.nums["pads"] = a.vec_of(2, u) ? to_d(u) : std::vector<double>{0, 0, 0, 0};
  } else if (type == "MaxPool" || type == "AveragePool") {
    need(type == "MaxPool" ? kMaxPoolAttrs : kAveragePoolAttrs);
    if (!a.vec_of(0, u) || u.size() < 2) attr_error();  // kernel_size (required)
    out.nums["kernel_size"] = {(double)u[0], (double)u[1]};
    read_padding(a, 1, 2, out);
    if (a.vec_of(3, u)) {
      if (u.size() < 2) attr_error();
      out.nums["strides"] = {(double)u[0], (double)u[1]};
    } else {
      out.nums["strides"] = {1, 1};
    }
    if (type == "AveragePool") out.nums["count_include_pad"] = {(double)a.scalar<uint8_t>(4, 0)};
  } else if (type == "BatchNormalization" || type == "InstanceNormalization") {
    // (InstanceNormalization reads BatchNormalizationAttrs, op_registry.rs:556-564)
    need(kBatchNormalizationAttrs);
    out.nums["epsilon"] = {(double)a.scalar<float>(0, 0.f)};
  } else if (type == "Gemm") {
    need(kGemmAttrs);
    out.nums["alpha"] = {(double)a.scalar<float>(0, 0.f)};
    out.nums["beta"] = {(double)a.scalar<float>(1, 0.f)};
    out.nums["transA"] = {(double)a.scalar<uint8_t>(2, 0)};
    out.nums["transB"] = {(double)a.scalar<uint8_t>(3, 0)};
  } else if (type == "Flatten") {
    need(kFlattenAttrs);
    out.nums["axis"] = {(double)a.scalar<int32_t>(0, 0)};
  } else if (type == "Softmax" || type == "LogSoftmax") {
    // (LogSoftmax reads SoftmaxAttrs, op_registry.rs:587)
    need(kSoftmaxAttrs);
    out.nums["axis"] = {(double)a.scalar<int32_t>(0, 0)};
  } else if (type == "LayerNormalization") {
    need(kLayerNormalizationAttrs);
    out.nums["axis"] = {(double)a.scalar<int32_t>(0, 0)};
    out.nums["epsilon"] = {(double)a.scalar<float>(1, 0.f)};
  } else if (type == "Transpose") {
    need(kTransposeAttrs);
    if (a.vec_of(0, u)) out.nums["perm"] = to_d(u);
  } else if (type == "Reshape") {
    need(kReshapeAttrs);
    out.nums["allowzero"] = {(double)a.scalar<uint8_t>(0, 0)};
  } else if (type == "Gelu") {
    need(kGeluAttrs);
  } else if (type == "Gather") {
    need(kGatherAttrs);  // impl_read_op!(Gather, attrs_as_gather_attrs, axis)
    out.nums["axis"] = {(double)a.scalar<int32_t>(0, 0)};
  } else if (type == "Cast") {
    need(kCastAttrs);  // op_registry.rs:421-428: DataType::Int32, anything else Float
    out.nums["to"] = {a.scalar<uint8_t>(0, 0) == 0 ? (double)RTENHIP_DTYPE_INT32
                                                   : (double)RTENHIP_DTYPE_FLOAT32};
  } else if (type == "Concat") {
    need(kConcatAttrs);  // impl_read_op!(Concat, attrs_as_concat_attrs, axis)
    out.nums["axis"] = {(double)a.scalar<int32_t>(0, 0)};
  } else if (type == "ReduceMean") {
    // impl_read_op!(.., reduce_axes) (op_registry.rs:351-366): axes optional
    need(kReduceMeanAttrs);
    std::vector<int32_t> ax;
    if (a.vec_of(0, ax)) out.nums["axes"] = std::vector<double>(ax.begin(), ax.end());
    out.nums["keep_dims"] = {(double)a.scalar<uint8_t>(1, 0)};
  } else if (type == "ConstantOfShape") {
    // op_registry.rs:444-456: value union Scalar {IntScalar = 1, FloatScalar = 2},
    // Scalar::Int(0) when neither.
    need(kConstantOfShapeAttrs);
    const uint8_t vt = a.scalar<uint8_t>(0, 0);
    const Table v = a.table(1);
    if (vt == 2 && v) {
      out.strs["dtype"] = "float";
      out.nums["value"] = {(double)v.scalar<float>(0, 0.f)};
    } else {
      out.strs["dtype"] = "int32";
      out.nums["value"] = {vt == 1 && v ? (double)v.scalar<int32_t>(0, 0) : 0.0};
    }
  } else {
    static const char* const no_attrs[] = {"Add", "Sub", "Mul", "Div", "Clip", "Relu", "Erf",
                                           "Exp", "Sigmoid", "Tanh", "MatMul", "Identity",
                                           "GlobalAveragePool", "Where", "Unsqueeze", "Squeeze",
                                           "Pow", "Sqrt", "Shape", "Slice", "Expand"};
    for (const char* t : no_attrs)
      if (type == t) return;
    throw LoadError{RTENHIP_UNSUPPORTED_VALUE,
                    "operator error: operator " + type + " is not supported or not enabled"};
  }
}

// Header::from_buf (header.rs:84-131).  Returns false for a V1 file (no magic).
bool read_header(const uint8_t* b, size_t n, uint64_t& model_off, uint64_t& model_len,
                 uint64_t& tensor_off) {
  if (n < 4) throw LoadError{RTENHIP_INVALID_VALUE, "invalid header: header is too short"};
  if (std::memcmp(b, "RTEN", 4) != 0) return false;
  if (n < 32) throw LoadError{RTENHIP_INVALID_VALUE, "invalid header: header is too short"};
  uint32_t version;
  std::memcpy(&version, b + 4, 4);
  if (version != 2) throw LoadError{RTENHIP_INVALID_VALUE, "invalid header: unsupported file version"};
  std::memcpy(&model_off, b + 8, 8);
  std::memcpy(&model_len, b + 16, 8);
  std::memcpy(&tensor_off, b + 24, 8);
  if (model_off < 32 || model_off > n)
    throw LoadError{RTENHIP_INVALID_VALUE, "invalid header: segment offset is invalid"};
  if (model_len > n - model_off)
    throw LoadError{RTENHIP_INVALID_VALUE, "invalid header: segment length is invalid"};
  if (tensor_off < 32 || tensor_off > n)
    throw LoadError{RTENHIP_INVALID_VALUE, "invalid header: segment offset is invalid"};
  return true;
}

PModel parse(const uint8_t* bytes, size_t len) {
  if (!bytes) throw LoadError{RTENHIP_MISSING_INPUTS, "read error: no data"};
  uint64_t model_off = 0, model_len = len, tensor_off = 0;
  const bool v2 = read_header(bytes, len, model_off, model_len, tensor_off);
  Fb fb{bytes + model_off, (size_t)model_len};
  const Table model = Table::at(fb, fb.rd<uint32_t>(0));
  if (model.scalar<int32_t>(0, 0) != 1) throw LoadError{RTENHIP_INVALID_VALUE, "unsupported schema version"};
  const Table graph = model.table(1);
  if (!graph) throw LoadError{RTENHIP_INVALID_VALUE, "parse error: missing required field `graph`"};
  PModel pm;
  std::vector<uint32_t> ids;
  if (graph.vec_of(1, ids)) pm.inputs.assign(ids.begin(), ids.end());
  if (graph.vec_of(2, ids)) pm.outputs.assign(ids.begin(), ids.end());
  if (graph.has(3) && graph.vec_of(3, ids) && !ids.empty())
    throw LoadError{RTENHIP_UNSUPPORTED_VALUE, "graph error: captured values (subgraphs) are not supported"};
  uint32_t n_nodes = 0;
  size_t nodes_data = 0;
  if (graph.vec(0, n_nodes, nodes_data, 4)) {
    pm.nodes.resize(n_nodes);
    for (uint32_t i = 0; i < n_nodes; i++) {
      const Table node = graph.vec_table(nodes_data, i);
      PNode& pn = pm.nodes[i];
      node.str(0, pn.name);
      const uint8_t kind = node.scalar<uint8_t>(1, 0);
      const Table data = node.table(2);
      if (kind == kOperatorNode && data) {
        pn.kind = NodeKind::Operator;
        const uint8_t t = data.scalar<uint8_t>(0, 0);
        if (t >= kNumOpTypes)
          throw LoadError{RTENHIP_UNSUPPORTED_VALUE, "operator error: operator is not supported or not enabled"};
        pn.op_type = kOpTypes[t];
        read_op(pn.op_type, data.scalar<uint8_t>(1, 0), data.table(2), pn.attrs);
        std::vector<int32_t> v;
        auto link = [&](int slot, std::vector<int>& out, const char* what) {
          if (!data.vec_of(slot, v)) return;
          for (int32_t id : v) {
            if (id >= (int32_t)i)
              throw LoadError{RTENHIP_INVALID_VALUE, std::string("graph error: operator ") + what + " is invalid"};
            out.push_back(id < 0 ? -1 : id);
          }
        };
        link(3, pn.inputs, "input");
        link(4, pn.outputs, "output");
        for (int o : pn.outputs)
          if (o < 0 || pm.nodes[o].kind != NodeKind::Value)
            throw LoadError{RTENHIP_INVALID_VALUE, "graph error: operator output is invalid"};
      } else if (kind == kValueNode && data) {
        pn.kind = NodeKind::Value;
      } else if (kind == kConstantNode && data) {
        pn.kind = NodeKind::Constant;
        std::vector<uint32_t> shape;
        if (!data.vec_of(0, shape)) throw LoadError{RTENHIP_INVALID_VALUE, "parse error: missing required field `shape`"};
        pn.shape.assign(shape.begin(), shape.end());
        // Element count and byte size with overflow checks: a file whose dims
        // multiply past 2^62 elements is malformed, not a huge allocation.
        uint64_t count64 = 1;
        for (uint32_t dim : shape)
          if (__builtin_mul_overflow(count64, (uint64_t)dim, &count64) || count64 > (UINT64_MAX >> 2))
            throw LoadError{RTENHIP_INVALID_VALUE, "graph error: constant shape is too large"};
        const size_t count = (size_t)count64;
        if (data.has(4)) {
          // External data in the tensor segment (model.rs:477-503).
          if (!v2) throw LoadError{RTENHIP_INVALID_VALUE, "graph error: tensor data section missing"};
          const uint64_t off = tensor_off + data.scalar<uint64_t>(4, 0);
          const uint16_t dtype = data.scalar<uint16_t>(3, 0xffff);
          if (dtype != 0 && dtype != 1)
            throw LoadError{RTENHIP_INVALID_VALUE, "graph error: unsupported data type for external constant"};
          if (off > len || count * 4 > len - off)
            throw LoadError{RTENHIP_INVALID_VALUE, "graph error: invalid tensor data offset"};
          if (dtype == 1) {
            pn.data.resize(count);
            if (count) std::memcpy(pn.data.data(), bytes + off, count * 4);
          } else {
            pn.dtype = RTENHIP_DTYPE_INT32;
            pn.idata.resize(count);
            if (count) std::memcpy(pn.idata.data(), bytes + off, count * 4);
          }
        } else {
          // Inline FloatData / IntData (model.rs:504-520).
          const uint8_t ct = data.scalar<uint8_t>(1, 0);
          const Table cd = data.table(2);
          if (!cd || (ct != kFloatData && ct != kIntData))
            throw LoadError{RTENHIP_INVALID_VALUE, "graph error: unsupported data type for inline constant"};
          uint32_t n;
          size_t d;
          if (!cd.vec(0, n, d, 4)) throw LoadError{RTENHIP_INVALID_VALUE, "parse error: missing required field `data`"};
          if (n != count) throw LoadError{RTENHIP_INVALID_VALUE, "graph error: constant data does not match its shape"};
          if (ct == kFloatData) {
            pn.data.resize(n);
            if (n) std::memcpy(pn.data.data(), fb.p + d, (size_t)n * 4);
          } else {
            pn.dtype = RTENHIP_DTYPE_INT32;
            pn.idata.resize(n);
            for (uint32_t k = 0; k < n; k++) pn.idata[k] = fb.rd<int32_t>(d + 4 * (size_t)k);
          }
        }
      } else {
        throw LoadError{RTENHIP_INVALID_VALUE, "graph error: unknown node type"};
      }
    }
  }
  for (int id : pm.inputs)
    if (id < 0 || id >= (int)pm.nodes.size()) throw LoadError{RTENHIP_INVALID_VALUE, "graph error: invalid input id"};
  for (int id : pm.outputs)
    if (id < 0 || id >= (int)pm.nodes.size()) throw LoadError{RTENHIP_INVALID_VALUE, "graph error: invalid output id"};
  return pm;
}

std::string describe(const PModel& pm) {
  std::string s;
  auto ints = [](const std::vector<int>& v) {
    std::string r;
    for (size_t i = 0; i < v.size(); i++) r += (i ? "," : "") + std::to_string(v[i]);
    return r;
  };
  s += "inputs " + ints(pm.inputs) + "\noutputs " + ints(pm.outputs) + "\n";
  for (size_t i = 0; i < pm.nodes.size(); i++) {
    const PNode& n = pm.nodes[i];
    s += std::to_string(i) + " ";
    if (n.kind == NodeKind::Value) {
      s += "value " + n.name + "\n";
    } else if (n.kind == NodeKind::Constant) {
      std::string sh;
      for (size_t k = 0; k < n.shape.size(); k++) sh += (k ? "x" : "") + std::to_string(n.shape[k]);
      double sum = 0;
      for (float v : n.data) sum += v;
      for (int32_t v : n.idata) sum += v;
      char buf[64];
      snprintf(buf, sizeof buf, " sum=%.9g", sum);
      s += "const " + n.name + " " + sh + (n.dtype == RTENHIP_DTYPE_INT32 ? " i32" : "") + buf + "\n";
    } else {
      s += "op " + n.name + " " + n.op_type + " in=" + ints(n.inputs) + " out=" + ints(n.outputs);
      for (auto& kv : n.attrs.nums) {
        s += " " + kv.first + "=";
        for (size_t k = 0; k < kv.second.size(); k++) {
          char buf[32];
          snprintf(buf, sizeof buf, "%s%.9g", k ? "," : "", kv.second[k]);
          s += buf;
        }
      }
      for (auto& kv : n.attrs.strs) s += " " + kv.first + "=" + kv.second;
      s += "\n";
    }
  }
  return s;
}

}  // namespace
}  // namespace rtenhip

using namespace rtenhip;

extern "C" {

rtenhip_graph* rtenhip_model_load_with_options(rtenhip_ctx* ctx, const uint8_t* bytes, size_t len,
                                               int optimize) {
  PModel pm;
  try {
    pm = parse(bytes, len);
  } catch (const LoadError& e) {
    set_error(e.code, e.msg);
    return nullptr;
  } catch (const std::exception& e) {
    // bad_alloc / length_error from a malformed size: a load error, never an
    // exception across the C ABI.
    set_error(RTENHIP_INVALID_VALUE, std::string("read error: ") + e.what());
    return nullptr;
  }
  rtenhip_graph* g = rtenhip_graph_create(ctx);
  for (size_t i = 0; i < pm.nodes.size(); i++) {
    const PNode& n = pm.nodes[i];
    int32_t id = -1;
    if (n.kind == NodeKind::Value) {
      id = rtenhip_graph_add_value(g, n.name.c_str());
    } else if (n.kind == NodeKind::Constant) {
      id = n.dtype == RTENHIP_DTYPE_INT32
               ? rtenhip_graph_add_constant_i32(g, n.name.c_str(), n.idata.data(), n.shape.data(),
                                                (int32_t)n.shape.size())
               : rtenhip_graph_add_constant(g, n.name.c_str(), n.data.data(), n.shape.data(),
                                            (int32_t)n.shape.size());
    } else {
      Node node;
      node.kind = NodeKind::Operator;
      node.name = n.name;
      node.op_type = n.op_type;
      node.attrs = n.attrs;
      node.inputs = n.inputs;
      node.outputs = n.outputs;
      id = reinterpret_cast<Graph*>(g)->add_node(std::move(node));
    }
    if (id != (int32_t)i) {
      if (id >= 0) set_error(RTENHIP_INVALID_VALUE, "graph error: node ids out of order");
      rtenhip_graph_destroy(g);
      return nullptr;
    }
  }
  rtenhip_status st = rtenhip_graph_set_io(g, pm.inputs.data(), (int32_t)pm.inputs.size(),
                                           pm.outputs.data(), (int32_t)pm.outputs.size());
  if (!st && optimize) st = rtenhip_graph_optimize(g);
  if (st) {
    rtenhip_graph_destroy(g);
    return nullptr;
  }
  return g;
}

rtenhip_graph* rtenhip_model_load(rtenhip_ctx* ctx, const uint8_t* bytes, size_t len) {
  return rtenhip_model_load_with_options(ctx, bytes, len, 1);
}

const char* rtenhip_model_describe(const uint8_t* bytes, size_t len) {
  static thread_local std::string out;
  try {
    out = describe(parse(bytes, len));
  } catch (const LoadError& e) {
    set_error(e.code, e.msg);
    return nullptr;
  } catch (const std::exception& e) {
    set_error(RTENHIP_INVALID_VALUE, std::string("read error: ") + e.what());
    return nullptr;
  }
  return out.c_str();
}

}  // extern "C"
