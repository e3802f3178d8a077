// Plan-time (host) evaluation of the shape subgraph of a graph.
//
// An ONNX export computes Reshape targets, position ids and masks with small
// int32 operator chains on the input's shape (Shape -> Gather -> Unsqueeze ->
// Concat -> Reshape, Slice of a position-id buffer ...).  RTen runs them as
// CPU operators on every Model::run (graph.rs:797-1073); a device plan here is
// specialised to its input shapes, so their results are fixed per plan: they
// are computed once when the plan is made, the operators are never launched,
// and a value a kernel (or the caller) reads is uploaded once.
//
// Semantics follow the reference operators exactly: Shape (layout.rs:347-363),
// Gather (gather.rs:21-76), Unsqueeze / Squeeze / Reshape / Flatten
// (layout.rs), Concat (concat.rs:15-121), Slice (slice.rs:18-65 with
// rten-tensor SliceRange clamping, slice_range.rs:242-331), Expand
// (layout.rs:17-101), ConstantOfShape (generate.rs:28-42), Cast
// (convert.rs:6-17) and Add / Sub / Mul / Div (binary_elementwise.rs; i32
// wrapping arithmetic, f32 IEEE single operations).
#include <algorithm>
#include <cmath>
#include <cstring>

#include "graph.h"

namespace rtenhip {

const HostVal* Graph::host_value(int id, HostVal& tmp) const {
  if (id < 0 || id >= (int)nodes.size()) return nullptr;
  const Node& n = nodes[id];
  if (n.kind == NodeKind::Constant) {
    if (!n.has_host) return nullptr;
    tmp.dtype = n.dtype;
    tmp.shape = n.shape;
    tmp.raw = n.host_raw;
    return &tmp;
  }
  if (planning_host) {
    auto it = planning_host->find(id);
    if (it != planning_host->end()) return &it->second;
  }
  return nullptr;
}

namespace {

std::vector<int64_t> strides_of(const Shape& s) {
  std::vector<int64_t> st(s.size(), 1);
  for (int i = (int)s.size() - 2; i >= 0; i--) st[i] = st[i + 1] * s[i + 1];
  return st;
}

// out[idx] = src[sum idx[d] * src_strides[d] + base] over out_shape.
void strided_copy(const HostVal& src, int64_t base, const std::vector<int64_t>& sst, const Shape& out_shape,
                  std::vector<uint32_t>& out) {
  const int64_t n = prod(out_shape);
  out.resize((size_t)n);
  std::vector<int64_t> idx(out_shape.size(), 0);
  for (int64_t k = 0; k < n; k++) {
    int64_t off = base;
    for (size_t d = 0; d < idx.size(); d++) off += idx[d] * sst[d];
    out[(size_t)k] = src.raw[(size_t)off];
    for (int d = (int)idx.size() - 1; d >= 0; d--) {
      if (++idx[d] < out_shape[d]) break;
      idx[d] = 0;
    }
  }
}

// Rust `as i32` from f32: truncation toward zero, saturating, NaN -> 0.
int32_t f2i_sat(float f) {
  if (std::isnan(f)) return 0;
  if (f >= 2147483648.f) return INT32_MAX;
  if (f <= -2147483648.f) return INT32_MIN;
  return (int32_t)f;
}

uint32_t f2u(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return u;
}

}  // namespace

bool Graph::host_eval(int op_id, const std::vector<const Shape*>& in_shapes, const Shape& out_shape,
                      int out_dtype, HostVal& out, rtenhip_status& st) {
  st = RTENHIP_OK;
  const Node& op = nodes[op_id];
  const std::string& t = op.op_type;
  out.dtype = out_dtype;
  out.shape = out_shape;
  if (t == "Shape") {
    if (in_shapes.empty() || !in_shapes[0]) return false;
    for (int64_t d : *in_shapes[0]) out.raw.push_back((uint32_t)(int32_t)d);
    return true;
  }
  static const char* const kHostOps[] = {"Identity", "Flatten", "Reshape", "Unsqueeze", "Squeeze", "Cast",
                                         "Gather",   "Concat",  "Slice",   "Expand",    "ConstantOfShape",
                                         "Add",      "Sub",     "Mul",     "Div"};
  if (std::none_of(std::begin(kHostOps), std::end(kHostOps), [&](const char* k) { return t == k; }))
    return false;
  if (prod(out_shape) > kHostEvalMax) return false;
  // Every present input must be known on the host.
  std::vector<HostVal> tmps(op.inputs.size());
  std::vector<const HostVal*> in(op.inputs.size(), nullptr);
  for (size_t i = 0; i < op.inputs.size(); i++) {
    if (op.inputs[i] < 0) continue;
    in[i] = host_value(op.inputs[i], tmps[i]);
    if (!in[i]) return false;
  }
  if (in.empty() || !in[0]) return false;
  const HostVal& x = *in[0];
  if (t == "Identity" || t == "Flatten" || t == "Reshape" || t == "Unsqueeze" || t == "Squeeze") {
    out.raw = x.raw;  // row-major data is unchanged by these
    return true;
  }
  if (t == "Cast") {
    out.raw.resize(x.raw.size());
    for (size_t k = 0; k < x.raw.size(); k++) {
      if (x.dtype == out_dtype)
        out.raw[k] = x.raw[k];
      else if (out_dtype == RTENHIP_DTYPE_INT32)
        out.raw[k] = (uint32_t)f2i_sat(HostVal::u2f(x.raw[k]));
      else
        out.raw[k] = f2u((float)(int32_t)x.raw[k]);
    }
    return true;
  }
  if (t == "ConstantOfShape") {
    const bool is_int = op.attrs.str("dtype", "int32") == "int32";
    const double v = op.attrs.num("value", 0);
    out.raw.assign((size_t)prod(out_shape), is_int ? (uint32_t)(int32_t)v : f2u((float)v));
    return true;
  }
  if (t == "Gather") {
    if (!in[1] || in[1]->dtype != RTENHIP_DTYPE_INT32) return false;
    const int64_t nd = (int64_t)x.shape.size();
    int64_t axis = (int64_t)op.attrs.num("axis", 0);
    if (axis < 0) axis += nd;
    const int64_t n = x.shape[axis];
    const std::vector<int64_t> xs = strides_of(x.shape);
    const int64_t outer = prod(x.shape, 0, axis), inner = prod(x.shape, axis + 1);
    const int64_t ni = in[1]->numel();
    out.raw.resize((size_t)(outer * ni * inner));
    for (int64_t o = 0; o < outer; o++)
      for (int64_t j = 0; j < ni; j++) {
        int64_t ix = (int32_t)in[1]->raw[(size_t)j];
        if (ix < 0) ix += n;
        if (ix < 0 || ix >= n) {
          st = fail(RTENHIP_INVALID_VALUE, "Entry in `indices` is out of range");
          return false;
        }
        for (int64_t r = 0; r < inner; r++)
          out.raw[(size_t)((o * ni + j) * inner + r)] = x.raw[(size_t)((o * n + ix) * inner + r)];
      }
    return true;
  }
  if (t == "Concat") {
    int64_t axis = (int64_t)op.attrs.num("axis", 0);
    if (axis < 0) axis += (int64_t)x.shape.size();
    const int64_t outer = prod(out_shape, 0, axis), inner = prod(out_shape, axis + 1);
    out.raw.resize((size_t)prod(out_shape));
    int64_t col = 0;
    const int64_t out_row = out_shape[axis] * inner;
    for (size_t i = 0; i < in.size(); i++) {
      if (!in[i]) continue;
      const int64_t w = in[i]->shape[axis] * inner;
      for (int64_t o = 0; o < outer; o++)
        std::copy(in[i]->raw.begin() + o * w, in[i]->raw.begin() + (o + 1) * w, out.raw.begin() + o * out_row + col);
      col += w;
    }
    return true;
  }
  if (t == "Slice" || t == "Expand") {
    // Both are strided views of x: a base offset and per-dim source strides.
    int64_t base = 0;
    std::vector<int64_t> sst;
    if (t == "Slice") {
      std::vector<int64_t> dims;
      if (!slice_view(*this, op, x.shape, base, dims, sst, st)) return false;
    } else {
      const std::vector<int64_t> xs = strides_of(x.shape);
      const size_t nd = out_shape.size(), off = nd - x.shape.size();
      sst.assign(nd, 0);
      for (size_t d = 0; d < x.shape.size(); d++) sst[d + off] = x.shape[d] == 1 ? 0 : xs[d];
    }
    strided_copy(x, base, sst, out_shape, out.raw);
    return true;
  }
  // Add / Sub / Mul / Div with broadcasting.
  if (!in[1]) return false;
  const HostVal& y = *in[1];
  if (x.dtype != y.dtype) {
    st = fail(RTENHIP_INCORRECT_INPUT_TYPE, "Input 1 has incorrect type");
    return false;
  }
  const size_t nd = out_shape.size();
  auto bst = [&](const HostVal& v) {
    const std::vector<int64_t> vs = strides_of(v.shape);
    std::vector<int64_t> r(nd, 0);
    const size_t off = nd - v.shape.size();
    for (size_t d = 0; d < v.shape.size(); d++) r[d + off] = v.shape[d] == 1 ? 0 : vs[d];
    return r;
  };
  std::vector<uint32_t> xa, ya;
  strided_copy(x, 0, bst(x), out_shape, xa);
  strided_copy(y, 0, bst(y), out_shape, ya);
  out.raw.resize(xa.size());
  for (size_t k = 0; k < xa.size(); k++) {
    if (x.dtype == RTENHIP_DTYPE_INT32) {
      const int32_t a = (int32_t)xa[k], b = (int32_t)ya[k];
      uint32_t r;
      if (t == "Add") {
        r = (uint32_t)a + (uint32_t)b;
      } else if (t == "Sub") {
        r = (uint32_t)a - (uint32_t)b;
      } else if (t == "Mul") {
        r = (uint32_t)((int64_t)a * (int64_t)b);
      } else {
        if (b == 0) {
          st = fail(RTENHIP_INVALID_VALUE, "Division by zero");
          return false;
        }
        r = (a == INT32_MIN && b == -1) ? (uint32_t)INT32_MIN : (uint32_t)(a / b);
      }
      out.raw[k] = r;
    } else {
      const float a = HostVal::u2f(xa[k]), b = HostVal::u2f(ya[k]);
      volatile float r;  // one IEEE single operation, never contracted
      if (t == "Add") r = a + b;
      else if (t == "Sub") r = a - b;
      else if (t == "Mul") r = a * b;
      else r = a / b;
      out.raw[k] = f2u(r);
    }
  }
  return true;
}

// Slice (slice.rs:18-65): the per-dim SliceRange of the inputs, clamped and
// resolved (slice_range.rs:212-331), as a strided view of an input of shape xs:
// base element offset, output dims, source strides (negative for negative
// steps).  Needs starts / ends / axes / steps known on the host.
bool slice_view(const Graph& g, const Node& op, const Shape& xs, int64_t& base, std::vector<int64_t>& out_dims,
                std::vector<int64_t>& sst, rtenhip_status& st) {
  st = RTENHIP_OK;
  HostVal t1, t2, t3, t4;
  auto get = [&](size_t i, HostVal& tmp) -> const HostVal* {
    return i < op.inputs.size() && op.inputs[i] >= 0 ? g.host_value(op.inputs[i], tmp) : nullptr;
  };
  const HostVal* starts = get(1, t1);
  const HostVal* ends = get(2, t2);
  const bool has_axes = op.inputs.size() > 3 && op.inputs[3] >= 0;
  const bool has_steps = op.inputs.size() > 4 && op.inputs[4] >= 0;
  const HostVal* axes = get(3, t3);
  const HostVal* steps = get(4, t4);
  if (!starts || !ends || (has_axes && !axes) || (has_steps && !steps)) return false;
  const int64_t nd = (int64_t)xs.size();
  if (steps)
    for (size_t k = 0; k < steps->raw.size(); k++)
      if (steps->i(k) == 0) {
        st = fail(RTENHIP_INVALID_VALUE, "steps must be non-zero");
        return false;
      }
  std::vector<int64_t> s(nd, 0), e(nd), stp(nd, 1);
  for (int64_t d = 0; d < nd; d++) e[d] = xs[d];
  const size_t n = std::min(starts->raw.size(), ends->raw.size());
  for (size_t i = 0; i < n; i++) {
    int64_t ax = (int64_t)i;
    if (axes) {
      ax = axes->i(i);
      if (ax < -nd || ax >= nd) {
        st = fail(RTENHIP_INVALID_VALUE, "Axis is invalid");
        return false;
      }
      if (ax < 0) ax += nd;
    }
    s[ax] = starts->i(i);
    e[ax] = ends->i(i);
    stp[ax] = steps ? steps->i(i) : 1;
  }
  const std::vector<int64_t> xst = strides_of(xs);
  base = 0;
  out_dims.assign(nd, 0);
  sst.assign(nd, 0);
  for (int64_t d = 0; d < nd; d++) {
    const int64_t len = xs[d], step = stp[d];
    const int64_t lo = step > 0 ? -len : -len - 1, hi = step > 0 ? len : len - 1;
    const int64_t cs = std::max(lo, std::min(hi, s[d])), ce = std::max(lo, std::min(hi, e[d]));
    int64_t first, count;
    if (step > 0) {
      const int64_t rs = cs >= 0 ? cs : len + cs;
      const int64_t re = std::max(rs, ce >= 0 ? ce : len + ce);
      first = rs;
      count = re > rs ? (re - rs + step - 1) / step : 0;
    } else {
      // resolve() counts from the end; index_range maps back (slice_range.rs:318-331)
      const int64_t rs = cs >= 0 ? len - 1 - cs : -cs - 1;
      const int64_t re = std::max(rs, ce >= 0 ? len - 1 - ce : -ce - 1);
      first = len - 1 - rs;
      count = re > rs ? (re - rs + (-step) - 1) / (-step) : 0;
    }
    out_dims[d] = count;
    sst[d] = step * xst[d];
    if (count > 0) base += first * xst[d];
  }
  return true;
}

}  // namespace rtenhip
