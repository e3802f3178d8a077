"""Restatement of RTen's load-time graph optimizer (src/optimize.rs:286-518 and
src/optimize/pattern_matcher.rs) over a ModelSpec, so the oracle runs the
graph RTen would run after ``Model::load`` (ModelOptions::enable_optimization
defaults to true, src/model.rs:155-207).

TEST INFRASTRUCTURE ONLY (the parity checker's view of the graph).

Passes, in the reference's order (optimize.rs:286-297):
  propagate_constants  every operator whose inputs are all constants (after
                       pruning, graph.rs:1185-1234) is evaluated once and its
                       leaf outputs become constants;
  fuse_transpose       MatMul(Transpose(X), ..) reads X through a permuted view
                       (numerically identical, so the oracle only renames it);
  fuse_silu            x * Sigmoid(x)                         -> Silu(x)
  fuse_gelu            x * (Erf(x / sqrt(2)) + 1) * 0.5       -> Gelu(x)
  fuse_layer_norm      (x - mean) / Sqrt(eps + mean(pow(x - mean, 2))) * scale
                       + bias (ReduceMean over axis -1 only)  -> LayerNormalization
A fused operator replaces the subgraph's final node in place (it keeps that
node's name and output value, like Fusion::apply + replace_value); the
intermediate nodes stay and are pruned when nothing reads them.
"""
from __future__ import annotations

import copy
from typing import Dict, List, Optional

import numpy as np

CONST_TOLERANCE = 1e-4  # pattern_matcher.rs:70
COMMUTATIVE = {"Add", "Mul", "And", "Or", "Xor", "Equal"}  # Operator::is_commutative


# ---------------------------------------------------------------- patterns
class Sym:
    def __init__(self, name, const=False):
        self.name, self.const = name, const


class Const:
    def __init__(self, value):
        self.value = float(value)


class Op:
    def __init__(self, name, inputs, key=None):
        self.name, self.inputs, self.key = name, list(inputs), key


def _wrap(p):
    return p if isinstance(p, (Sym, Const, Op)) else Const(p)


def binop(name, a, b):
    return Op(name, [_wrap(a), _wrap(b)])


class _Graph:
    """Views of a ModelSpec the matcher needs: producers and constants."""

    def __init__(self, spec):
        self.spec = spec
        self.producer = {}
        self.consts = {}
        for n in spec.nodes:
            if n.kind == "op":
                for o in n.outputs:
                    self.producer[o] = n
            elif n.kind == "const":
                self.consts[n.name] = n.data


def _test(pat, vid, g: _Graph, syms: List):
    """Pattern::test_impl (pattern_matcher.rs:188-238) on value / constant `vid`."""
    if isinstance(pat, Op):
        op = g.producer.get(vid)
        if op is None:
            return False
        if not _op_matches(pat, op, g, syms):
            return False
        if pat.key:
            syms.append((pat.key, op.name))
        return True
    if isinstance(pat, Const):
        c = g.consts.get(vid)
        if c is None or c.dtype != np.float32 or c.size != 1:
            return False
        return abs(float(c.reshape(-1)[0]) - pat.value) <= CONST_TOLERANCE
    # Symbol: a value or a constant (const symbols: constants only)
    if pat.const and vid not in g.consts:
        return False
    for name, node in syms:
        if name == pat.name:
            return node == vid
    syms.append((pat.name, vid))
    return True


def _op_matches(pat: Op, op, g, syms):
    """OpPattern::matches (pattern_matcher.rs:102-137)."""
    if op.op_type != pat.name or len(pat.inputs) != len(op.inputs):
        return False
    if op.op_type in COMMUTATIVE and len(pat.inputs) == 2 and all(i is not None for i in op.inputs):
        mark = len(syms)
        if _test(pat.inputs[0], op.inputs[0], g, syms) and _test(pat.inputs[1], op.inputs[1], g, syms):
            return True
        del syms[mark:]
        return _test(pat.inputs[1], op.inputs[0], g, syms) and _test(pat.inputs[0], op.inputs[1], g, syms)
    for p, i in zip(pat.inputs, op.inputs):
        if i is None or not _test(p, i, g, syms):
            return False
    return True


def _resolved(syms, name):
    for n, v in syms:
        if n == name:
            return v
    return None


def match(pat, vid, g):
    syms = []
    return syms if _test(pat, vid, g, syms) else None


# ---------------------------------------------------------------- passes
def _reachable_ops(spec):
    prod = {o: n for n in spec.nodes if n.kind == "op" for o in n.outputs}
    seen, stack, order = set(), list(spec.outputs), []
    while stack:
        v = stack.pop()
        n = prod.get(v)
        if n is None or n.name in seen:
            continue
        seen.add(n.name)
        stack.extend(i for i in n.inputs if i is not None)
    return seen


NONDETERMINISTIC = {"RandomUniform", "RandomUniformLike", "RandomNormal", "RandomNormalLike", "Dropout"}


def propagate_constants(spec, run_op):
    """optimize.rs:301-327 with Graph::partial_run / prune_plan
    (graph.rs:1147-1234): evaluate the operators reachable from the outputs
    whose inputs are all constants; the leaf values (read by an operator that
    is not evaluable, or a model output) become constant nodes."""
    live = _reachable_ops(spec)
    known = {n.name: n.data for n in spec.nodes if n.kind == "const"}
    evaluated = set()
    leaves_needed = set()
    for n in spec.nodes:
        if n.kind != "op" or n.name not in live:
            continue
        ins = [i for i in n.inputs if i is not None]
        if n.op_type in NONDETERMINISTIC or not all(i in known for i in ins):
            leaves_needed.update(i for i in ins if i in known)
            continue
        outs = run_op(n, [known[i] if i is not None else None for i in n.inputs])
        if not isinstance(outs, (list, tuple)):
            outs = [outs]
        for o, v in zip(n.outputs, outs):
            known[o] = v
            evaluated.add(o)
    leaves = [v for v in evaluated if v in spec.outputs or v in leaves_needed]
    if not leaves:
        return spec
    out = copy.copy(spec)
    out.nodes = []
    leafset = set(leaves)
    for n in spec.nodes:
        if n.kind == "value" and n.name in leafset:
            # the value becomes a constant carrying its computed data
            c = copy.copy(n)
            c.kind, c.data = "const", np.array(known[n.name], order="C", copy=True)
            out.nodes.append(c)
            continue
        if n.kind == "op" and any(o in leafset for o in n.outputs):
            n = copy.copy(n)
            n.outputs = [o if o not in leafset else f"{o}#folded" for o in n.outputs]
        out.nodes.append(n)
    return out


def _rewrite(spec, node_name, op_type, inputs, attrs):
    for n in spec.nodes:
        if n.kind == "op" and n.name == node_name:
            n.op_type, n.inputs, n.attrs = op_type, list(inputs), dict(attrs)
            return


def fuse_transpose(spec):
    """optimize.rs:333-377.  MatMul is the only target; the fused operator is
    named "FusedTranspose(MatMul)".  Numerically the permuted-view read is the
    materialised transpose, so the oracle keeps the Transpose."""
    g = _Graph(spec)
    consumers: Dict[str, list] = {}
    for n in spec.nodes:
        if n.kind == "op":
            for i in n.inputs:
                if i is not None:
                    consumers.setdefault(i, []).append(n)
    for n in list(spec.nodes):
        if n.kind != "op" or n.op_type != "Transpose" or len(n.inputs) != 1 or len(n.outputs) != 1:
            continue
        tgt = consumers.get(n.outputs[0], [])
        if len(tgt) == 1 and tgt[0].op_type == "MatMul" and len(tgt[0].outputs) == 1:
            tgt[0].attrs = dict(tgt[0].attrs, **{"_fused_name": "FusedTranspose(MatMul)"})
    return spec


def fuse_silu(spec):
    """optimize.rs:380-398."""
    x = Sym("x")
    pat = binop("Mul", x, Op("Sigmoid", [x]))
    return _apply(spec, pat, lambda m, op: ("Silu", [_resolved(m, "x")], {}))


def fuse_gelu(spec):
    """optimize.rs:401-424: x * (Erf(x / sqrt(2)) + 1.0) * 0.5."""
    x = Sym("x")
    pat = binop("Mul", binop("Mul", x, binop("Add", Op("Erf", [binop("Div", x, np.float32(2.0) ** 0.5)]), 1.0)),
                0.5)
    return _apply(spec, pat, lambda m, op: ("Gelu", [_resolved(m, "x")], {}))


def fuse_layer_norm(spec):
    """optimize.rs:427-518."""
    x = Sym("x")
    center = binop("Sub", x, Op("ReduceMean", [x], key="center_mean"))
    eps = Sym("epsilon", const=True)
    norm = binop("Div", x, Op("Sqrt", [binop("Add", eps, Op("ReduceMean", [binop("Pow", x, 2.0)],
                                                                key="norm_mean"))]))
    shift_scale = binop("Add", binop("Mul", x, Sym("scale", const=True)), Sym("bias", const=True))

    def fusion(g, op):
        m = match(shift_scale, op.outputs[0], g)
        if m is None:
            return None
        m2 = match(norm, _resolved(m, "x"), g)
        if m2 is None or not _reduces_last_axis(g, _resolved(m2, "norm_mean")):
            return None
        m3 = match(center, _resolved(m2, "x"), g)
        if m3 is None or not _reduces_last_axis(g, _resolved(m3, "center_mean")):
            return None
        e = g.consts.get(_resolved(m2, "epsilon"))
        if e is None or e.size != 1 or e.dtype != np.float32:  # Constant::as_scalar (f32 item)
            return None
        return ("LayerNormalization", [_resolved(m3, "x"), _resolved(m, "scale"), _resolved(m, "bias")],
                {"axis": -1, "epsilon": float(e.reshape(-1)[0])})

    return _apply_fn(spec, fusion)


def _reduces_last_axis(g, op_name):
    """mean_op_reduces_last_axis (optimize.rs:453-474): axes attr == [-1], or
    an axes input that is a constant vector [-1]."""
    op = next(n for n in g.spec.nodes if n.kind == "op" and n.name == op_name)
    axes = op.attrs.get("axes")
    if axes is not None and [int(a) for a in axes] == [-1]:
        return True
    if len(op.inputs) > 1 and op.inputs[1] is not None:
        c = g.consts.get(op.inputs[1])
        return c is not None and c.ndim == 1 and c.dtype == np.int32 and c.tolist() == [-1]
    return False


def _apply(spec, pat, make):
    def fusion(g, op):
        if len(op.outputs) != 1:
            return None
        m = match(pat, op.outputs[0], g)
        return None if m is None else make(m, op)

    return _apply_fn(spec, fusion)


def _apply_fn(spec, fusion):
    """GraphMutator::apply_fusion (optimize.rs:128-143): every fusion is found
    on the unmodified graph first, then all are applied."""
    g = _Graph(spec)
    found = []
    for n in spec.nodes:
        if n.kind == "op" and len(n.outputs) == 1:
            f = fusion(g, n)
            if f is not None:
                found.append((n.name, f))
    for name, (op_type, inputs, attrs) in found:
        _rewrite(spec, name, op_type, inputs, attrs)
    return spec


def optimize(spec, run_op):
    """GraphOptimizer::optimize (optimize.rs:286-297) on a deep copy of spec."""
    s = copy.deepcopy(spec)
    s = propagate_constants(s, run_op)
    s = fuse_transpose(s)
    s = fuse_silu(s)
    s = fuse_gelu(s)
    s = fuse_layer_norm(s)
    return s


def fused_name(node) -> str:
    """Operator::name() of a (possibly fused) node, as the reference's tests see it."""
    return node.attrs.get("_fused_name", node.op_type)
