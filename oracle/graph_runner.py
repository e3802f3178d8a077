"""Run a ModelSpec on the CPU oracle, op by op, exactly as RTen's Graph::run
would (src/graph.rs:797-1073): topological order, no fusion.

TEST INFRASTRUCTURE ONLY (parity checker and cpu_baseline timing).
"""
from __future__ import annotations

import numpy as np

import extra_ops as X
import optimizer
import rten_oracle as O


def _clip_bounds(env, node):
    lo = hi = None
    if len(node.inputs) > 1 and node.inputs[1] is not None:
        lo = float(np.asarray(env[node.inputs[1]]).reshape(-1)[0])
    if len(node.inputs) > 2 and node.inputs[2] is not None:
        hi = float(np.asarray(env[node.inputs[2]]).reshape(-1)[0])
    lo = node.attrs.get("min", lo)
    hi = node.attrs.get("max", hi)
    return lo, hi


def run_op(node, ins):
    t, a = node.op_type, node.attrs
    x = ins[0]
    if t == "Conv":
        return O.conv(x, ins[1], ins[2] if len(ins) > 2 else None, pads=a.get("pads", (0, 0, 0, 0)),
                      strides=a.get("strides", (1, 1)), dilations=a.get("dilations", (1, 1)),
                      groups=a.get("groups", 1),
                      padding="same" if a.get("auto_pad", "notset").lower() in ("same", "same_upper") else "fixed")
    if t == "ConvTranspose":
        one_d = x.ndim == 3
        return O.conv_transpose(x, ins[1], ins[2] if len(ins) > 2 else None,
                                pads=a.get("pads", (0, 0) if one_d else (0, 0, 0, 0)),
                                strides=a.get("strides", (1,) if one_d else (1, 1)),
                                padding="same" if a.get("auto_pad", "notset").lower() in ("same", "same_upper") else "fixed")
    if t in ("Relu", "Gelu", "Erf", "Sigmoid", "Tanh", "Exp", "Silu"):
        return O.unary(t, x)
    if t in ("Add", "Sub", "Mul", "Div"):
        if np.asarray(x).dtype == np.int32 or np.asarray(ins[1]).dtype == np.int32:
            if np.asarray(x).dtype != np.asarray(ins[1]).dtype:
                raise O.OpError(1, "Input 1 has incorrect type")
            return X.int_binary(t, x, ins[1])
        return O.binary(t, x, ins[1])
    if t == "Pow":
        return X.pow_(x, ins[1])
    if t == "Sqrt":
        return X.sqrt(x)
    if t == "ReduceMean":
        axes = a.get("axes")
        if len(ins) > 1 and ins[1] is not None:  # get_axes: the axes input wins (reduce.rs:534-543)
            axes = [int(v) for v in np.asarray(ins[1]).reshape(-1)]
        return X.reduce_mean(x, axes, bool(a.get("keep_dims", 0)))
    if t == "Shape":
        return X.shape(x)
    if t == "ConstantOfShape":
        return X.constant_of_shape(x, a.get("value", 0))
    if t == "Concat":
        return X.concat(ins, int(a.get("axis", 0)))
    if t == "Slice":
        return X.slice_(x, ins[1], ins[2], ins[3] if len(ins) > 3 else None, ins[4] if len(ins) > 4 else None)
    if t == "Expand":
        return X.expand(x, ins[1])
    if t == "MaxPool":
        return O.max_pool(x, a["kernel_size"], a.get("strides", (1, 1)), a.get("pads", (0, 0, 0, 0)))
    if t == "AveragePool":
        return O.average_pool(x, a["kernel_size"], a.get("strides", (1, 1)),
                              a.get("pads", (0, 0, 0, 0)), bool(a.get("count_include_pad", 0)))
    if t == "GlobalAveragePool":
        return O.global_average_pool(x)
    if t == "Flatten":
        ax = a.get("axis", 1)
        return x.reshape(int(np.prod(x.shape[:ax])), -1)
    if t == "Gemm":
        return O.gemm_op(x, ins[1], ins[2] if len(ins) > 2 else None, a.get("alpha", 1.0),
                         a.get("beta", 1.0), bool(a.get("transA", 0)), bool(a.get("transB", 0)))
    if t == "MatMul":
        return O.matmul(x, ins[1])
    if t == "BatchNormalization":
        return O.batch_norm(x, ins[1], ins[2], ins[3], ins[4], a.get("epsilon", 1e-5))
    if t == "LayerNormalization":
        return O.layer_norm(x, ins[1], ins[2] if len(ins) > 2 else None, a.get("axis", -1),
                            a.get("epsilon", 1e-5))
    if t == "Softmax":
        return O.softmax(x, a.get("axis", -1))
    if t == "LogSoftmax":
        return O.log_softmax(x, a.get("axis", -1))
    if t == "InstanceNormalization":
        return O.instance_norm(x, ins[1], ins[2], a.get("epsilon", 1e-5))
    if t == "Transpose":
        return np.ascontiguousarray(np.transpose(x, a.get("perm")))
    if t == "Reshape":
        shape = [int(v) for v in np.asarray(ins[1]).reshape(-1)]
        shape = [x.shape[i] if (d == 0 and not a.get("allowzero", 0)) else d for i, d in enumerate(shape)]
        return x.reshape(shape)
    if t == "Identity":
        return x
    if t == "Gather":
        return O.gather(x, ins[1], int(a.get("axis", 0)))
    if t == "Where":
        return O.where(x, ins[1], ins[2])
    if t == "Cast":
        # CastAttrs::to: 0 = Int32 (the schema default), 1 = Float (schema.fbs DataType)
        to_int = int(a.get("to", 0)) == 0
        if to_int:
            return x.astype(np.int32) if x.dtype == np.int32 else O.cast_f32_to_i32(x)
        return x.astype(np.float32) if x.dtype == np.float32 else O.cast_i32_to_f32(x)
    if t == "Unsqueeze":
        # unsqueeze_in_place (src/ops/layout.rs:522-548)
        nd = x.ndim + np.asarray(ins[1]).size
        axes = sorted(int(v) % nd for v in np.asarray(ins[1]).reshape(-1))
        out = x
        for ax in axes:
            out = np.expand_dims(out, ax)
        return out
    if t == "Squeeze":
        if len(ins) > 1 and ins[1] is not None:
            return np.squeeze(x, axis=tuple(int(v) % x.ndim for v in np.asarray(ins[1]).reshape(-1)))
        return np.squeeze(x)
    raise NotImplementedError(t)


_OPT_CACHE = {}


def optimized(spec):
    """The graph RTen runs after Model::load's optimizer (oracle/optimizer.py),
    cached per spec object."""
    key = id(spec)
    hit = _OPT_CACHE.get(key)
    if hit is None or hit[0] is not spec:
        hit = (spec, optimizer.optimize(spec, _run_node))
        _OPT_CACHE[key] = hit
    return hit[1]


def _run_node(n, ins):
    if n.op_type == "Clip":
        env = {}
        names = []
        for k, v in enumerate(ins):
            env[f"#{k}"] = v
            names.append(f"#{k}" if v is not None else None)
        lo, hi = _clip_bounds(env, type("N", (), {"inputs": names, "attrs": n.attrs})())
        return O.clip(ins[0], lo, hi)
    return run_op(n, ins)


def _live(spec, outs):
    prod = {o: n for n in spec.nodes if n.kind == "op" for o in n.outputs}
    seen, stack = set(), list(outs)
    while stack:
        n = prod.get(stack.pop())
        if n is not None and n.name not in seen:
            seen.add(n.name)
            stack.extend(i for i in n.inputs if i is not None)
    return seen


def run(spec, inputs: dict, outputs=None, optimize: bool = True):
    """inputs: {value name: np.ndarray}; returns {output name: np.ndarray}.
    optimize: run the graph as RTen's optimizer leaves it (the default of
    ModelOptions, src/model.rs:155-207), or as stored."""
    if optimize:
        spec = optimized(spec)
    outs = outputs or spec.outputs
    live = _live(spec, outs)
    env = {n.name: n.data for n in spec.nodes if n.kind == "const"}
    env.update({k: np.ascontiguousarray(v, np.int32 if np.asarray(v).dtype == np.int32 else np.float32)
                for k, v in inputs.items()})
    for n in spec.nodes:
        if n.kind != "op" or n.name not in live:
            continue
        if n.op_type == "Clip":
            lo, hi = _clip_bounds(env, n)
            env[n.outputs[0]] = O.clip(env[n.inputs[0]], lo, hi)
            continue
        ins = [env[i] if i is not None else None for i in n.inputs]
        env[n.outputs[0]] = run_op(n, ins)
    return {o: env[o] for o in outs}
