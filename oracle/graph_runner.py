"""Run a ModelSpec on the CPU oracle, op by op, exactly as RTen's Graph::run
would (src/graph.rs:797-1073): topological order, no fusion.

TEST INFRASTRUCTURE ONLY (parity checker and cpu_baseline timing).
"""
from __future__ import annotations

import numpy as np

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
        return O.binary(t, x, ins[1])
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


def run(spec, inputs: dict, outputs=None):
    """inputs: {value name: np.ndarray}; returns {output name: np.ndarray}."""
    env = {n.name: n.data for n in spec.nodes if n.kind == "const"}
    env.update({k: np.ascontiguousarray(v, np.int32 if np.asarray(v).dtype == np.int32 else np.float32)
                for k, v in inputs.items()})
    for n in spec.nodes:
        if n.kind != "op":
            continue
        if n.op_type == "Clip":
            lo, hi = _clip_bounds(env, n)
            env[n.outputs[0]] = O.clip(env[n.inputs[0]], lo, hi)
            continue
        ins = [env[i] if i is not None else None for i in n.inputs]
        env[n.outputs[0]] = run_op(n, ins)
    outs = outputs or spec.outputs
    return {o: env[o] for o in outs}
