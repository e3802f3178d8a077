"""RTen's load-time optimizer (src/optimize.rs) and the operators an ONNX export
feeds it, on the CPU side of the parity harness:

- oracle/extra_ops.py against the reference's own known answers (reduce.rs,
  slice.rs tests) and the reduction order of slice_sum / iter_sum;
- oracle/optimizer.py against the reference's fusion tests
  (optimize.rs:546-716: constant propagation, FusedTranspose, Silu, Gelu,
  LayerNormalization) and pattern matcher tests (pattern_matcher.rs:350-461);
- the unfused BERT spec (LayerNorm / GELU as ONNX primitives, the head
  reshapes through a Shape / Gather / Unsqueeze / Concat subgraph) optimizes
  to the fused operator mix of the fused spec, and runs to the same bits.
"""
import numpy as np
import pytest

import extra_ops as X
import graph_runner
import optimizer as OPT
from rten_oracle import OpError


# ---------------------------------------------------------------- extra ops
def test_reduce_mean_reference_cases():
    """reduce.rs:1030-1113 (test_reduce_mean / _invalid_inputs)."""
    x = np.arange(1, 10, dtype=np.float32).reshape(3, 3)
    assert X.reduce_mean(x, [-1]).tolist() == [2, 5, 8]
    assert X.reduce_mean(x, [-1], keep_dims=True).shape == (3, 1)
    assert X.reduce_mean(x, [0]).tolist() == [4, 5, 6]
    assert X.reduce_mean(x, None).tolist() == 5.0
    assert X.reduce_mean(x, []).tolist() == 5.0
    y = np.array([5, 1, 20, 2, 30, 1, 40, 2, 55, 1, 60, 2], np.float32).reshape(3, 2, 2)
    assert X.reduce_mean(y, [1]).tolist() == [[12.5, 1.5], [35, 1.5], [57.5, 1.5]]
    assert float(X.reduce_mean(np.array(5.0, np.float32), [])) == 5.0
    for bad in ([3], [-3]):
        with pytest.raises(OpError, match="Axis is invalid"):
            X.reduce_mean(x, bad)
    with pytest.raises(OpError, match="Cannot reduce empty tensor"):
        X.reduce_mean(np.zeros(0, np.float32), [0])


def _slice_sum(xs):
    total = np.float32(0)
    for c in range(0, len(xs), 8):
        ch = xs[c:c + 8]
        if len(ch) == 8:
            z = [ch[i] + ch[i + 4] for i in range(4)]
            s = ((z[0] + z[1]) + z[2]) + z[3]
        else:
            s = np.float32(0)
            for v in ch:
                s = s + v
        total = total + s
    return total


def _iter_sum(xs):
    total, i, n = np.float32(0), 0, len(xs)
    while n > 4:
        n -= 4
        total = total + ((xs[i] + xs[i + 1]) + (xs[i + 2] + xs[i + 3]))
        i += 4
    for v in xs[i:]:
        total = total + v
    return total


@pytest.mark.parametrize("shape,axes", [((5, 771), [-1]), ((4, 13, 6), [1]), ((3, 4, 5), [0, 2]),
                                        ((6, 7), None), ((2, 3, 9), [-1, -2])])
def test_reduce_mean_summation_order(shape, axes):
    """Scalar restatements of slice_sum (last axis) and iter_sum (everything
    else, reduce.rs:250-318) give the vectorised oracle's bits."""
    rng = np.random.default_rng(len(shape) * 31 + shape[-1])
    x = (rng.standard_normal(shape) * 100).astype(np.float32)
    got = X.reduce_mean(x, axes, keep_dims=True)
    nd = x.ndim
    res = sorted(a % nd for a in axes) if axes else list(range(nd))
    keep = [d for d in range(nd) if d not in res]
    t = np.transpose(x, keep + res).reshape(-1, int(np.prod([shape[d] for d in res])))
    single_last = res == [nd - 1]
    exp = np.array([(_slice_sum(r) if single_last else _iter_sum(r)) / np.float32(t.shape[1]) for r in t],
                   np.float32)
    assert np.array_equal(got.reshape(-1).view(np.uint32), exp.view(np.uint32))


def test_slice_reference_cases():
    """slice.rs:337-456."""
    x = np.arange(1, 10, dtype=np.int32).reshape(3, 3)
    assert X.slice_(x, [0], [2], [-1]).reshape(-1).tolist() == [1, 2, 4, 5, 7, 8]
    assert X.slice_(x, [0], [2], [-2]).reshape(-1).tolist() == [1, 2, 3, 4, 5, 6]
    assert X.slice_(x, [-3], [2], [-1]).reshape(-1).tolist() == [1, 2, 4, 5, 7, 8]
    assert X.slice_(x, [-2], [2], [-1]).reshape(-1).tolist() == [2, 5, 8]
    assert X.slice_(x, [0], [-1], [-1]).reshape(-1).tolist() == [1, 2, 4, 5, 7, 8]
    assert X.slice_(x, [0], [-2], [-1]).reshape(-1).tolist() == [1, 4, 7]
    r = np.random.default_rng(3).random((20, 20), dtype=np.float32)
    assert np.array_equal(X.slice_(r, [-(2 ** 31 - 1), -100], [2 ** 31 - 1, 100]), r)
    # negative steps follow numpy / ONNX semantics
    v = np.arange(10, dtype=np.int32)
    for s, e, st in [(-1, -11, -1), (8, 1, -3), (2 ** 31 - 1, -(2 ** 31), -2), (3, 7, 2)]:
        assert X.slice_(v, [s], [e], None, [st]).tolist() == v[slice(s if s < 2**30 else None,
                                                                        e if e > -2**30 else None, st)].tolist()
    with pytest.raises(OpError, match="steps must be non-zero"):
        X.slice_(v, [0], [1], None, [0])


def test_concat_expand_shape_cases():
    a = np.zeros((2, 3), np.float32)
    b = np.ones((2, 1), np.float32)
    assert X.concat([a, b], -1).shape == (2, 4)
    with pytest.raises(OpError, match="Dimensions must be the same except for concat axis"):
        X.concat([a, b], 0)
    with pytest.raises(OpError, match="Tensors must have the same number of dimensions"):
        X.concat([a, np.zeros(3, np.float32)], 0)
    assert X.expand(np.arange(3, dtype=np.float32).reshape(3, 1), np.array([2, 3, 4], np.int32)).shape == (2, 3, 4)
    with pytest.raises(OpError, match="Cannot broadcast input with target shape"):
        X.expand(np.zeros((3, 2), np.float32), np.array([4, 3], np.int32))
    assert X.shape(np.zeros((4, 5, 6))).tolist() == [4, 5, 6]
    c = X.constant_of_shape(np.array([2, 3], np.int32), 7)
    assert c.dtype == np.int32 and c.tolist() == [[7] * 3] * 2
    assert X.constant_of_shape(np.array([2], np.int32), 0.5).dtype == np.float32
    assert X.int_binary("Div", np.array([-7, 7], np.int32), np.array([2, -2], np.int32)).tolist() == [-3, -3]


def test_pow_fast_paths():
    """powf (binary_elementwise.rs:742-751): exponent 2 is x*x, 3 is x*x*x."""
    x = np.random.default_rng(1).standard_normal(1000).astype(np.float32) * 3
    assert np.array_equal(X.pow_(x, np.float32(2)), x * x)
    assert np.array_equal(X.pow_(x, np.array([3.0], np.float32)), (x * x) * x)
    assert np.allclose(X.pow_(np.abs(x), np.float32(0.256)), np.abs(x).astype(np.float64) ** 0.256, rtol=1e-6)


# ---------------------------------------------------------------- optimizer
def _spec():
    from rten_hip.graph import ModelSpec

    return ModelSpec("t")


def _producer(spec, value):
    return next(n for n in spec.nodes if n.kind == "op" and value in n.outputs)


def test_constant_propagation():
    """optimize.rs:546-601."""
    m = _spec()
    a = m.const("const_a", np.array([1, 2, 3], np.int32))
    b = m.const("const_b", np.array([4, 5, 6], np.int32))
    s1 = m.op("Add", [a, b], name="add_1")
    x = m.value("input")
    m.inputs = ["input"]
    s2 = m.op("Add", [s1, x], name="add_2")
    m.outputs = [s1, s2]
    o = OPT.optimize(m, graph_runner._run_node)
    c = next(n for n in o.nodes if n.name == s1)
    assert c.kind == "const" and c.data.tolist() == [5, 7, 9] and c.data.dtype == np.int32
    assert _producer(o, s2).inputs == [s1, "input"]


def test_fuse_transpose():
    m = _spec()
    i1, i2 = m.value("i1"), m.value("i2")
    m.inputs = [i1, i2]
    t = m.op("Transpose", [i1], name="transpose")
    m.outputs = [m.op("MatMul", [t, i2], name="matmul")]
    o = OPT.optimize(m, graph_runner._run_node)
    n = _producer(o, o.outputs[0])
    assert OPT.fused_name(n) == "FusedTranspose(MatMul)" and n.name == "matmul"


def test_fuse_silu():
    m = _spec()
    x = m.value("x")
    m.inputs = [x]
    s = m.op("Sigmoid", [x], name="sigmoid")
    m.outputs = [m.op("Mul", [x, s], name="mul")]
    o = OPT.optimize(m, graph_runner._run_node)
    n = _producer(o, o.outputs[0])
    assert (n.op_type, n.name, n.inputs) == ("Silu", "mul", [x])


def test_fuse_gelu():
    m = _spec()
    sq = m.const("sqrt2", np.array(np.sqrt(np.float32(2)), np.float32))
    one = m.const("one", np.array(1.0, np.float32))
    half = m.const("half", np.array(0.5, np.float32))
    x = m.value("x")
    m.inputs = [x]
    d = m.op("Div", [x, sq], name="div")
    e = m.op("Erf", [d], name="erf")
    a = m.op("Add", [e, one], name="add")
    mu = m.op("Mul", [x, a], name="mul")
    m.outputs = [m.op("Mul", [mu, half], name="mul_half")]
    o = OPT.optimize(m, graph_runner._run_node)
    n = _producer(o, o.outputs[0])
    assert (n.op_type, n.name, n.inputs) == ("Gelu", "mul_half", [x])


def _layer_norm_spec(eps=1e-6, axes=(-1,), pow_exp=2.0):
    """optimize.rs:663-704 (layer_norm_graph)."""
    m = _spec()
    x = m.value("x")
    m.inputs = [x]
    mean = m.op("ReduceMean", [x], {"axes": list(axes), "keep_dims": 0}, name="mean")
    sub = m.op("Sub", [x, mean], name="sub")
    two = m.const("two", np.array(pow_exp, np.float32))
    p = m.op("Pow", [sub, two], name="pow")
    vm = m.op("ReduceMean", [p], {"axes": list(axes), "keep_dims": 0}, name="var_mean")
    e = m.const("eps", np.array(eps, np.float32))
    ae = m.op("Add", [e, vm], name="add_eps")
    sq = m.op("Sqrt", [ae], name="sqrt")
    dv = m.op("Div", [sub, sq], name="div")
    bias = m.const("bias", np.array([1, 2, 3], np.float32))
    scale = m.const("scale", np.array([3, 4, 5], np.float32))
    mu = m.op("Mul", [dv, scale], name="mul")
    m.outputs = [m.op("Add", [mu, bias], name="final_add")]
    return m


def test_fuse_layer_norm():
    o = OPT.optimize(_layer_norm_spec(), graph_runner._run_node)
    n = _producer(o, o.outputs[0])
    assert (n.op_type, n.name) == ("LayerNormalization", "final_add")
    assert n.attrs["epsilon"] == pytest.approx(1e-6) and n.inputs == ["x", "scale", "bias"]


@pytest.mark.parametrize("kw", [{"axes": (0,)}, {"axes": (-2, -1)}, {"pow_exp": 3.0}])
def test_layer_norm_not_fused(kw):
    """Only ReduceMean over axis -1 (optimize.rs:453-474) and Pow(., 2) match."""
    o = OPT.optimize(_layer_norm_spec(**kw), graph_runner._run_node)
    assert _producer(o, o.outputs[0]).op_type == "Add"


def _softsign():
    """pattern_matcher.rs:350-361."""
    m = _spec()
    x = m.value("x")
    a = m.op("Abs", [x], name="abs")
    one = m.const("one", np.array(1.0, np.float32))
    ad = m.op("Add", [one, a], name="add")
    out = m.op("Div", [x, ad], name="div")
    return m, out


def test_pattern_matcher_cases():
    """pattern_matcher.rs:363-450."""
    x, c = OPT.Sym("x"), OPT.Sym("c", const=True)
    cases = [
        (OPT.binop("Div", x, OPT.binop("Add", 1.0, OPT.Op("Abs", [x]))), True),
        (OPT.binop("Div", x, OPT.binop("Add", c, OPT.Op("Abs", [x]))), True),
        (OPT.binop("Div", OPT.binop("Add", 1.0, OPT.Op("Abs", [x])), x), False),
        (OPT.binop("Div", x, OPT.binop("Add", OPT.Op("Abs", [x]), 1.0)), True),
        (OPT.binop("Div", x, OPT.binop("Sub", 1.0, OPT.Op("Abs", [x]))), False),
        (OPT.binop("Div", x, OPT.binop("Add", 1.1, OPT.Op("Abs", [x]))), False),
        (OPT.binop("Div", x, OPT.binop("Add", 1.00001, OPT.Op("Abs", [x]))), True),
        (OPT.binop("Div", x, OPT.binop("Add", x, OPT.Op("Abs", [x]))), False),
        (OPT.binop("Div", c, OPT.binop("Add", 1.0, OPT.Op("Abs", [x]))), False),
    ]
    m, out = _softsign()
    g = OPT._Graph(m)
    for i, (pat, expect) in enumerate(cases):
        res = OPT.match(pat, out, g)
        assert (res is not None) == expect, i
        if res is not None:
            assert OPT._resolved(res, "x") == "x"
    key = OPT.binop("Div", x, OPT.binop("Add", 1.0, OPT.Op("Abs", [x], key="abs_op")))
    assert OPT._resolved(OPT.match(key, out, g), "abs_op") == "abs"


# ---------------------------------------------------------------- BERT export
def test_unfused_bert_optimizes_to_fused_mix():
    """bert_encoder(unfused=True) -- LayerNorm and GELU as their ONNX
    primitives, head reshapes through a Shape subgraph, a constant-foldable
    attention scale -- becomes the fused operator mix under the optimizer, and
    runs to the fused spec's exact bits."""
    from rten_hip import models

    fused = models.bert_encoder(layers=2, seq=16, embeddings=True, vocab=50)
    raw = models.bert_encoder(layers=2, seq=16, embeddings=True, vocab=50, unfused=True)
    o = OPT.optimize(raw, graph_runner._run_node)
    live = graph_runner._live(o, o.outputs)
    types = sorted(n.op_type for n in o.nodes if n.kind == "op" and n.name in live)
    assert "Erf" not in types and "ReduceMean" not in types and "Pow" not in types
    assert types.count("Gelu") == 2 and types.count("LayerNormalization") == 5
    rng = np.random.default_rng(9)
    feed = {"input_ids": rng.integers(0, 50, (2, 16)).astype(np.int32),
            "token_type_ids": rng.integers(0, 2, (2, 16)).astype(np.int32),
            "attention_mask": np.ones((2, 16), np.int32)}
    feed["attention_mask"][1, 12:] = 0
    a = graph_runner.run(fused, feed)[fused.outputs[0]]
    b = graph_runner.run(raw, feed)[raw.outputs[0]]
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    # without the optimizer the primitives differ from the fused kernels
    c = graph_runner.run(raw, feed, optimize=False)[raw.outputs[0]]
    assert not np.array_equal(a.view(np.uint32), c.view(np.uint32))
    assert np.allclose(a, c, rtol=1e-4, atol=1e-4)
