"""RTen's load-time optimizer on the device graph (csrc/graph_optimize.cpp) and
the ONNX-export operators (csrc/graph_host.cpp plan-time shape subgraph,
ReduceMean / Pow / Sqrt / Concat / Slice / Expand / ConstantOfShape kernels),
against the oracle running the graph RTen's optimizer would leave
(oracle/optimizer.py).  Bar: bit-exact, except Pow with an exponent other than
2 or 3 (the reference calls libm powf; the device rounds a double-precision
pow once: within 1 ULP).

Fusion tests mirror src/optimize.rs:546-716: the fused operator's name
(Operator::name()) and node name, on the device graph's own description.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rh():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import rten_hip

    rten_hip.default_context()
    return rten_hip


def _bits_equal(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and a.dtype == b.dtype and np.array_equal(a.view(np.uint32), b.view(np.uint32))


def _spec(name="t"):
    from rten_hip.graph import ModelSpec

    return ModelSpec(name)


def _run_device(spec, feed, runs=3, optimize=True, graph=None):
    import torch

    g = graph or spec.to_graph(optimize=optimize)
    dev = {g.input_ids[i]: torch.from_numpy(np.ascontiguousarray(feed[n])).cuda() for i, n in enumerate(spec.inputs)}
    outs, out = [], None
    for _ in range(runs):
        out = g.run(dev, g.output_ids, out=out)
        torch.cuda.synchronize()
        outs.append([o.cpu().numpy() for o in out])
    return g, outs


def _check(spec, feed, optimize=True, runs=3, graph=None):
    import graph_runner

    exp = graph_runner.run(spec, feed, optimize=optimize)
    g, outs = _run_device(spec, feed, runs, optimize, graph)
    for r, got in enumerate(outs):
        for name, o in zip(spec.outputs, got):
            e = exp[name]
            assert _bits_equal(o, np.asarray(e, o.dtype)), (r, name, np.abs(o.astype(np.float64) - e).max())
    return g


# ------------------------------------------------------------ fusion tests
def test_constant_propagation(rh):
    """optimize.rs:546-601: Add of two constants becomes a constant, output
    and consumer included."""
    m = _spec()
    a = m.const("const_a", np.array([1, 2, 3], np.float32))
    b = m.const("const_b", np.array([4, 5, 6], np.float32))
    s1 = m.op("Add", [a, b], name="add_1")
    x = m.value("input")
    m.inputs = [x]
    s2 = m.op("Add", [s1, x], name="add_2")
    m.outputs = [s1, s2]
    g = _check(m, {"input": np.array([10, 20, 30], np.float32)})
    d = {n["id"]: n for n in g.describe()}
    assert d[g.output_ids[0]]["kind"] == "const"
    assert g.producer(g.output_ids[0]) is None
    assert g.producer(g.output_ids[1])["name"] == "add_2"


def test_fuse_transpose(rh):
    m = _spec()
    i1, i2 = m.value("i1"), m.value("i2")
    m.inputs = [i1, i2]
    t = m.op("Transpose", [i1], name="transpose")
    m.outputs = [m.op("MatMul", [t, i2], name="matmul")]
    rng = np.random.default_rng(1)
    g = _check(m, {"i1": rng.random((20, 16), dtype=np.float32), "i2": rng.random((20, 24), dtype=np.float32)})
    p = g.producer(g.output_ids[0])
    assert (p["op"], p["name"]) == ("FusedTranspose(MatMul)", "matmul")


def test_fuse_silu(rh):
    m = _spec()
    x = m.value("x")
    m.inputs = [x]
    s = m.op("Sigmoid", [x], name="sigmoid")
    m.outputs = [m.op("Mul", [x, s], name="mul")]
    g = _check(m, {"x": np.linspace(-8, 8, 3001, dtype=np.float32)})
    p = g.producer(g.output_ids[0])
    assert (p["op"], p["name"]) == ("Silu", "mul")


def _gelu_spec(swap=False):
    m = _spec()
    sq = m.const("sqrt2", np.array(np.sqrt(2.0), np.float32))
    one = m.const("one", np.array(1.0, np.float32))
    half = m.const("half", np.array(0.5, np.float32))
    x = m.value("x")
    m.inputs = [x]
    d = m.op("Div", [x, sq], name="div")
    e = m.op("Erf", [d], name="erf")
    a = m.op("Add", [one, e] if swap else [e, one], name="add")
    mu = m.op("Mul", [a, x] if swap else [x, a], name="mul")
    m.outputs = [m.op("Mul", [half, mu] if swap else [mu, half], name="mul_half")]
    return m


@pytest.mark.parametrize("swap", [False, True])
def test_fuse_gelu(rh, swap):
    g = _check(_gelu_spec(swap), {"x": np.linspace(-6, 6, 4097, dtype=np.float32)})
    p = g.producer(g.output_ids[0])
    assert (p["op"], p["name"]) == ("Gelu", "mul_half")


def _layer_norm_spec(axes=(-1,), keep=1, eps=1e-6, n=3):
    m = _spec()
    x = m.value("x")
    m.inputs = [x]
    mean = m.op("ReduceMean", [x], {"axes": list(axes), "keep_dims": keep}, name="mean")
    sub = m.op("Sub", [x, mean], name="sub")
    p = m.op("Pow", [sub, m.const("two", np.array(2.0, np.float32))], name="pow")
    vm = m.op("ReduceMean", [p], {"axes": list(axes), "keep_dims": keep}, name="var_mean")
    ae = m.op("Add", [m.const("eps", np.array(eps, np.float32)), vm], name="add_eps")
    sq = m.op("Sqrt", [ae], name="sqrt")
    dv = m.op("Div", [sub, sq], name="div")
    rng = np.random.default_rng(n)
    mu = m.op("Mul", [dv, m.const("scale", rng.uniform(0.5, 1.5, n).astype(np.float32))], name="mul")
    m.outputs = [m.op("Add", [mu, m.const("bias", rng.uniform(-1, 1, n).astype(np.float32))], name="final_add")]
    return m


def test_fuse_layer_norm(rh):
    """optimize.rs:663-716, at BERT's width."""
    m = _layer_norm_spec(n=768)
    x = np.random.default_rng(4).standard_normal((64, 768)).astype(np.float32)
    g = _check(m, {"x": x})
    p = g.producer(g.output_ids[0])
    assert (p["op"], p["name"]) == ("LayerNormalization", "final_add")


def test_layer_norm_over_axis0_runs_unfused(rh):
    """ReduceMean over axis 0 does not match (optimize.rs:453-474): the
    primitives run on the device -- ReduceMean's iter_sum order, Pow's x * x,
    Sqrt -- with the oracle's bits."""
    m = _layer_norm_spec(axes=(0,), n=5)
    g = _check(m, {"x": np.random.default_rng(5).standard_normal((37, 5)).astype(np.float32)})
    assert g.producer(g.output_ids[0])["op"] == "Add"


# ------------------------------------------------------------ export ops
@pytest.mark.parametrize("shape,axes,keep", [((64, 771), [-1], 1), ((4, 13, 6), [1], 0), ((3, 4, 5), [0, 2], 1),
                                             ((6, 7), None, 0), ((2, 3, 9), [-1, -2], 0), ((9,), [0], 1)])
def test_reduce_mean(rh, shape, axes, keep):
    m = _spec()
    x = m.value("x")
    m.inputs = [x]
    attrs = {"keep_dims": keep}
    if axes is not None:
        attrs["axes"] = axes
    m.outputs = [m.op("ReduceMean", [x], attrs, name="rm")]
    x0 = (np.random.default_rng(len(shape)).standard_normal(shape) * 50).astype(np.float32)
    _check(m, {"x": x0}, optimize=False)


def test_reduce_mean_per_op_errors(rh):
    import torch

    x = torch.zeros((3, 3), device="cuda")
    with pytest.raises(rh.OpError, match="Axis is invalid"):
        rh.reduce_mean(x, [3])
    with pytest.raises(rh.OpError, match="Cannot reduce empty tensor"):
        rh.reduce_mean(torch.zeros((0,), device="cuda"), [0])


@pytest.mark.parametrize("exp", [2.0, 3.0, 0.5, -1.5])
def test_pow(rh, exp):
    import graph_runner

    m = _spec()
    x = m.value("x")
    m.inputs = [x]
    m.outputs = [m.op("Pow", [x, m.const("e", np.array([exp], np.float32))], name="pow")]
    x0 = np.random.default_rng(8).uniform(0.01, 30, 10000).astype(np.float32)
    if exp in (2.0, 3.0):
        x0 = x0 - np.float32(15)
        _check(m, {"x": x0}, optimize=False)
        return
    exp_out = graph_runner.run(m, {"x": x0}, optimize=False)[m.outputs[0]]
    _, outs = _run_device(m, {"x": x0}, runs=1, optimize=False)
    got = outs[0][0]
    ulp = np.abs(got.view(np.int32).astype(np.int64) - exp_out.view(np.int32).astype(np.int64))
    assert ulp.max() <= 1  # tolerance: 1 ULP of libm powf (see module docstring)


def test_shape_subgraph_and_data_ops(rh):
    """Shape -> Gather -> Unsqueeze -> Concat -> Reshape (plan-time), a
    ConstantOfShape too big for the host, Slice with negative steps, Expand,
    Concat of device tensors, Sqrt, and int32 arithmetic on shapes."""
    m = _spec()
    x = m.value("x")
    m.inputs = [x]
    sh = m.op("Shape", [x], name="shape")
    d0 = m.op("Gather", [sh, m.const("i0", np.array(0, np.int32))], {"axis": 0}, name="d0")
    d1 = m.op("Gather", [sh, m.const("i1", np.array(1, np.int32))], {"axis": 0}, name="d1")
    d1h = m.op("Div", [d1, m.const("two", np.array(2, np.int32))], name="d1_half")
    ax = m.const("ax0", np.array([0], np.int32))
    shp = m.op("Concat", [m.op("Unsqueeze", [d0, ax], name="u0"), m.op("Unsqueeze", [d1h, ax], name="u1"),
                          m.const("two1", np.array([2], np.int32))], {"axis": 0}, name="shp")
    r = m.op("Reshape", [x, shp], name="reshape")                      # [B, W/2, 2]
    sl = m.op("Slice", [r, m.const("st", np.array([-1, 1], np.int32)), m.const("en", np.array([-100, 2], np.int32)),
                        m.const("axs", np.array([1, 2], np.int32)), m.const("sp", np.array([-2, 1], np.int32))],
              name="slice")                                             # [B, ceil(W/4), 1]
    ex = m.op("Expand", [sl, m.const("tgt", np.array([1, 1, 3], np.int32))], name="expand")
    cat = m.op("Concat", [ex, m.op("Sqrt", [ex], name="sqrt")], {"axis": -1}, name="cat")
    big = m.op("ConstantOfShape", [m.const("bigshape", np.array([300, 301], np.int32))], {"value": 0.5}, name="fill")
    small = m.op("ConstantOfShape", [shp], {"value": 7}, name="fill_i")
    m.outputs = [cat, big, small, shp]
    x0 = np.random.default_rng(3).uniform(0, 9, (3, 40)).astype(np.float32)
    _check(m, {"x": x0})


# ------------------------------------------------------------ the BERT export
@pytest.mark.parametrize("source", ["spec", "rten"])
def test_unfused_bert_export_bitexact(rh, source):
    """An ONNX-export BERT (LayerNorm / GELU as primitives, head reshapes via
    the Shape subgraph, position ids sliced from a buffer, a folded Sqrt scale)
    loads, fuses to the fused mix on the device (Gelu / LayerNormalization /
    FusedAttention) and gives the oracle's bits -- the same bits as the fused
    spec -- eager and replayed."""
    import graph_runner
    from rten_hip import models, rten_file

    raw = models.bert_encoder(layers=2, seq=32, embeddings=True, vocab=300, unfused=True)
    fused = models.bert_encoder(layers=2, seq=32, embeddings=True, vocab=300)
    rng = np.random.default_rng(12)
    feed = {"input_ids": rng.integers(0, 300, (3, 32)).astype(np.int32),
            "token_type_ids": rng.integers(0, 2, (3, 32)).astype(np.int32),
            "attention_mask": np.ones((3, 32), np.int32)}
    feed["attention_mask"][1, 20:] = 0
    graph = rten_file.load_model(rten_file.to_rten_bytes(raw)) if source == "rten" else None
    g = _check(raw, feed, graph=graph)
    ref = graph_runner.run(fused, feed)[fused.outputs[0]]
    got = graph_runner.run(raw, feed)[raw.outputs[0]]
    assert _bits_equal(got, ref)
    ops = _live_ops(g)
    assert ops.count("LayerNormalization") == 5 and ops.count("FusedAttention") == 2
    for prim in ("Erf", "ReduceMean", "Pow", "Sqrt", "Gelu"):  # Gelu: in the FFN1 MatMul's epilogue
        assert prim not in ops, prim


def _live_ops(g):
    """Operator names the graph's outputs depend on (the fused subgraphs'
    leftover intermediates stay in the graph but are never planned)."""
    nodes = g.describe()
    prod = {o: n for n in nodes if n["kind"] == "op" for o in n["outputs"]}
    seen, stack, names = set(), list(g.output_ids), []
    while stack:
        n = prod.get(stack.pop())
        if n is None or n["id"] in seen:
            continue
        seen.add(n["id"])
        names.append(n["op"])
        stack.extend(n["inputs"])
    return names
