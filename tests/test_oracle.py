"""Pin the CPU oracle (the parity checker) before trusting it.

1. Known-answer vectors from the reference's own unit tests
   (tests/golden/kats.json, each entry cites its source test).
2. The reference's own naive oracles (reference_gemm, src/gemm.rs:1126-1147)
   and its shape sweeps (src/gemm.rs:1185-1238; src/ops/conv.rs:814-1153).
3. An independent cross-check against torch CPU in float64.

The oracle's exact summation order (its bits) is pinned structurally: it
restates the reference's loops (KC = 256 K blocks folded in order, the 6 x 16
kernel's fma chains, slice_sum / iter_sum orders), and test_gemm_kc_block_order
checks the block fold against an explicit float32 restatement.
"""
import json
import math
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
KATS = json.load(open(os.path.join(HERE, "golden", "kats.json")))


def expect_equal(actual, expected, atol=1e-8, rtol=1e-5):
    """rten-tensor/src/test_util.rs:46-62 (|a-e| <= atol + rtol*|e|)."""
    actual = np.asarray(actual, np.float32).ravel()
    expected = np.asarray(expected, np.float32).ravel()
    assert actual.shape == expected.shape
    bad = np.abs(actual - expected) > atol + rtol * np.abs(expected)
    assert not bad.any(), f"mismatch at {np.nonzero(bad)[0][:8]}: {actual[bad][:8]} vs {expected[bad][:8]}"


def expect_eq_1e4(actual, expected):
    expect_equal(actual, expected, atol=1e-4, rtol=0.0)


def check(tol, actual, expected):
    if tol == "eq":
        expect_equal(actual, expected)
    elif tol == "1e4":
        expect_eq_1e4(actual, expected)
    elif tol == "ulp0":
        assert np.array_equal(np.asarray(actual, np.float32).view(np.uint32),
                              np.asarray(expected, np.float32).view(np.uint32))
    else:
        raise ValueError(tol)


def _arr(v):
    return np.array([float(x) for x in v], np.float32)


# --------------------------------------------------------------------------
# 1. Known-answer vectors
# --------------------------------------------------------------------------

@pytest.mark.parametrize("case", KATS["conv"], ids=lambda c: c["source"])
def test_kat_conv(oracle, case):
    x = np.array(case["x"], np.float32).reshape(case["x_shape"])
    w = np.array(case["w"], np.float32).reshape(case["w_shape"])
    b = np.array(case["bias"], np.float32) if case["bias"] else None
    y = oracle.conv(x, w, b, pads=case["pads"], strides=case["strides"],
                    dilations=case["dilations"], groups=case["groups"])
    assert list(y.shape) == case["y_shape"]
    if "y_parts" in case:
        expected = [np.float32(a) + np.float32(c) for a, c in case["y_parts"]]
    else:
        expected = case["y"]
    check(case["tol"], y, expected)


def test_kat_graph_conv_relu(oracle):
    c = KATS["graph_conv_relu"]
    x = np.array(c["x"], np.float32).reshape(c["x_shape"])
    w = np.array(c["w"], np.float32).reshape(c["w_shape"])
    y = oracle.relu(oracle.conv(x, w, None, pads=(1, 1, 1, 1)))
    check(c["tol"], y, c["y"])


def test_kat_average_pool(oracle):
    c = KATS["average_pool"][0]
    x = np.array(c["x"], np.float32).reshape(c["x_shape"])
    for case in c["cases"]:
        y = oracle.average_pool(x, case["kernel"], case["strides"])
        assert list(y.shape) == case["y_shape"]
        check(c["tol"], y, case["y"])
    c = KATS["average_pool"][1]
    plane = np.array(c["plane"], np.float32).reshape(4, 4)
    x = np.broadcast_to(plane, (1, c["channels"], 4, 4)).copy()
    for key, incl in (("y_exclude_pad", False), ("y_include_pad", True)):
        y = oracle.average_pool(x, c["kernel"], c["strides"], c["pads"], count_include_pad=incl)
        exp = np.broadcast_to(np.array(c[key], np.float32).reshape(3, 3), y.shape)
        check(c["tol"], y, exp)


def test_kat_global_average_pool(oracle):
    c = KATS["global_average_pool"]
    x = np.array(c["x"], np.float32).reshape(c["x_shape"])
    check(c["tol"], oracle.global_average_pool(x), c["y"])


def test_kat_max_pool(oracle):
    c = KATS["max_pool"][0]
    x = np.array(c["x"], np.float32).reshape(c["x_shape"])
    for case in c["cases"]:
        y = oracle.max_pool(x, case["kernel"], case["strides"])
        assert list(y.shape) == case["y_shape"]
        check(c["tol"], y, case["y"])
    x = np.zeros((1, 1, 9, 9), np.float32)
    for case in KATS["max_pool_shapes"]["cases"]:
        if case["same"]:
            y = oracle.max_pool(x, (2, 2), case["strides"], padding="same")
        else:
            y = oracle.max_pool(x, (2, 2), case["strides"], case["pads"])
        assert list(y.shape) == case["out"]


def test_kat_output_size_and_padding(oracle):
    for case in KATS["output_size_and_padding"]["cases"]:
        mode = "same" if case["same"] else "fixed"
        pads = case["pads"] or (0, 0, 0, 0)
        if "error" in case:
            with pytest.raises(oracle.OpError) as e:
                oracle.output_size_and_padding(case["in"], case["k"], case["s"], mode, pads, case["d"])
            assert str(e.value) == case["error"] and e.value.kind == "InvalidValue"
        else:
            out, pads_out = oracle.output_size_and_padding(case["in"], case["k"], case["s"], mode,
                                                           pads, case["d"])
            assert list(out) == case["out"] and list(pads_out) == case["pads_out"]


def test_kat_batch_norm(oracle):
    c = KATS["batch_norm"]
    x = np.array(c["x"], np.float32).reshape(c["x_shape"])
    sc, b, m, v = (np.array(c[k], np.float32) for k in ("scale", "bias", "mean", "var"))
    eps = np.float32(c["epsilon"])
    # The test's own formula: (x - mean) / sqrt(var + eps) * scale + bias.
    exp = [(x.ravel()[i] - m[i]) / np.sqrt(v[i] + eps) * sc[i] + b[i] for i in range(2)]
    check(c["tol"], oracle.batch_norm(x, sc, b, m, v, c["epsilon"]), exp)
    # 3-D (NCT) case of the same test.
    check(c["tol"], oracle.batch_norm(x.reshape(1, 2, 1), sc, b, m, v, c["epsilon"]), exp)
    err = KATS["errors"][0]
    with pytest.raises(oracle.OpError) as e:
        oracle.batch_norm(np.zeros(err["x_shape"], np.float32), sc, b, m, v)
    assert str(e.value) == err["message"] and e.value.kind == err["kind"]


def test_kat_layer_norm(oracle):
    c = KATS["layer_norm"]
    x = np.array(c["x"], np.float32).reshape(c["x_shape"])
    y = oracle.layer_norm(x, np.array(c["scale"], np.float32), np.array(c["bias"], np.float32),
                          c["axis"], c["epsilon"])
    check(c["tol"], y, c["y"])


@pytest.mark.parametrize("case", KATS["softmax"], ids=lambda c: c["source"])
def test_kat_softmax(oracle, case):
    x = np.array(case["x"], np.float32).reshape(case["x_shape"])
    if case.get("transpose_input"):
        x = x.T.copy()
    check(case["tol"], oracle.softmax(x, case["axis"]), case["y"])


@pytest.mark.parametrize("case", KATS["log_softmax"], ids=lambda c: c["source"])
def test_kat_log_softmax(oracle, case):
    x = np.array(case["x"], np.float32).reshape(case["x_shape"])
    check(case["tol"], oracle.log_softmax(x, case["axis"]), case["y"])


def test_kat_instance_norm(oracle):
    c = KATS["instance_norm"]
    x = np.array(c["x"], np.float32).reshape(c["x_shape"])
    sc, b = np.array(c["scale"], np.float32), np.array(c["bias"], np.float32)
    check(c["tol"], oracle.instance_norm(x, sc, b), c["y"])
    # the reference's error order (norm.rs:161-177)
    for args, msg in [((x[0, 0], sc, b), "expected input with >= 2 dims"),
                      ((x, sc[:4], b), "scale length should match channel count"),
                      ((x, sc, b[:4]), "bias length should match channel count")]:
        with pytest.raises(oracle.OpError) as e:
            oracle.instance_norm(*args)
        assert str(e.value) == msg


@pytest.mark.parametrize("case", KATS["unary"], ids=lambda c: c["source"])
def test_kat_unary(oracle, case):
    x = _arr(case["x"])
    y = oracle.unary(case["op"], x)
    exp = _arr(case["y"])
    if case["tol"] == "nan_eq":
        assert np.array_equal(np.isnan(y), np.isnan(exp))
        m = ~np.isnan(exp)
        assert np.array_equal(y[m], exp[m])
    else:
        check(case["tol"], y, exp)


@pytest.mark.parametrize("case", KATS["accuracy"], ids=lambda c: c["source"])
def test_erf_accuracy(oracle, case):
    # arange(-6., 6., 0.001f32) accumulates in f32 (rten-vecmath testing.rs).
    xs = []
    x = np.float32(case["lo"])
    step = np.float32(case["step"])
    while x < case["hi"]:
        xs.append(x)
        x = np.float32(x + step)
    xs = np.array(xs, np.float32)
    exp = np.array([np.float32(math.erf(float(v))) for v in xs], np.float32)
    diff = np.abs(oracle.unary("Erf", xs) - exp).max()
    assert diff <= case["max_abs_err"] * 1.0001, diff


# --------------------------------------------------------------------------
# 2. Reference-style sweeps against its own naive oracles
# --------------------------------------------------------------------------

def _rng_mat(oracle, seed, rows, cols):
    return oracle.xorshift(seed, rows * cols).reshape(rows, cols)


def test_xorshift_matches_reference():
    # rng.rs:17-35 restated in numpy with u64 wrap-around.
    import rten_oracle as o

    s = np.uint64(1234)
    vals = []
    with np.errstate(over="ignore"):
        for _ in range(5):
            s ^= (s << np.uint64(13)) & np.uint64(0xFFFFFFFFFFFFFFFF)
            s ^= s >> np.uint64(7)
            s ^= (s << np.uint64(17)) & np.uint64(0xFFFFFFFFFFFFFFFF)
            vals.append(np.float32(np.float32(int(s >> np.uint64(24))) * np.float32(1.0 / (1 << 40))))
    assert np.array_equal(o.xorshift(1234, 5), np.array(vals, np.float32))


@pytest.mark.parametrize("m,n,k", [
    (m, n, k)
    for m in (0, 2, 8, 10, 16, 64, 80)
    for n in (0, 2, 4, 5, 8, 1024, 1025)
    for k in (0, 2, 20, 256, 300)
    if m * n * k <= 80 * 1025 * 300
][::5] + [(s, s, s) for s in list(range(1, 20)) + [30, 64, 65]])
def test_gemm_sweep_vs_reference_gemm(oracle, m, n, k):
    """test_gemm_with_kernel shape sweep (src/gemm.rs:1185-1238), XorShiftRng(1234)."""
    a = _rng_mat(oracle, 1234, m, k) if m * k else np.zeros((m, k), np.float32)
    b = _rng_mat(oracle, 1235, k, n) if k * n else np.zeros((k, n), np.float32)
    out = oracle.gemm(a, b)
    ref = oracle.reference_gemm(a, b)
    expect_equal(out, ref)


def test_gemm_alpha_beta_bias(oracle):
    a = _rng_mat(oracle, 1, 33, 300)
    b = _rng_mat(oracle, 2, 300, 47)
    bias = oracle.xorshift(3, 33)
    for alpha, beta in ((1.0, 0.0), (1.0, 1.0), (0.5, 0.0), (0.5, 2.0), (2.0, 0.5)):
        init = _rng_mat(oracle, 4, 33, 47)
        out = oracle.gemm(a, b, alpha, beta, out=init.copy(), bias=bias)
        ref = oracle.reference_gemm(a, b, alpha, beta, out=init.copy(), bias=bias)
        expect_equal(out, ref, atol=1e-5)


def test_gemm_beta_zero_ignores_nan(oracle):
    """β=0 must not read the output (src/gemm.rs:1272-1300 NaN case)."""
    a = _rng_mat(oracle, 5, 20, 20)
    b = _rng_mat(oracle, 6, 20, 20)
    out = np.full((20, 20), np.nan, np.float32)
    oracle.gemm(a, b, 1.0, 0.0, out=out)
    assert not np.isnan(out).any()


def fma32(a, b, c):
    """Correctly rounded f32 fma(a, b, c) (no math.fma on Python 3.10): the
    product of two f32 is exact in f64; only a tie after the f64 sum can
    double-round, and that case is settled exactly with Fractions."""
    from fractions import Fraction

    s = float(a) * float(b) + float(c)
    r = np.float32(s)
    if float(r) != s:
        other = np.nextafter(r, np.float32(np.inf) if s > float(r) else np.float32(-np.inf))
        if abs(float(other) - s) == abs(float(r) - s):
            exact = Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c))
            if abs(Fraction(float(other)) - exact) < abs(Fraction(float(r)) - exact):
                return np.float32(other)
    return r


def test_gemm_kc_block_order(oracle):
    """The oracle's summation order IS the reference's: per-KC=256 fma
    chains from +0, summed in block order, bias after block 0."""
    m, n, k = 7, 17, 600
    a = _rng_mat(oracle, 7, m, k) - np.float32(0.5)
    b = _rng_mat(oracle, 8, k, n) - np.float32(0.5)
    bias = oracle.xorshift(9, m)
    out = oracle.gemm(a, b, bias=bias)
    ref = np.zeros((m, n), np.float32)
    for i in range(m):
        for j in range(n):
            total = None
            for k0 in range(0, k, 256):
                acc = np.float32(0)
                for kk in range(k0, min(k, k0 + 256)):
                    acc = fma32(a[i, kk], b[kk, j], acc)
                if total is None:
                    total = np.float32(acc + bias[i])
                else:
                    total = np.float32(total + acc)
            ref[i, j] = total
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))


def _torch_conv(x, w, b, pads, strides, dil, groups):
    import torch
    import torch.nn.functional as F

    xt = torch.tensor(x, dtype=torch.float64)
    xt = F.pad(xt, (pads[1], pads[3], pads[0], pads[2]))
    return F.conv2d(xt, torch.tensor(w, dtype=torch.float64),
                    None if b is None else torch.tensor(b, dtype=torch.float64),
                    stride=strides, dilation=dil, groups=groups).numpy()


CONV_CASES = [
    # (N, C, H, W, O, kh, kw, pads, strides, dil, groups)
    (1, 3, 10, 10, 4, 3, 3, (1, 1, 1, 1), (1, 1), (1, 1), 1),
    (2, 3, 20, 20, 4, 3, 3, (0, 0, 0, 0), (2, 2), (1, 1), 1),
    (1, 2, 5, 5, 3, 3, 3, (1, 1, 1, 1), (3, 3), (1, 1), 1),
    (1, 2, 4, 4, 3, 3, 3, (0, 1, 0, 1), (1, 3), (1, 1), 1),
    (1, 4, 9, 9, 4, 3, 3, (2, 2, 2, 2), (1, 1), (2, 2), 1),
    (2, 4, 8, 8, 6, 3, 3, (1, 1, 1, 1), (1, 1), (1, 1), 2),
    (2, 6, 8, 8, 6, 3, 3, (1, 1, 1, 1), (2, 2), (1, 1), 6),   # depthwise
    (1, 6, 7, 7, 6, 5, 5, (2, 2, 2, 2), (1, 1), (1, 1), 6),   # depthwise 5x5
    (2, 16, 7, 7, 32, 1, 1, (0, 0, 0, 0), (1, 1), (1, 1), 1),  # pointwise
    (2, 16, 14, 14, 32, 1, 1, (0, 0, 0, 0), (2, 2), (1, 1), 1),  # 1x1 stride 2 (im2col)
    (1, 300, 6, 6, 5, 1, 1, (0, 0, 0, 0), (1, 1), (1, 1), 1),  # K > KC
    (1, 40, 6, 6, 7, 3, 3, (1, 0, 2, 1), (1, 1), (1, 1), 1),  # uneven padding, K=360
    (1, 1, 6, 6, 1, 3, 3, (1, 1, 1, 1), (1, 1), (1, 1), 1),
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_vs_torch(oracle, case):
    N, Cc, H, W, O, kh, kw, pads, strides, dil, groups = case
    x = oracle.xorshift(1234, N * Cc * H * W).reshape(N, Cc, H, W) - np.float32(0.5)
    w = oracle.xorshift(4321, O * (Cc // groups) * kh * kw).reshape(O, Cc // groups, kh, kw) - np.float32(0.5)
    b = oracle.xorshift(99, O)
    y = oracle.conv(x, w, b, pads=pads, strides=strides, dilations=dil, groups=groups)
    ref = _torch_conv(x, w, b, pads, strides, dil, groups)
    assert y.shape == ref.shape
    expect_equal(y, ref, atol=1e-5, rtol=1e-5)


def test_conv_1d(oracle):
    x = oracle.xorshift(1, 2 * 3 * 17).reshape(2, 3, 17)
    w = oracle.xorshift(2, 4 * 3 * 3).reshape(4, 3, 3)
    y = oracle.conv(x, w, None, pads=(1, 1), strides=(2,), dilations=(1,))
    import torch.nn.functional as F
    import torch

    ref = F.conv1d(torch.tensor(x, dtype=torch.float64), torch.tensor(w, dtype=torch.float64),
                   stride=2, padding=1).numpy()
    expect_equal(y, ref, atol=1e-5)


def test_conv_errors(oracle):
    """Error strings asserted by src/ops/conv.rs:1034-1079."""
    x = np.zeros((1, 3, 4, 4), np.float32)
    with pytest.raises(oracle.OpError) as e:
        oracle.conv(x, np.zeros((2, 2, 3, 3), np.float32))
    assert "does not match kernel input channels" in str(e.value)
    with pytest.raises(oracle.OpError) as e:
        oracle.conv(x, np.zeros((2, 3, 5, 5), np.float32))
    assert str(e.value) == "Input too small for kernel size"
    with pytest.raises(oracle.OpError) as e:
        oracle.conv(x, np.zeros((2, 3, 3, 3), np.float32), strides=(0, 0))
    assert str(e.value) == "Strides must be > 0"


def test_pooling_vs_torch(oracle):
    import torch
    import torch.nn.functional as F

    x = oracle.xorshift(11, 2 * 5 * 13 * 13).reshape(2, 5, 13, 13) - np.float32(0.5)
    y = oracle.max_pool(x, (3, 3), (2, 2), (1, 1, 1, 1))
    ref = F.max_pool2d(torch.tensor(x), 3, 2, 1).numpy()
    assert np.array_equal(y, ref)
    y = oracle.average_pool(x, (3, 3), (2, 2), (1, 1, 1, 1), count_include_pad=True)
    ref = F.avg_pool2d(torch.tensor(x, dtype=torch.float64), 3, 2, 1, count_include_pad=True).numpy()
    expect_equal(y, ref, atol=1e-6)


def test_elementwise_vs_torch(oracle):
    import torch

    x = np.linspace(-8, 8, 4001).astype(np.float32)
    xt = torch.tensor(x, dtype=torch.float64)
    expect_equal(oracle.unary("Gelu", x), torch.nn.functional.gelu(xt).numpy(), atol=2e-6)
    expect_equal(oracle.unary("Sigmoid", x), torch.sigmoid(xt).numpy(), atol=1e-7)
    expect_equal(oracle.unary("Tanh", x), torch.tanh(xt).numpy(), atol=1e-7)
    expect_equal(oracle.clip(x, 0.0, 6.0), np.clip(x, 0, 6))


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def test_clip_clamp_trait_semantics(oracle):
    """Clip is RTen's Clamp::clamp = self.max(lo).min(hi) with the trait's own
    max (self > val ? self : val) and min (self < val ? self : val)
    (src/ops/unary_elementwise.rs:263-323): NaN -> lo, and a zero that equals a
    bound takes that bound's zero -- unlike f32::clamp / np.clip."""
    nan, inf = np.float32(np.nan), np.float32(np.inf)
    x = np.array([nan, -0.0, 0.0, 7.0, -3.0, 6.0, inf, -inf, 2.5], np.float32)
    assert (_bits(oracle.clip(x, 0.0, 6.0)) == _bits([0.0, 0.0, 0.0, 6.0, 0.0, 6.0, 6.0, 0.0, 2.5])).all()
    # Upper bound +0: -0 (not below -1) compares equal to +0, so min returns hi = +0.
    y = np.array([nan, -0.0, 0.5, -2.0, -0.5], np.float32)
    assert (_bits(oracle.clip(y, -1.0, 0.0)) == _bits([-1.0, 0.0, 0.0, -1.0, -0.5])).all()
    # Lower bound -0: +0 is not greater than -0, so max returns lo = -0.
    assert (_bits(oracle.clip(np.array([0.0], np.float32), -0.0, 1.0)) == _bits([-0.0])).all()


def test_binary_broadcast(oracle):
    """Add / Mul broadcasting and the incompatible-shape error
    (src/ops/binary_elementwise.rs:23-45, 158-439)."""
    a = oracle.xorshift(1, 2 * 3 * 4).reshape(2, 3, 4)
    b = oracle.xorshift(2, 4)
    assert np.array_equal(oracle.add(a, b), a + b)
    assert np.array_equal(oracle.binary("Mul", a, b.reshape(1, 1, 4)), a * b)
    with pytest.raises(oracle.OpError):
        oracle.add(a, np.zeros(3, np.float32))


def test_matmul_and_gemm_op_vs_numpy(oracle):
    a = oracle.xorshift(1, 2 * 3 * 5 * 64).reshape(2, 3, 5, 64)
    b = oracle.xorshift(2, 3 * 64 * 7).reshape(3, 64, 7)
    expect_equal(oracle.matmul(a, b), a.astype(np.float64) @ b, atol=1e-5)
    b2 = oracle.xorshift(3, 64 * 9).reshape(64, 9)
    expect_equal(oracle.matmul(a, b2), a.astype(np.float64) @ b2, atol=1e-5)
    A = oracle.xorshift(4, 1 * 2048).reshape(1, 2048)
    W = oracle.xorshift(5, 1000 * 2048).reshape(1000, 2048)
    c = oracle.xorshift(6, 1000)
    out = oracle.gemm_op(A, W, c, trans_b=True)   # batch-1 FC -> gemv_transposed
    expect_equal(out, A.astype(np.float64) @ W.T + c, atol=1e-4)
    A = oracle.xorshift(7, 4 * 2048).reshape(4, 2048)
    out = oracle.gemm_op(A, W, c, trans_b=True)
    expect_equal(out, A.astype(np.float64) @ W.T + c, atol=1e-4)
    with pytest.raises(oracle.OpError) as e:
        oracle.gemm_op(A, W, np.zeros(7, np.float32), trans_b=True)
    assert str(e.value) == "Cannot broadcast c to output shape"


@pytest.mark.parametrize("case", KATS["conv_transpose"], ids=lambda c: c["source"])
def test_kat_conv_transpose(oracle, case):
    """ConvTranspose known answers (PyTorch values in the reference's tests)."""
    x = np.array(case["x"], np.float32).reshape(case["x_shape"])
    w = np.array(case["w"], np.float32).reshape(case["w_shape"])
    b = np.array(case["bias"], np.float32) if case["bias"] else None
    y = oracle.conv_transpose(x, w, b, pads=case["pads"], strides=case["strides"],
                              padding=case["padding"])
    assert list(y.shape) == case["y_shape"]
    if case["y"] is not None:
        # expect_equal: atol 1e-8 + rtol 1e-5 (rten-tensor/src/test_util.rs:46-62)
        np.testing.assert_allclose(y.reshape(-1), case["y"], rtol=1e-5, atol=1e-8)


def test_kat_conv_transpose_output_size(oracle):
    for c in KATS["conv_transpose_output_size"]["cases"]:
        if "error" in c:
            with pytest.raises(oracle.OpError, match=c["error"]):
                oracle.conv_transpose_output_size(c["in"], c["k"], c["strides"], c["padding"], c["pads"])
        else:
            out, pads = oracle.conv_transpose_output_size(c["in"], c["k"], c["strides"], c["padding"],
                                                          c["pads"])
            assert list(out) == c["out"] and list(pads) == c["pads_out"]


@pytest.mark.parametrize("shape", [((2, 5, 7, 6), (5, 3, 3, 4), (2, 3), (1, 2, 0, 1)),
                                   ((1, 4, 5, 5), (4, 2, 2, 2), (2, 2), (0, 0, 0, 0)),
                                   ((3, 8, 4, 9), (8, 6, 5, 3), (1, 2), (2, 1, 2, 1))])
def test_conv_transpose_vs_torch(oracle, shape):
    """The oracle against torch's conv_transpose2d (fp tolerance: different
    summation order) on random shapes, fixed padding as output cropping."""
    torch = pytest.importorskip("torch")
    import torch.nn.functional as F

    xs, ws, st, pads = shape
    x = oracle.xorshift(11, int(np.prod(xs))).reshape(xs) - np.float32(0.5)
    w = oracle.xorshift(12, int(np.prod(ws))).reshape(ws) - np.float32(0.5)
    b = oracle.xorshift(13, ws[1])
    got = oracle.conv_transpose(x, w, b, pads=pads, strides=st)
    full = F.conv_transpose2d(torch.from_numpy(x), torch.from_numpy(w), torch.from_numpy(b),
                              stride=st).numpy()
    ref = full[:, :, pads[0]:full.shape[2] - pads[2], pads[1]:full.shape[3] - pads[3]]
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5)


# --------------------------------------------------------------------------
# Gather / Where / Cast (gather.rs, binary_elementwise.rs, convert.rs)
# --------------------------------------------------------------------------

def _f32_vals(v):
    return np.array([{"f32::MIN": -3.4028235e38, "f32::MAX": 3.4028235e38}.get(e, e) for e in v],
                    np.float32)


def test_kat_gather(oracle):
    c = KATS["gather"]
    for case in c["cases"]:
        x = np.array(case["x"], np.float32).reshape(case["x_shape"])
        idx = np.array(case["indices"], np.int32).reshape(case["indices_shape"])
        y = oracle.gather(x, idx, case["axis"])
        assert list(y.shape) == case["y_shape"]
        assert np.array_equal(y.ravel(), np.array(case["y"], np.float32)), case
    r = c["rand_case"]
    x = oracle.xorshift(r["seed"], int(np.prod(r["x_shape"]))).reshape(r["x_shape"])
    y = oracle.gather(x, np.array(r["indices"], np.int32).reshape(r["indices_shape"]), r["axis"])
    assert list(y.shape) == r["y_shape"] and np.array_equal(y.reshape(4, 10), x[r["indices"]])
    for case in c["errors"]:
        x = np.zeros(case["x_shape"], np.float32)
        idx = np.array(case["indices"], np.int32).reshape(case["indices_shape"])
        with pytest.raises(oracle.OpError) as e:
            oracle.gather(x, idx, case["axis"])
        assert e.value.code == case["code"] and str(e.value) == case["message"]


def test_kat_where_and_cast(oracle):
    c = KATS["where"]
    for case in c["cases"]:
        out = oracle.where(np.array(case["cond"], np.int32).reshape(case["cond_shape"]),
                           np.array(case["x"], np.float32).reshape(case["x_shape"]),
                           np.array(case["y"], np.float32).reshape(case["y_shape"]))
        assert list(out.shape) == case["out_shape"]
        assert np.array_equal(out.ravel(), np.array(case["out"], np.float32)), case
    for case in c["errors"]:
        with pytest.raises(oracle.OpError) as e:
            oracle.where(np.array(case["cond"], np.int32), np.array(case["x"], np.float32),
                         np.array(case["y"], np.float32))
        assert e.value.code == case["code"] and str(e.value) == case["message"]
    for case in KATS["cast"]["i32_to_f32"]:
        y = oracle.cast_i32_to_f32(np.array(case["x"], np.int32))
        assert np.array_equal(y, np.array(case["y"], np.float32))
    for case in KATS["cast"]["f32_to_i32"]:
        y = oracle.cast_f32_to_i32(_f32_vals(case["x"]))
        assert np.array_equal(y, np.array(case["y"], np.int32))
