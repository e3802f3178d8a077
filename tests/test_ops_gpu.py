"""GPU parity tests: every HIP operator against the CPU oracle.

The oracle restates RTen's CPU path including its summation order, so the bar
here is BIT-EXACT equality (compared as uint32 bit patterns) for every op
whose reference order the kernels reproduce.  Inputs are XorShiftRng streams
(rten-tensor/src/rng.rs) shifted to [-0.5, 0.5).  Sizes are small enough for
the oracle to finish in well under a second each; full-size ResNet-50 parity
lives in test_model_gpu.py.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def rh():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import rten_hip

    rten_hip.default_context()
    return rten_hip


def dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).cuda()


def host(t):
    import torch

    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def rnd(oracle, seed, *shape, scale=1.0, shift=0.5):
    n = int(np.prod(shape)) if shape else 1
    v = (oracle.xorshift(seed, n) - np.float32(shift)) * np.float32(scale)
    return v.astype(np.float32).reshape(shape)


def assert_bits(actual, expected, what=""):
    actual = np.asarray(actual, np.float32)
    expected = np.asarray(expected, np.float32)
    assert actual.shape == expected.shape, (what, actual.shape, expected.shape)
    a = actual.view(np.uint32)
    e = expected.view(np.uint32)
    same = (a == e) | (np.isnan(actual) & np.isnan(expected))
    if not same.all():
        idx = np.argwhere(~same)[:5]
        diff = np.abs(actual.astype(np.float64) - expected).max()
        rel = diff / max(1e-30, np.abs(expected).max())
        pytest.fail(f"{what}: {int((~same).sum())}/{same.size} differ (max abs {diff:.3g}, "
                    f"rel {rel:.3g}); first at {idx.tolist()}: "
                    f"{[actual[tuple(i)] for i in idx]} vs {[expected[tuple(i)] for i in idx]}")


# --------------------------------------------------------------------------
# GEMM engine
# --------------------------------------------------------------------------

GEMM_SHAPES = [(1, 1, 1), (2, 3, 4), (7, 17, 33), (64, 64, 64), (65, 130, 257), (128, 128, 256),
               (100, 300, 600), (33, 1025, 300), (257, 129, 1000), (64, 1000, 2048),
               (16, 16, 0),
               # dense LDS-DMA route (A packed per call, B read in place)
               (256, 256, 256), (300, 516, 700), (520, 768, 1030), (512, 3072, 768)]


@pytest.mark.parametrize("m,n,k", GEMM_SHAPES)
def test_gemm_bitexact(rh, oracle, m, n, k):
    a = rnd(oracle, 1, m, k)
    b = rnd(oracle, 2, k, n)
    bias = rnd(oracle, 3, m)
    exp = oracle.gemm(a, b, bias=bias)
    got = host(rh.gemm(dev(a), dev(b), bias=dev(bias)))
    assert_bits(got, exp, f"gemm {m}x{n}x{k}")


def test_gemm_alpha_beta(rh, oracle):
    m, n, k = 70, 50, 520
    a, b = rnd(oracle, 4, m, k), rnd(oracle, 5, k, n)
    init = rnd(oracle, 6, m, n)
    for alpha, beta in ((1.0, 1.0), (1.0, 0.0)):
        exp = oracle.gemm(a, b, alpha, beta, out=init.copy())
        out = dev(init)
        rh.gemm(dev(a), dev(b), alpha, beta, out=out)
        assert_bits(host(out), exp, f"alpha={alpha} beta={beta}")


def test_gemm_strided_b_rows(rh, oracle):
    """B with a row stride larger than N (a column slice) on the dense DMA route."""
    m, n, k = 260, 512, 300
    a = rnd(oracle, 12, m, k)
    bfull = rnd(oracle, 13, k, n + 64)
    exp = oracle.gemm(a, np.ascontiguousarray(bfull[:, 32:32 + n]))
    got = host(rh.gemm(dev(a), dev(bfull)[:, 32:32 + n]))
    assert_bits(got, exp, "strided B rows")


def test_gemm_transposed_views(rh, oracle):
    """Strided A/B (transposed views, FusedTranspose) read in place."""
    m, n, k = 45, 70, 300
    at = rnd(oracle, 7, k, m)
    bt = rnd(oracle, 8, n, k)
    exp = oracle.gemm(at.T, bt.T)
    got = host(rh.gemm(dev(at).t(), dev(bt).t()))
    assert_bits(got, exp, "transposed")


@pytest.mark.parametrize("n,k,transposed", [(1000, 2048, True), (1000, 2048, False), (37, 13, True),
                                            (300, 700, False), (129, 9, True),
                                            # wave-per-column kernel: > 8 K blocks (two passes),
                                            # a ragged last block, depth < 8, partial tiles
                                            (1000, 4617, True), (130, 1003, True), (77, 5, True),
                                            (2, 512, True), (260, 4096, True)])
def test_gemv_bitexact(rh, oracle, n, k, transposed):
    """M == 1 takes the reference's gemv path and summation order."""
    a = rnd(oracle, 9, 1, k)
    if transposed:
        b = rnd(oracle, 10, n, k).T  # unit row stride -> simd_gemv_transposed
    else:
        b = rnd(oracle, 10, k, n)
    bias = rnd(oracle, 11, 1)
    exp = oracle.gemm(a, b, bias=bias)
    bd = dev(b.T).t() if transposed else dev(b)
    got = host(rh.gemm(dev(a), bd, bias=dev(bias)))
    assert_bits(got, exp, "gemv")


@pytest.mark.parametrize("alpha,beta", [(0.5, 0.75), (1.0, 1.0), (-2.0, 0.0)])
def test_gemv_transposed_alpha_beta(rh, oracle, alpha, beta):
    """simd_gemv_transposed with alpha / beta: beta scales the prior output on
    the first K block only, then blocks accumulate with 1.0 (gemm.rs:651-704)."""
    n, k = 203, 1500
    a = rnd(oracle, 12, 1, k)
    b = rnd(oracle, 13, n, k).T
    out0 = rnd(oracle, 14, 1, n)
    exp = oracle.gemm(a, b, alpha=alpha, beta=beta, out=out0.copy())
    out = dev(out0)
    rh.gemm(dev(a), dev(b.T).t(), alpha=alpha, beta=beta, out=out)
    assert_bits(host(out), exp, "gemv alpha/beta")


# --------------------------------------------------------------------------
# Conv
# --------------------------------------------------------------------------

CONV_CASES = [
    # name, (N, C, H, W), (O, kh, kw), pads, strides, dilations, groups
    ("resnet-conv1", (2, 3, 30, 30), (64, 7, 7), (3, 3, 3, 3), (2, 2), (1, 1), 1),
    ("3x3-s1", (2, 64, 14, 14), (64, 3, 3), (1, 1, 1, 1), (1, 1), (1, 1), 1),
    ("3x3-s2-K1152", (2, 128, 14, 14), (128, 3, 3), (1, 1, 1, 1), (2, 2), (1, 1), 1),
    ("1x1-pointwise", (2, 256, 7, 7), (128, 1, 1), (0, 0, 0, 0), (1, 1), (1, 1), 1),
    ("1x1-pointwise-K1024", (3, 1024, 5, 5), (96, 1, 1), (0, 0, 0, 0), (1, 1), (1, 1), 1),
    ("1x1-s2-im2col", (2, 64, 14, 14), (256, 1, 1), (0, 0, 0, 0), (2, 2), (1, 1), 1),
    ("3x3-layer4", (2, 512, 7, 7), (512, 3, 3), (1, 1, 1, 1), (1, 1), (1, 1), 1),
    ("grouped", (2, 8, 9, 9), (12, 3, 3), (1, 1, 1, 1), (1, 1), (1, 1), 2),
    ("dilated", (1, 4, 11, 11), (6, 3, 3), (2, 2, 2, 2), (1, 1), (2, 2), 1),
    ("uneven-pad", (1, 40, 6, 6), (7, 3, 3), (1, 0, 2, 1), (1, 1), (1, 1), 1),
    ("strided-1x3", (1, 5, 9, 9), (3, 3, 3), (1, 1, 1, 1), (1, 3), (1, 1), 1),
    ("depthwise-s1", (2, 32, 12, 12), (32, 3, 3), (1, 1, 1, 1), (1, 1), (1, 1), 32),
    ("depthwise-s2", (2, 96, 13, 13), (96, 3, 3), (1, 1, 1, 1), (2, 2), (1, 1), 96),
    ("depthwise-pad3-s2", (1, 4, 10, 10), (4, 3, 3), (3, 3, 3, 3), (2, 2), (1, 1), 4),
    ("pointwise-O1-gemv", (2, 20, 6, 6), (1, 1, 1), (0, 0, 0, 0), (1, 1), (1, 1), 1),
    # 4-output-column depthwise kernel (OW % 4 == 0): s1 / s2, row slices that
    # do not divide OH, asymmetric and zero left padding.
    ("depthwise4-s1-28", (2, 24, 28, 28), (24, 3, 3), (1, 1, 1, 1), (1, 1), (1, 1), 24),
    ("depthwise4-s1-56", (1, 8, 56, 56), (8, 3, 3), (1, 1, 1, 1), (1, 1), (1, 1), 8),
    ("depthwise4-s2-56", (2, 16, 56, 56), (16, 3, 3), (1, 1, 1, 1), (2, 2), (1, 1), 16),
    ("depthwise4-s2-112", (1, 4, 112, 112), (4, 3, 3), (1, 1, 1, 1), (2, 2), (1, 1), 4),
    ("depthwise4-ragged-rows", (1, 3, 46, 12), (3, 3, 3), (1, 1, 1, 1), (1, 1), (1, 1), 3),
    ("depthwise4-pad-br", (1, 6, 24, 24), (6, 3, 3), (0, 0, 2, 2), (1, 1), (1, 1), 6),
    # whole-plane staging of rows of 14 / 7 floats (16-byte copies of the
    # block's contiguous planes), incl. a last block whose range ends mid-float4
    ("depthwise-flat-14", (2, 32, 14, 14), (32, 3, 3), (1, 1, 1, 1), (1, 1), (1, 1), 32),
    ("depthwise-flat-7-tail", (2, 19, 7, 7), (19, 3, 3), (1, 1, 1, 1), (1, 1), (1, 1), 19),
]


@pytest.mark.parametrize("case", CONV_CASES, ids=[c[0] for c in CONV_CASES])
def test_conv_bitexact(rh, oracle, case):
    name, xs, (O, kh, kw), pads, strides, dil, groups = case
    x = rnd(oracle, 21, *xs)
    w = rnd(oracle, 22, O, xs[1] // groups, kh, kw, scale=0.3)
    b = rnd(oracle, 23, O)
    exp = oracle.conv(x, w, b, pads=pads, strides=strides, dilations=dil, groups=groups)
    got = host(rh.conv(dev(x), dev(w), dev(b), padding=pads, groups=groups, strides=strides,
                       dilations=dil))
    assert_bits(got, exp, name)


def test_depthwise4_fused_residual_clip(rh, oracle):
    """4-column depthwise kernel with the fused residual Add and Clip epilogue."""
    x = rnd(oracle, 35, 2, 16, 28, 28)
    w = rnd(oracle, 36, 16, 1, 3, 3, scale=0.3)
    b = rnd(oracle, 37, 16)
    res = rnd(oracle, 38, 2, 16, 28, 28)
    exp = oracle.clip(oracle.add(oracle.conv(x, w, b, pads=(1, 1, 1, 1), groups=16), res), 0.0, 0.4)
    got = host(rh.conv(dev(x), dev(w), dev(b), padding=(1, 1, 1, 1), groups=16, residual=dev(res),
                       act="clip", act_range=(0.0, 0.4)))
    assert_bits(got, exp, "depthwise4 residual clip")


@pytest.mark.parametrize("shape", [(2, 20, 14, 14, 1), (2, 38, 7, 7, 1), (2, 40, 14, 14, 2), (1, 7, 14, 14, 1)],
                         ids=lambda s: "x".join(map(str, s)))
def test_depthwise_flat_residual_clip(rh, oracle, shape):
    """Whole-plane depthwise blocks (rows of 14 / 7 floats) with the fused
    residual Add and Clip: outputs staged in LDS and stored as 16-byte runs
    where a block's planes allow it, per element otherwise (ragged tails)."""
    N, C, H, W, s = shape
    x = rnd(oracle, 41, N, C, H, W)
    w = rnd(oracle, 42, C, 1, 3, 3, scale=0.3)
    b = rnd(oracle, 43, C)
    oh = (H + 2 - 3) // s + 1
    res = rnd(oracle, 44, N, C, oh, oh)
    exp = oracle.clip(oracle.add(oracle.conv(x, w, b, pads=(1, 1, 1, 1), strides=(s, s), groups=C), res), 0.0, 0.4)
    got = host(rh.conv(dev(x), dev(w), dev(b), padding=(1, 1, 1, 1), strides=(s, s), groups=C, residual=dev(res),
                       act="clip", act_range=(0.0, 0.4)))
    assert_bits(got, exp, "depthwise flat residual clip")


DW_STREAM_CASES = [
    # (N, C, H, stride, act): MobileNetV2's 14x14 / 7x7 / 14 -> 7 depthwise
    # layers and ragged batches (blocks with one or several groups, the ring's
    # short tails)
    (3, 384, 14, 1, "clip"), (5, 576, 14, 1, "clip"), (3, 960, 7, 1, "clip"), (2, 576, 14, 2, "clip"),
    (9, 32, 14, 1, "relu"), (7, 64, 7, 1, None), (11, 16, 14, 2, "relu"), (1, 16, 14, 1, None),
    # 28x28: two row segments per thread (window edges per segment)
    (3, 192, 28, 1, "clip"), (2, 8, 28, 1, "relu"), (5, 12, 28, 1, None),
]


@pytest.mark.parametrize("case", DW_STREAM_CASES, ids=lambda c: "x".join(map(str, c[:4])) + f"-{c[4]}")
def test_depthwise_stream_bitexact(rh, oracle, case):
    """Streaming depthwise kernel (dw_stream.hip: persistent blocks, LDS-DMA
    ring of plane groups) == the reference depthwise + activation, and the
    kernel is the one that ran (its launch counter moves)."""
    import ctypes as C

    N, Ch, H, s, act = case
    x = rnd(oracle, 51, N, Ch, H, H)
    w = rnd(oracle, 52, Ch, 1, 3, 3, scale=0.6)
    b = rnd(oracle, 53, Ch)
    exp = oracle.conv(x, w, b, pads=(1, 1, 1, 1), strides=(s, s), groups=Ch)
    if act == "clip":
        exp = oracle.clip(exp, 0.0, 0.25)
    elif act == "relu":
        exp = np.maximum(exp, np.float32(0.0))
    lib = rh.lib()
    lib.rtenhip_debug_dw_stream_launches.restype = C.c_longlong
    before = lib.rtenhip_debug_dw_stream_launches()
    kw = {"act": act, "act_range": (0.0, 0.25)} if act == "clip" else ({"act": act} if act else {})
    got = host(rh.conv(dev(x), dev(w), dev(b), padding=(1, 1, 1, 1), strides=(s, s), groups=Ch, **kw))
    assert lib.rtenhip_debug_dw_stream_launches() == before + 1
    assert_bits(got, exp, f"dw stream {case}")


def test_conv_fused_residual_relu(rh, oracle):
    """Conv -> Add(residual) -> Relu fused epilogue == the three reference ops."""
    x = rnd(oracle, 31, 2, 64, 14, 14)
    w = rnd(oracle, 32, 256, 64, 1, 1, scale=0.3)
    b = rnd(oracle, 33, 256)
    res = rnd(oracle, 34, 2, 256, 14, 14)
    exp = oracle.relu(oracle.add(oracle.conv(x, w, b), res))
    got = host(rh.conv(dev(x), dev(w), dev(b), residual=dev(res), act="relu"))
    assert_bits(got, exp, "conv+add+relu")
    exp = oracle.clip(oracle.conv(x, w, b), 0.0, 6.0)
    got = host(rh.conv(dev(x), dev(w), dev(b), act="clip", act_range=(0.0, 6.0)))
    assert_bits(got, exp, "conv+clip")


def test_conv_1d(rh, oracle):
    x = rnd(oracle, 41, 2, 6, 30)
    w = rnd(oracle, 42, 5, 6, 3)
    exp = oracle.conv(x, w, None, pads=(1, 1), strides=(2,), dilations=(1,))
    got = host(rh.conv(dev(x), dev(w), None, padding=(1, 1), strides=(2,), dilations=(1,)))
    assert_bits(got, exp, "conv1d")


def test_conv_errors(rh):
    import torch

    x = torch.zeros(1, 3, 4, 4, device="cuda")
    with pytest.raises(rh.OpError) as e:
        rh.conv(x, torch.zeros(2, 2, 3, 3, device="cuda"))
    assert e.value.kind == "IncompatibleInputShapes"
    assert "does not match kernel input channels" in str(e.value)
    with pytest.raises(rh.OpError) as e:
        rh.conv(x, torch.zeros(2, 3, 5, 5, device="cuda"))
    assert str(e.value) == "Input too small for kernel size" and e.value.kind == "InvalidValue"
    with pytest.raises(rh.OpError) as e:
        rh.conv(x, torch.zeros(2, 3, 3, 3, device="cuda"), strides=(0, 0))
    assert str(e.value) == "Strides must be > 0"


# --------------------------------------------------------------------------
# Pooling / normalisation / elementwise
# --------------------------------------------------------------------------

def test_pooling_bitexact(rh, oracle):
    x = rnd(oracle, 51, 2, 6, 17, 17)
    assert_bits(host(rh.max_pool(dev(x), (3, 3), (2, 2), (1, 1, 1, 1))),
                oracle.max_pool(x, (3, 3), (2, 2), (1, 1, 1, 1)), "maxpool")
    for incl in (False, True):
        assert_bits(host(rh.average_pool(dev(x), (3, 3), (2, 2), (1, 1, 1, 1), incl)),
                    oracle.average_pool(x, (3, 3), (2, 2), (1, 1, 1, 1), incl), "avgpool")
    assert_bits(host(rh.max_pool(dev(x), (2, 2), (2, 2), "same")),
                oracle.max_pool(x, (2, 2), (2, 2), padding="same"), "maxpool same")
    g = rnd(oracle, 52, 3, 37, 7, 7)
    assert_bits(host(rh.global_average_pool(dev(g))), oracle.global_average_pool(g), "gap")


@pytest.mark.parametrize("hw", [112, 50])
def test_pooling_plane_kernel_bitexact(rh, oracle, hw):
    """Planes that fit LDS take the plane-staged kernel (ResNet stem maxpool);
    W % 4 != 0 stages with scalar loads."""
    x = rnd(oracle, 53, 2, 3, hw, hw)
    assert_bits(host(rh.max_pool(dev(x), (3, 3), (2, 2), (1, 1, 1, 1))),
                oracle.max_pool(x, (3, 3), (2, 2), (1, 1, 1, 1)), "maxpool")
    for incl in (False, True):
        assert_bits(host(rh.average_pool(dev(x), (3, 3), (1, 1), (1, 1, 1, 1), incl)),
                    oracle.average_pool(x, (3, 3), (1, 1), (1, 1, 1, 1), incl), "avgpool")


def test_batch_norm_bitexact(rh, oracle):
    x = rnd(oracle, 61, 2, 5, 6, 7)
    sc, bi, mu = rnd(oracle, 62, 5), rnd(oracle, 63, 5), rnd(oracle, 64, 5)
    var = oracle.xorshift(65, 5) + np.float32(0.5)
    assert_bits(host(rh.batch_norm(dev(x), dev(sc), dev(bi), dev(mu), dev(var), 1e-5)),
                oracle.batch_norm(x, sc, bi, mu, var, 1e-5), "batchnorm")


@pytest.mark.parametrize("op", ["Relu", "Gelu", "Erf", "Sigmoid", "Tanh", "Exp", "Silu"])
def test_unary_bitexact(rh, oracle, op):
    x = rnd(oracle, 71, 40001, scale=24.0)
    x[:8] = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-30, -1e-30, 104.0], np.float32)
    assert_bits(host(rh.unary(op, dev(x))), oracle.unary(op, x), op)


def test_clip_bitexact(rh, oracle):
    x = rnd(oracle, 72, 1001, scale=20.0)
    x[:8] = np.array([np.nan, -0.0, 0.0, np.inf, -np.inf, 6.0, -1e-30, 7.0], np.float32)
    assert_bits(host(rh.clip(dev(x), 0.0, 6.0)), oracle.clip(x, 0.0, 6.0), "clip")
    assert_bits(host(rh.clip(dev(x), -1.0, 0.0)), oracle.clip(x, -1.0, 0.0), "clip upper zero")


@pytest.mark.parametrize("batch", [1, 2])
def test_conv_clip_nan(rh, oracle, batch):
    """NaN conv outputs through the fused Clip epilogue become lo, as RTen's
    Clamp::clamp makes them (the DMA GEMM at batch 2, the latency GEMM at 1)."""
    x = rnd(oracle, 73, batch, 32, 10, 10)
    x[0, 3, 4, 4] = np.nan
    w = rnd(oracle, 74, 48, 32, 3, 3, scale=0.3)
    b = rnd(oracle, 75, 48)
    exp = oracle.clip(oracle.conv(x, w, b, pads=(1, 1, 1, 1)), 0.0, 6.0)
    assert np.isnan(oracle.conv(x, w, b, pads=(1, 1, 1, 1))).any()
    got = host(rh.conv(dev(x), dev(w), dev(b), padding=(1, 1, 1, 1), act="clip", act_range=(0.0, 6.0)))
    assert_bits(got, exp, "conv+clip with NaN")


@pytest.mark.parametrize("op", ["Add", "Sub", "Mul", "Div"])
@pytest.mark.parametrize("shapes", [((2, 3, 4, 5), (2, 3, 4, 5)), ((2, 3, 4, 5), (5,)),
                                    ((2, 3, 4, 5), (3, 1, 1)), ((2, 3, 4, 5), (1,)),
                                    ((3, 1, 5), (2, 1, 4, 1)), ((32, 12, 128, 128), (32, 1, 1, 128))])
def test_binary_bitexact(rh, oracle, op, shapes):
    a = rnd(oracle, 81, *shapes[0])
    b = rnd(oracle, 82, *shapes[1]) + np.float32(0.75)
    assert_bits(host(rh.binary(op, dev(a), dev(b))), oracle.binary(op, a, b), f"{op} {shapes}")


def test_binary_broadcast_error(rh):
    import torch

    with pytest.raises(rh.OpError) as e:
        rh.add(torch.zeros(2, 3, device="cuda"), torch.zeros(4, device="cuda"))
    assert e.value.kind == "IncompatibleInputShapes"


@pytest.mark.parametrize("shape,axis", [((32, 12, 4, 128), -1), ((7, 300), 1), ((5, 6), 0),
                                        ((3, 5000), -1), ((4, 1, 9), 2)])
def test_softmax_bitexact(rh, oracle, shape, axis):
    x = rnd(oracle, 91, *shape, scale=8.0)
    assert_bits(host(rh.softmax(dev(x), axis)), oracle.softmax(x, axis), f"softmax {shape}")


@pytest.mark.parametrize("shape", [(4, 128, 768), (5, 2), (3, 7, 13), (3, 13, 1024), (7, 64),
                                   (2, 5, 4096), (3, 12), (2, 3, 8), (1, 3, 8192), (9, 24), (5, 40),
                                   (17, 520), (33, 16)])
def test_layer_norm_bitexact(rh, oracle, shape):
    x = rnd(oracle, 92, *shape, scale=4.0)
    sc = rnd(oracle, 93, shape[-1]) + np.float32(1.0)
    bi = rnd(oracle, 94, shape[-1])
    assert_bits(host(rh.layer_normalization(dev(x), dev(sc), dev(bi), -1, 1e-12)),
                oracle.layer_norm(x, sc, bi, -1, 1e-12), f"layernorm {shape}")


@pytest.mark.parametrize("shape,axis", [((6,), 0), ((2, 3), 1), ((2, 3), 0), ((64, 1000), -1), ((3, 4097), 1),
                                        ((4, 37, 5), 1), ((2, 3, 130), 0), ((1, 1), 0)])
def test_log_softmax(rh, oracle, shape, axis):
    """LogSoftmax vs the oracle (libm expf / logf, as Rust's f32::exp / ln).
    The GPU forms exp and ln in f64 rounded once (the correctly rounded
    values); libm's expf / logf differ from those in ~0.05% of arguments by
    1 ULP, so this is a tolerance check (well inside north_star's 1e-4 rel):
    |d| <= 4 ULP of the output scale.  (A 1-ULP change of a row's ln(sum)
    moves every element of the row, so no bit-equal fraction is asserted.)"""
    x = rnd(oracle, 95, *shape, scale=8.0)
    got = host(rh.log_softmax(dev(x), axis))
    exp = oracle.log_softmax(x, axis)
    tol = 4 * np.spacing(np.maximum(np.abs(exp), 1.0).astype(np.float32))
    assert np.all(np.abs(got - exp) <= tol), np.abs(got - exp).max()


def test_log_softmax_reference_kats(rh):
    for c in KATS["log_softmax"]:
        x = np.array(c["x"], np.float32).reshape(c["x_shape"])
        np.testing.assert_allclose(host(rh.log_softmax(dev(x), c["axis"])), np.array(c["y"]).reshape(x.shape),
                                   atol=1e-4, rtol=0)


@pytest.mark.parametrize("shape", [(1, 5, 2), (2, 3, 7, 9), (2, 64, 56, 56), (3, 4, 1027), (4, 6), (1, 2, 3, 4, 5)])
def test_instance_norm_bitexact(rh, oracle, shape):
    x = rnd(oracle, 96, *shape, scale=3.0)
    sc = rnd(oracle, 97, shape[1]) + np.float32(1.0)
    bi = rnd(oracle, 98, shape[1])
    assert_bits(host(rh.instance_normalization(dev(x), dev(sc), dev(bi))), oracle.instance_norm(x, sc, bi),
                f"instancenorm {shape}")


def test_instance_norm_reference_kat_and_errors(rh):
    c = KATS["instance_norm"]
    x = np.array(c["x"], np.float32).reshape(c["x_shape"])
    sc, bi = np.array(c["scale"], np.float32), np.array(c["bias"], np.float32)
    np.testing.assert_allclose(host(rh.instance_normalization(dev(x), dev(sc), dev(bi))),
                               np.array(c["y"]).reshape(x.shape), atol=1e-4, rtol=0)
    for args, msg in [((x[0, 0], sc, bi), "expected input with >= 2 dims"),
                      ((x, sc[:4], bi[:4]), "scale length should match channel count"),
                      ((x, sc, bi[:4]), "bias length should match channel count")]:
        with pytest.raises(rh.OpError) as e:
            rh.instance_normalization(*(dev(a) for a in args))
        assert str(e.value) == msg


def test_log_softmax_instance_norm_graph(rh, oracle):
    """Both ops as graph nodes: eager, captured, replayed."""
    import torch
    import graph_runner
    from rten_hip.graph import ModelSpec

    m = ModelSpec("norms")
    x = m.value("x")
    m.inputs = ["x"]
    sc = m.const("sc", rnd(oracle, 99, 8) + np.float32(1.0))
    bi = m.const("bi", rnd(oracle, 100, 8))
    h = m.op("InstanceNormalization", [x, sc, bi], {"epsilon": 1e-3})
    y = m.op("LogSoftmax", [h], {"axis": 1})
    m.outputs = [y]
    ins = {"x": rnd(oracle, 101, 2, 8, 5, 6, scale=2.0)}
    exp = graph_runner.run(m, ins)[y]
    g = m.to_graph()
    xd = torch.from_numpy(ins["x"]).cuda()
    out = None
    for _ in range(3):
        out = g.run({g.input_ids[0]: xd}, g.output_ids, out=out)
        torch.cuda.synchronize()
        got = out[0].cpu().numpy()
        assert np.all(np.abs(got - exp) <= 4 * np.spacing(np.maximum(np.abs(exp), 1.0))), np.abs(got - exp).max()


# --------------------------------------------------------------------------
# ConvTranspose (src/ops/conv.rs:329-577)
# --------------------------------------------------------------------------

CT_CASES = {
    "s2-k2": ((2, 8, 7, 9), (8, 4, 2, 2), (2, 2), (0, 0, 0, 0), True),
    "s2-k3-pads": ((2, 16, 10, 10), (16, 8, 3, 3), (2, 2), (1, 1, 1, 1), True),
    "s3x2-k4x3-uneven": ((1, 5, 6, 7), (5, 3, 4, 3), (3, 2), (1, 2, 0, 1), False),
    "same-odd-pad": ((2, 6, 5, 5), (6, 4, 4, 3), (2, 2), "same", True),
    "K300-gemm-blocks": ((2, 300, 6, 6), (300, 16, 2, 2), (2, 2), (0, 0, 0, 0), True),
    "s1-k3": ((1, 32, 12, 12), (32, 32, 3, 3), (1, 1), (1, 1, 1, 1), True),
    "single-out-gemv": ((2, 9, 4, 4), (9, 1, 1, 1), (1, 1), (0, 0, 0, 0), False),
}


@pytest.mark.parametrize("case", list(CT_CASES), ids=list(CT_CASES))
def test_conv_transpose_bitexact(rh, oracle, case):
    xs, ws, st, pads, has_b = CT_CASES[case]
    x = rnd(oracle, 131, *xs)
    w = rnd(oracle, 132, *ws, scale=0.2)
    b = rnd(oracle, 133, ws[1]) if has_b else None
    same = pads == "same"
    exp = oracle.conv_transpose(x, w, b, pads=(0, 0, 0, 0) if same else pads, strides=st,
                                padding="same" if same else "fixed")
    got = host(rh.conv_transpose(dev(x), dev(w), dev(b) if has_b else None,
                                 padding="same" if same else pads, strides=st))
    assert_bits(got, exp, f"conv_transpose {case}")


def test_conv_transpose_1d_and_errors(rh, oracle):
    x = rnd(oracle, 134, 2, 6, 11)
    w = rnd(oracle, 135, 6, 5, 3, scale=0.2)
    b = rnd(oracle, 136, 5)
    exp = oracle.conv_transpose(x, w, b, pads=(1, 2), strides=(2,))
    assert_bits(host(rh.conv_transpose(dev(x), dev(w), dev(b), padding=(1, 2), strides=(2,))), exp,
                "conv_transpose 1d")
    with pytest.raises(rh.OpError, match="Input channels does not match kernel input channels"):
        rh.conv_transpose(dev(rnd(oracle, 1, 1, 3, 4, 4)), dev(rnd(oracle, 2, 4, 2, 2, 2)))
    with pytest.raises(rh.OpError, match="Strides must be > 0"):
        rh.conv_transpose(dev(rnd(oracle, 1, 1, 3, 4, 4)), dev(rnd(oracle, 2, 3, 2, 2, 2)), strides=(0, 0))
    with pytest.raises(rh.OpError, match="Input is too small"):
        rh.conv_transpose(dev(rnd(oracle, 1, 1, 3, 4, 4)), dev(rnd(oracle, 2, 3, 2, 3, 3)),
                          padding=(4, 4, 4, 4))


# --------------------------------------------------------------------------
# Gemm / MatMul operators
# --------------------------------------------------------------------------

@pytest.mark.parametrize("batch", [64, 4, 1])
def test_gemm_op_fc_bitexact(rh, oracle, batch):
    """ResNet-50 FC: Gemm(transB=1) with broadcast bias C (matmul.rs:27-81)."""
    a = rnd(oracle, 101, batch, 2048)
    w = rnd(oracle, 102, 1000, 2048, scale=0.05)
    c = rnd(oracle, 103, 1000)
    exp = oracle.gemm_op(a, w, c, trans_b=True)
    got = host(rh.gemm_op(dev(a), dev(w), dev(c), transpose_b=True))
    assert_bits(got, exp, f"fc batch {batch}")


@pytest.mark.parametrize("sa,sb", [((2, 3, 5, 64), (3, 64, 7)), ((4, 33, 70), (70, 9)),
                                   ((2, 12, 128, 64), (2, 12, 64, 128)), ((6, 1, 40), (6, 40, 30)),
                                   # BERT projections: batch folded into M, dense DMA route
                                   ((4, 128, 768), (768, 768)), ((2, 128, 3072), (3072, 768)),
                                   ((3, 100, 260), (260, 1028))])
def test_matmul_bitexact(rh, oracle, sa, sb):
    a = rnd(oracle, 111, *sa)
    b = rnd(oracle, 112, *sb)
    assert_bits(host(rh.matmul(dev(a), dev(b))), oracle.matmul(a, b), f"matmul {sa}x{sb}")


def test_matmul_fused_transpose_view(rh, oracle):
    """QK^T with K^T as a strided view (FusedTranspose, src/ops/fused.rs:45-80)."""
    q = rnd(oracle, 121, 2, 4, 128, 64)
    k = rnd(oracle, 122, 2, 4, 128, 64)
    exp = oracle.matmul(q, np.ascontiguousarray(np.swapaxes(k, -1, -2)))
    got = host(rh.matmul(dev(q), dev(k).transpose(-1, -2)))
    assert_bits(got, exp, "qk^T")


# --------------------------------------------------------------------------
# The reference's known-answer vectors, run on the GPU
# --------------------------------------------------------------------------

KATS = json.load(open(os.path.join(HERE, "golden", "kats.json")))


def test_kats_on_gpu(rh):
    for case in KATS["conv"]:
        x = np.array(case["x"], np.float32).reshape(case["x_shape"])
        w = np.array(case["w"], np.float32).reshape(case["w_shape"])
        b = dev(case["bias"]) if case["bias"] else None
        y = host(rh.conv(dev(x), dev(w), b, padding=case["pads"], groups=case["groups"],
                         strides=case["strides"], dilations=case["dilations"]))
        exp = ([np.float32(p) + np.float32(q) for p, q in case["y_parts"]] if "y_parts" in case
               else case["y"])
        tol = 1e-4 if case["tol"] == "1e4" else 1e-5 * np.abs(np.array(exp)) + 1e-8
        assert (np.abs(y.ravel() - np.array(exp, np.float32)) <= tol).all(), case["source"]
    c = KATS["graph_conv_relu"]
    y = host(rh.relu(rh.conv(dev(np.array(c["x"]).reshape(c["x_shape"])),
                             dev(np.array(c["w"]).reshape(c["w_shape"])), padding=(1, 1, 1, 1))))
    assert (np.abs(y.ravel() - np.array(c["y"], np.float32)) <= 1e-4).all()
    for case in KATS["softmax"]:
        x = np.array(case["x"], np.float32).reshape(case["x_shape"])
        if case.get("transpose_input"):
            xt = dev(x).t()  # strided view, like the reference test's permute
        else:
            xt = dev(x)
        y = host(rh.softmax(xt, case["axis"])).ravel()
        exp = np.array(case["y"], np.float32)
        if case["tol"] == "ulp0":
            assert np.array_equal(y.view(np.uint32), exp.view(np.uint32)), case["source"]
        else:
            assert (np.abs(y - exp) <= 1e-4).all(), case["source"]
    c = KATS["layer_norm"]
    y = host(rh.layer_normalization(dev(np.array(c["x"]).reshape(c["x_shape"])), dev(c["scale"]),
                                    dev(c["bias"]), c["axis"], c["epsilon"])).ravel()
    assert (np.abs(y - np.array(c["y"], np.float32)) <= 1e-4).all()
    for case in KATS["unary"]:
        x = np.array([float(v) for v in case["x"]], np.float32)
        y = host(rh.unary(case["op"], dev(x)))
        exp = np.array([float(v) for v in case["y"]], np.float32)
        m = ~np.isnan(exp)
        assert np.array_equal(np.isnan(y), np.isnan(exp)), case["source"]
        assert (np.abs(y[m] - exp[m]) <= 1e-8 + 1e-5 * np.abs(exp[m])).all(), case["source"]
    c = KATS["global_average_pool"]
    y = host(rh.global_average_pool(dev(np.array(c["x"], np.float32).reshape(c["x_shape"]))))
    assert np.allclose(y.ravel(), c["y"])
    for case in KATS["max_pool"][0]["cases"]:
        x = np.array(KATS["max_pool"][0]["x"], np.float32).reshape(1, 1, 4, 4)
        y = host(rh.max_pool(dev(x), case["kernel"], case["strides"]))
        assert np.allclose(y.ravel(), case["y"])


@pytest.mark.parametrize("case", CONV_CASES, ids=[c[0] for c in CONV_CASES])
def test_conv_bitexact_general_kernel(rh, oracle, case):
    """The register-staged general kernel (DMA path off) is bit-exact too."""
    import ctypes

    lib = rh.lib()
    lib.rtenhip_debug_set_dma.argtypes = [ctypes.c_void_p, ctypes.c_int]
    ctx = rh.default_context()
    lib.rtenhip_debug_set_dma(ctypes.c_void_p(ctx.ptr), 0)
    try:
        test_conv_bitexact(rh, oracle, case)
    finally:
        lib.rtenhip_debug_set_dma(ctypes.c_void_p(ctx.ptr), 1)


# --------------------------------------------------------------------------
# Gather / Where / Cast (gather.rs:21-76, binary_elementwise.rs:850-929,
# convert.rs:6-17): exact data movement, compared bit for bit
# --------------------------------------------------------------------------

def _idev(a):
    import torch

    # np.array keeps 0-d (scalar) indices 0-d; ascontiguousarray would make them 1-d
    return torch.from_numpy(np.array(a, dtype=np.int32, order="C")).cuda()


def test_gather_bitexact(rh, oracle):
    for case in KATS["gather"]["cases"]:
        x = np.array(case["x"], np.float32).reshape(case["x_shape"])
        idx = np.array(case["indices"], np.int32).reshape(case["indices_shape"])
        assert_bits(host(rh.gather(dev(x), _idev(idx), case["axis"])),
                    oracle.gather(x, idx, case["axis"]), case["source"] if "source" in case else "gather")
    rng = np.random.default_rng(5)
    # embedding lookup: [vocab, hidden] table, [batch, seq] ids (negative ids count from the end)
    table = rnd(oracle, 71, 1000, 768)
    ids = rng.integers(-1000, 1000, (32, 128)).astype(np.int32)
    assert_bits(host(rh.gather(dev(table), _idev(ids), 0)), oracle.gather(table, ids, 0), "embedding")
    # strided input view, inner axis, scalar index
    x = rnd(oracle, 72, 6, 50, 7)
    xt = dev(x).transpose(0, 2)
    idx = rng.integers(0, 50, (3, 4)).astype(np.int32)
    assert_bits(host(rh.gather(xt, _idev(idx), 1)), oracle.gather(x.transpose(2, 1, 0), idx, 1), "strided")
    assert_bits(host(rh.gather(dev(x), _idev(np.array(3, np.int32)), -1)), oracle.gather(x, np.array(3), -1), "scalar")
    for case in KATS["gather"]["errors"]:
        x = np.zeros(case["x_shape"], np.float32)
        idx = np.array(case["indices"], np.int32).reshape(case["indices_shape"])
        with pytest.raises(rh.OpError) as e:
            rh.gather(dev(x), _idev(idx), case["axis"])
        assert e.value.code == case["code"] and str(e.value) == case["message"]


def test_where_and_cast_bitexact(rh, oracle):
    for case in KATS["where"]["cases"]:
        c = np.array(case["cond"], np.int32).reshape(case["cond_shape"])
        x = np.array(case["x"], np.float32).reshape(case["x_shape"])
        y = np.array(case["y"], np.float32).reshape(case["y_shape"])
        assert_bits(host(rh.where(_idev(c), dev(x), dev(y))), oracle.where(c, x, y), "where")
    rng = np.random.default_rng(6)
    mask = (rng.random((2, 1, 1, 128)) > 0.3).astype(np.int32)  # BERT mask broadcast
    s = rnd(oracle, 73, 2, 12, 128, 128)
    fill = np.array(-10000.0, np.float32)
    assert_bits(host(rh.where(_idev(mask), dev(s), dev(fill))), oracle.where(mask, s, fill), "mask")
    for case in KATS["where"]["errors"]:
        with pytest.raises(rh.OpError) as e:
            rh.where(_idev(np.array(case["cond"], np.int32)), dev(np.array(case["x"], np.float32)),
                     dev(np.array(case["y"], np.float32)))
        assert e.value.code == case["code"] and str(e.value) == case["message"]
    vals = np.array([0.5, -0.5, 1.9999, -1.9999, 3e9, -3e9, np.nan, np.inf, -np.inf, 2147483520.0,
                     -2147483648.0, 123456789.0, -3.4028235e38, 3.4028235e38], np.float32)
    assert np.array_equal(host(rh.cast(dev(vals), "int32")), oracle.cast_f32_to_i32(vals))
    ints = np.array([0, 1, -1, 16777217, -16777217, 2 ** 31 - 1, -2 ** 31, 123456789], np.int32)
    assert_bits(host(rh.cast(_idev(ints), "float")), oracle.cast_i32_to_f32(ints), "cast i32->f32")
