"""Device shortcuts of rten-vecmath arithmetic (csrc/vecmath.h) against their
plain forms, bit for bit, on random and edge operands:
- div_by: softmax's p = e / sum with the divisor-only steps of the compiler's
  f32 division done once (used by the attention kernel), vs __fdiv_rn;
- vm_exp2: two vm_exp (rten-vecmath exp.rs:12-80 restatement) as packed f32
  operations, vs vm_exp;
- vm_gelu2: two vm_gelu (erf.rs:29-91) as packed operations (the GEMM
  epilogue's Gelu), vs vm_gelu.
Called through rtenhip_debug_vecmath_check (a test-only entry point)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    import torch
    import rten_hip
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    L = rten_hip.lib()
    L.rtenhip_debug_vecmath_check.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                              ctypes.c_void_p, ctypes.c_void_p]
    return L


def _run(lib, a, b):
    import torch
    ad, bd = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    out = torch.empty(7 * a.size, dtype=torch.float32, device="cuda")
    assert lib.rtenhip_debug_vecmath_check(ad.data_ptr(), bd.data_ptr(), a.size, out.data_ptr(), None) == 0
    torch.cuda.synchronize()
    return out.cpu().numpy().reshape(7, a.size)


def _bits(x):
    return x.view(np.uint32)


def test_div_by_matches_fdiv(lib):
    rng = np.random.default_rng(1)
    n = 1 << 23
    # softmax's range: e in [0, 1] (uniform, log-uniform down to 2^-80, exact
    # zeros), sum in [1, 128]; plus divisors and numerators outside the
    # shortcut's range (they take __fdiv_rn).
    a = np.concatenate([rng.random(n // 2, dtype=np.float32),
                        np.exp2(-rng.random(n // 4) * 80).astype(np.float32),
                        np.zeros(n // 16, np.float32), -np.zeros(n // 16, np.float32),
                        rng.uniform(-4, 4, n // 8).astype(np.float32)])
    b = np.concatenate([rng.uniform(1, 128, n - n // 16).astype(np.float32),
                        np.exp2(rng.uniform(-10, 20, n // 16)).astype(np.float32)])
    b[:8] = [1.0, np.nextafter(np.float32(1), np.float32(2)), 127.99999, 128.0, 256.0, 3.0, 7.0, 1.5]
    o = _run(lib, a, b)
    bad = _bits(o[0]) != _bits(o[1])
    assert not bad.any(), (a[bad][:5], b[bad][:5], o[0][bad][:5], o[1][bad][:5])


def test_vm_exp2_matches_vm_exp(lib):
    rng = np.random.default_rng(2)
    n = 1 << 22
    x = np.concatenate([rng.uniform(-110, 110, n // 2), rng.uniform(-1, 1, n // 4),
                        -rng.exponential(20, n // 4)]).astype(np.float32)
    x[:6] = [np.inf, -np.inf, np.nan, 104.0, -104.0, 0.0]
    o = _run(lib, x, np.ones_like(x))
    assert np.array_equal(_bits(o[2]), _bits(o[3]))


def test_vm_exp2_nonpos_matches_vm_exp2(lib):
    """The softmax / GELU exp (x <= 0 or NaN: attention's x - max, GELU's
    -z^2) equals vm_exp2 bit for bit, the clamp boundary and -inf included."""
    rng = np.random.default_rng(4)
    n = 1 << 22
    x = -np.concatenate([rng.uniform(0, 110, n // 4), rng.uniform(0, 1, n // 4),
                         rng.exponential(20, n // 4), rng.uniform(103, 105, n // 8),
                         np.exp2(rng.uniform(-140, 120, n // 8))]).astype(np.float32)
    x[:8] = [-np.inf, np.nan, -104.0, np.nextafter(np.float32(-104), np.float32(0)), 0.0, -0.0,
             -1e-45, -3.4e38]
    o = _run(lib, x, np.ones_like(x))
    assert np.array_equal(_bits(o[6]), _bits(o[2]))


def test_vm_gelu2_matches_vm_gelu(lib):
    rng = np.random.default_rng(3)
    n = 1 << 22
    x = np.concatenate([rng.normal(0, 3, n // 2), rng.uniform(-2000, 2000, n // 4),
                        rng.uniform(-1e-3, 1e-3, n // 4)]).astype(np.float32)
    x[:7] = [np.inf, -np.inf, np.nan, 0.0, -0.0, 1e-40, -1e-40]
    o = _run(lib, x, np.ones_like(x))
    assert np.array_equal(_bits(o[4]), _bits(o[5]))
