"""CPU-side checks of the drop-in boundary (no GPU, no compute calls).

- librten_hip.so loads and exports every function include/rten_hip.h declares;
- the Python binding's symbol list matches the header;
- status codes / enums in the header keep RTen's OpError numbering;
- the product path fails loudly (no CPU fallback) when the library is missing.
"""
import ctypes
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rten_hip.h")
PKG = os.path.join(ROOT, "rten-fork_amd")
LIB = os.path.join(PKG, "librten_hip.so")


def header_functions():
    text = open(HEADER).read()
    # strip comments
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    return sorted(set(re.findall(r"\b(rtenhip_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def built():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-j8", "-C", PKG])
    return LIB


def test_header_declares_the_boundary():
    fns = header_functions()
    for must in ("rtenhip_conv_f32", "rtenhip_gemm_f32", "rtenhip_gemm_op_f32", "rtenhip_matmul_f32",
                 "rtenhip_max_pool_f32", "rtenhip_average_pool_f32", "rtenhip_global_average_pool_f32",
                 "rtenhip_batch_norm_f32", "rtenhip_layer_norm_f32", "rtenhip_softmax_f32",
                 "rtenhip_unary_f32", "rtenhip_binary_f32", "rtenhip_graph_run"):
        assert must in fns


def test_library_exports_every_header_symbol(built):
    lib = ctypes.CDLL(built)
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, f"declared in rten_hip.h but not exported: {missing}"


def test_python_binding_lists_header_symbols():
    sys.path.insert(0, PKG)
    import rten_hip

    assert set(rten_hip.EXPORTED_SYMBOLS) == set(header_functions())


def test_status_codes_follow_operror():
    text = open(HEADER).read()
    codes = dict(re.findall(r"RTENHIP_([A-Z_]+)\s*=\s*(\d+)", text))
    assert codes["OK"] == "0"
    assert [codes[k] for k in ("INCORRECT_INPUT_TYPE", "INCORRECT_OUTPUT_TYPE",
                               "INCOMPATIBLE_INPUT_SHAPES", "MISSING_INPUTS",
                               "INVALID_VALUE", "UNSUPPORTED_VALUE", "HIP_ERROR")] == \
        ["1", "2", "3", "4", "5", "6", "7"]


def test_pure_host_entry_points(built):
    """Shape arithmetic runs without a device and matches the reference's
    calc_output_size_and_padding (pooling.rs:27-89)."""
    lib = ctypes.CDLL(built)
    f = lib.rtenhip_output_size_and_padding
    out = (ctypes.c_int64 * 2)()
    pads = (ctypes.c_int64 * 4)()
    pin = (ctypes.c_int64 * 4)(1, 1, 1, 1)
    st = f(ctypes.c_int64(56), ctypes.c_int64(56), ctypes.c_int64(3), ctypes.c_int64(3),
           ctypes.c_int64(2), ctypes.c_int64(2), 0, pin, ctypes.c_int64(1), ctypes.c_int64(1),
           out, pads)
    assert st == 0 and list(out) == [28, 28] and list(pads) == [1, 1, 1, 1]
    # "Same" padding, stride 2, 7x7 on 224 (SAME_UPPER split)
    st = f(ctypes.c_int64(224), ctypes.c_int64(224), ctypes.c_int64(7), ctypes.c_int64(7),
           ctypes.c_int64(2), ctypes.c_int64(2), 1, None, ctypes.c_int64(1), ctypes.c_int64(1),
           out, pads)
    assert st == 0 and list(out) == [112, 112] and list(pads) == [2, 2, 3, 3]
    # Input too small for kernel size
    st = f(ctypes.c_int64(2), ctypes.c_int64(2), ctypes.c_int64(3), ctypes.c_int64(3),
           ctypes.c_int64(1), ctypes.c_int64(1), 0, (ctypes.c_int64 * 4)(0, 0, 0, 0),
           ctypes.c_int64(1), ctypes.c_int64(1), out, pads)
    assert st == 5
    lib.rtenhip_last_error_message.restype = ctypes.c_char_p
    assert lib.rtenhip_last_error_message().decode() == "Input too small for kernel size"


def test_missing_library_fails_loudly(tmp_path):
    """No silent fallback: importing the binding against a tree without the
    built library raises as soon as an op needs it."""
    code = (
        "import sys, os\n"
        f"sys.path.insert(0, {PKG!r})\n"
        "import rten_hip\n"
        "rten_hip.LIB_PATH = os.path.join(%r, 'nope.so')\n"
        "rten_hip._lib = None\n"
        "try:\n"
        "    rten_hip.lib()\n"
        "except RuntimeError as e:\n"
        "    print('raised', e)\n"
        "    sys.exit(0)\n"
        "sys.exit(3)\n" % str(tmp_path)
    )
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "raised" in r.stdout
