"""Shared pytest setup.

- registers the ``gpu`` marker (tests that need an MI355X);
- puts ``oracle/`` (the CPU checker) and ``rten-fork_amd/`` (the host package)
  on sys.path;
- builds the oracle library when it is missing (a few seconds of g++).
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# The reference's gemv column blocking depends on its thread count
# (src/gemm.rs:673); pin it so the oracle and the GPU path agree.
os.environ.setdefault("RTEN_NUM_THREADS", "8")
ORACLE_DIR = os.path.join(ROOT, "oracle")
PKG_DIR = os.path.join(ROOT, "rten-fork_amd")
for p in (ORACLE_DIR, PKG_DIR, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an MI355X (HIP device)")
    if not os.path.exists(os.path.join(ORACLE_DIR, "librten_oracle.so")):
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])


@pytest.fixture(scope="session")
def oracle():
    import rten_oracle

    return rten_oracle


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False
