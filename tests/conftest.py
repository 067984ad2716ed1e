"""Test configuration: `-m gpu` tests need an MI355X (HIP device); everything else runs on CPU.

The GPU tests are the parity tests proper: they call libfhecore through its C ABI (ctypes) and
compare against the CPU oracle (oracle/, test infrastructure) and the committed golden fixtures
(tests/golden/, generated from the reference by tests/golden/make_golden.py).
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gpu-fhe_amd")
ORACLE = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); parity tests via the C ABI")
    config.addinivalue_line("markers", "slow: long-running")


def _ensure_built():
    lib = os.path.join(PKG, "lib", "libfhecore.so")
    olib = os.path.join(ORACLE, "_build", "liboracle.so")
    if not os.path.exists(olib):
        subprocess.run(["make", "-s", "-C", ORACLE], check=True)
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-j8", "-C", PKG], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def has_gpu():
    import torch

    return torch.cuda.is_available()


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
