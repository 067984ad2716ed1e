"""The header-only C++ Context/Ciphertext/Evaluator (include/fhecore.hpp) compiles against the C ABI
and, on a GPU, multiplies ciphertexts bit-exactly (checked inside the program against a schoolbook
negacyclic product)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "test_fhecore")


def _build():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "gpu-fhe_amd"), "cpptest"], check=True)


def test_cpp_api_compiles():
    _build()
    assert os.access(BIN, os.X_OK)


@pytest.mark.gpu
def test_cpp_api_runs_on_gpu():
    if not os.access(BIN, os.X_OK):
        _build()
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "cpp api ok" in r.stdout
