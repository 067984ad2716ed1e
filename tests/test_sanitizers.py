"""Host sanitizers: libfhecore's pure-host code -- moduli, roots, twiddle and
base-conversion tables (gpu-fhe_amd/csrc/host_tables.cpp), the FHEC wire parser (csrc/wire.cpp)
-- and the C oracle, built with AddressSanitizer + UndefinedBehaviorSanitizer
(tests/cpp/Makefile) and run through tests/cpp/host_sanitize.cpp's checks on the CPU: table
correctness, parser fuzzing (single-byte corruption, truncation, overflowing headers), oracle
NTT round trips and HomMult against the schoolbook product.  Any sanitizer report aborts the run."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs a host C++ compiler")
def test_host_code_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", HERE, "host_sanitize"], check=True,
                   stdout=subprocess.DEVNULL)
    # verify_asan_link_order=0: the environment may preload other libraries ahead of the ASan
    # runtime; they are left as they are
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(HERE, "host_sanitize")], env=env, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0 and "host_sanitize OK" in r.stdout, r.stdout + r.stderr
