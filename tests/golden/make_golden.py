#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ (run HERE, where /root/reference exists).

Data only: every .npz holds uint64 arrays and small metadata; nothing from the reference's
source is stored.  Regenerate with
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

vec_{add,sub,mul}: outputs of the reference itself (/root/reference/arithmetic.py:3-13), imported
    and called on dtype=object inputs so that it computes exact Python-int results (SURVEY.md
    §8c).  The reference's own uint64-dtype outputs are recorded too, as the documented divergence
    (a - b and a * b wrap mod 2^64 before the % there).
poly_add:  the reference's ' polynomial.py':3-5 called on a 2-component ciphertext; it returns
    None (recorded as ref_returns_none).
ntt_N4096_L1: the O(N^2) defining sum of SURVEY.md §8a' evaluated in Python big ints (the
    reference's NTT is the identity, arithmetic.py:15-16, so it cannot pin this).
"""
import importlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import pyoracle  # noqa: E402  (moduli + psi for the NTT fixture)


def load_reference():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    arithmetic = importlib.import_module("arithmetic")
    polynomial = importlib.import_module(" polynomial")
    return arithmetic, polynomial


def vec_fixture(arith, poly, log_n, L, seed, keep_u64):
    n = 1 << log_n
    qs = pyoracle.gen_moduli(log_n, L)
    rng = np.random.default_rng(seed)
    a = np.stack([rng.integers(0, q, n, dtype=np.uint64) for q in qs])
    b = np.stack([rng.integers(0, q, n, dtype=np.uint64) for q in qs])
    # edge values in the first few slots: 0, q-1, equal operands
    for i, q in enumerate(qs):
        a[i, :4] = [0, q - 1, q - 1, 5]
        b[i, :4] = [0, q - 1, 1, 5]
    mod_col = np.array(qs, dtype=object).reshape(L, 1)
    ao, bo = a.astype(object), b.astype(object)
    out = {"a": a, "b": b, "moduli": np.array(qs, dtype=np.uint64),
           "seed": np.array(seed), "numpy_version": np.array(np.__version__)}
    for op in ("add", "sub", "mul"):
        r = getattr(arith, "vec_" + op)(ao, bo, mod_col)
        out[op] = r.astype(np.uint64)
        if keep_u64:
            mod_u = np.array(qs, dtype=np.uint64).reshape(L, 1)
            out[op + "_ref_uint64"] = getattr(arith, "vec_" + op)(a, b, mod_u).astype(np.uint64)
    ct_a, ct_b = (ao, bo), (bo, ao)
    out["ref_poly_add_returns_none"] = np.array(poly.poly_add(ct_a, ct_b, mod_col) is None)
    return out


def ntt_fixture(log_n, seed):
    n = 1 << log_n
    q = pyoracle.gen_moduli(log_n, 1)[0]
    rng = np.random.default_rng(seed)
    x = rng.integers(0, q, n, dtype=np.uint64)
    x[:2] = [q - 1, 0]
    y = pyoracle.ntt_naive([int(v) for v in x], q)
    return {"x": x.reshape(1, n), "y": np.array(y, dtype=np.uint64).reshape(1, n),
            "moduli": np.array([q], dtype=np.uint64), "psi": np.array(pyoracle.psi_for(q, n), dtype=np.uint64),
            "seed": np.array(seed)}


def main():
    arith, poly = load_reference()
    np.savez(os.path.join(HERE, "vec_N4096_L1.npz"), **vec_fixture(arith, poly, 12, 1, 11, True))
    np.savez(os.path.join(HERE, "vec_N16384_L4.npz"), **vec_fixture(arith, poly, 14, 4, 12, False))
    np.savez(os.path.join(HERE, "ntt_N4096_L1.npz"), **ntt_fixture(12, 13))
    print("wrote", sorted(f for f in os.listdir(HERE) if f.endswith(".npz")))


if __name__ == "__main__":
    main()
