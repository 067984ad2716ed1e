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
hommult_*: ct x ct HomMult outputs (d0 = a0 b0, d1 = a0 b1 + a1 b0, d2 = a1 b1 in
    Z_q[X]/(X^N + 1), SURVEY.md §8a') computed ONLY with the reference's own exact vec_mul /
    vec_add / vec_sub (arithmetic.py:3-13) on dtype=object arrays: the schoolbook negacyclic
    product is a sum over offsets i of vec_mul(a_i, X^i b), where X^i b is b shifted by i with the
    wrapped coefficients negated by vec_sub(0, .).  The coefficient-form ring product does not
    depend on the NTT's psi or output ordering, so this pins the headline HomMult to the
    reference's arithmetic (the reference's NTT itself is the identity).  Shapes: N = 4096, L = 2
    on the N = 2^12 chain and N = 2048, L = 8 on the BASELINE configs[2] chain (the 8 largest
    60-bit primes = 1 mod 2^17, valid NTT primes for any N <= 2^16).
vec_N65536_L8: vec_* on the configs[2] modulus chain, 4096 coefficients per limb.
hommult_sampled_N65536_L8: BASELINE configs[2] at its full size (N = 2^16, the 8-limb chain):
    48 output coefficients of d0, d1, d2 for one ciphertext pair, each computed ONLY with the
    reference's own vec_mul / vec_sub / vec_add: coefficient k of a * b in Z_q[X]/(X^N + 1) is
    sum_i a_i * b'_i with b'_i = b_(k - i) for i <= k and -b_(N + k - i) (vec_sub(0, .)) above,
    i.e. ONE vec_mul of a against that signed reversal of b, summed by a vec_add halving tree.
    The inputs are not stored (16 MiB): the test regenerates them from the seed with numpy's
    PCG64 and checks their sha256 first.
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


def ref_negacyclic(arith, a, b, mod_col):
    """a * b mod (X^N + 1, q_l) per limb row, using only the reference's vec_* (object dtype)."""
    L, n = a.shape
    zeros = np.zeros((L, n), dtype=object)
    acc = zeros.copy()
    for i in range(n):
        xb = np.roll(b, i, axis=1)  # X^i b: coefficient k - i moves to k ...
        if i:
            xb[:, :i] = arith.vec_sub(zeros[:, :i], xb[:, :i], mod_col)  # ... X^N = -1 on the wrap
        ai = np.repeat(a[:, i:i + 1], n, axis=1)
        acc = arith.vec_add(acc, arith.vec_mul(ai, xb, mod_col), mod_col)
    return acc


def hommult_fixture(arith, log_n, qs, seed):
    n, L = 1 << log_n, len(qs)
    rng = np.random.default_rng(seed)
    a = np.stack([np.stack([rng.integers(0, q, n, dtype=np.uint64) for q in qs]) for _ in range(2)])
    b = np.stack([np.stack([rng.integers(0, q, n, dtype=np.uint64) for q in qs]) for _ in range(2)])
    for l, q in enumerate(qs):  # edge values: q - 1 and 0 in the leading coefficients
        a[0, l, :3] = [q - 1, 0, q - 1]
        b[1, l, :3] = [q - 1, q - 1, 0]
    mod_col = np.array(qs, dtype=object).reshape(L, 1)
    ao, bo = a.astype(object), b.astype(object)
    d0 = ref_negacyclic(arith, ao[0], bo[0], mod_col)
    d1 = arith.vec_add(ref_negacyclic(arith, ao[0], bo[1], mod_col),
                       ref_negacyclic(arith, ao[1], bo[0], mod_col), mod_col)
    d2 = ref_negacyclic(arith, ao[1], bo[1], mod_col)
    d = np.stack([d0, d1, d2]).astype(np.uint64)
    return {"a": a, "b": b, "d": d, "moduli": np.array(qs, dtype=np.uint64), "log_n": np.array(log_n),
            "seed": np.array(seed), "numpy_version": np.array(np.__version__)}


def vec_chain_fixture(arith, qs, cols, seed):
    """vec_* on given moduli rows (L, cols), reference outputs on object inputs."""
    L = len(qs)
    rng = np.random.default_rng(seed)
    a = np.stack([rng.integers(0, q, cols, dtype=np.uint64) for q in qs])
    b = np.stack([rng.integers(0, q, cols, dtype=np.uint64) for q in qs])
    for i, q in enumerate(qs):
        a[i, :4] = [0, q - 1, q - 1, 5]
        b[i, :4] = [0, q - 1, 1, 5]
    mod_col = np.array(qs, dtype=object).reshape(L, 1)
    out = {"a": a, "b": b, "moduli": np.array(qs, dtype=np.uint64), "seed": np.array(seed),
           "numpy_version": np.array(np.__version__)}
    for op in ("add", "sub", "mul"):
        out[op] = getattr(arith, "vec_" + op)(a.astype(object), b.astype(object), mod_col).astype(np.uint64)
    return out


def sampled_inputs(qs, n, seed):
    """The ciphertext pair of hommult_sampled_*: a, b [2][L][N], uniform residues per limb from
    numpy.random.default_rng(seed) (tests/test_gpu_parity.py regenerates them the same way)."""
    rng = np.random.default_rng(seed)
    a = np.stack([np.stack([rng.integers(0, q, n, dtype=np.uint64) for q in qs]) for _ in range(2)])
    b = np.stack([np.stack([rng.integers(0, q, n, dtype=np.uint64) for q in qs]) for _ in range(2)])
    for l, q in enumerate(qs):  # edge values in the leading and trailing coefficients
        a[0, l, :2] = [q - 1, 0]
        b[1, l, -2:] = [q - 1, q - 1]
    return a, b


def ref_coefficient(arith, a, b, k, mod_col):
    """Coefficient k of a * b mod (X^N + 1, q_l) per limb row, with the reference's vec_* only:
    one vec_mul against b's signed reversal, then a vec_add halving tree (object dtype)."""
    L, n = a.shape
    idx = (k - np.arange(n)) % n                # b index paired with a_i
    rev = b[:, idx]
    wrap = np.arange(n) > k                     # i > k: X^N = -1 flips the sign
    rev[:, wrap] = arith.vec_sub(np.zeros((L, int(wrap.sum())), dtype=object), rev[:, wrap],
                                 mod_col)
    t = arith.vec_mul(a, rev, mod_col)
    while t.shape[1] > 1:
        h = t.shape[1] // 2
        t = arith.vec_add(t[:, :h], t[:, h:], mod_col)
    return t[:, 0]


def hommult_sampled_fixture(arith, qs, log_n, seed, count):
    import hashlib

    n, L = 1 << log_n, len(qs)
    a, b = sampled_inputs(qs, n, seed)
    rng = np.random.default_rng(seed + 1)
    ks = sorted(set([0, 1, 2, n // 2, n - 2, n - 1] +
                    [int(v) for v in rng.choice(n, count, replace=False)]))[:count]
    mod_col = np.array(qs, dtype=object).reshape(L, 1)
    ao, bo = a.astype(object), b.astype(object)
    d = np.zeros((len(ks), 3, L), dtype=np.uint64)
    for j, k in enumerate(ks):
        d[j, 0] = ref_coefficient(arith, ao[0], bo[0], k, mod_col)
        d[j, 1] = arith.vec_add(ref_coefficient(arith, ao[0], bo[1], k, mod_col).reshape(L, 1),
                                ref_coefficient(arith, ao[1], bo[0], k, mod_col).reshape(L, 1),
                                mod_col)[:, 0]
        d[j, 2] = ref_coefficient(arith, ao[1], bo[1], k, mod_col)
    digest = hashlib.sha256(a.tobytes() + b.tobytes()).hexdigest()
    return {"index": np.array(ks, dtype=np.int64), "d": d, "moduli": np.array(qs, dtype=np.uint64),
            "log_n": np.array(log_n), "seed": np.array(seed), "inputs_sha256": np.array(digest),
            "numpy_version": np.array(np.__version__)}


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
    if "--sampled-only" in sys.argv:  # only the configs[2] sampled pin (the others unchanged)
        np.savez(os.path.join(HERE, "hommult_sampled_N65536_L8.npz"),
                 **hommult_sampled_fixture(arith, pyoracle.gen_moduli(16, 8), 16, 17, 48))
        print("wrote hommult_sampled_N65536_L8.npz")
        return
    np.savez(os.path.join(HERE, "vec_N4096_L1.npz"), **vec_fixture(arith, poly, 12, 1, 11, True))
    np.savez(os.path.join(HERE, "vec_N16384_L4.npz"), **vec_fixture(arith, poly, 14, 4, 12, False))
    np.savez(os.path.join(HERE, "ntt_N4096_L1.npz"), **ntt_fixture(12, 13))
    chain16 = pyoracle.gen_moduli(16, 8)  # BASELINE configs[2] chain (SURVEY.md §8a')
    np.savez(os.path.join(HERE, "vec_N65536_L8.npz"), **vec_chain_fixture(arith, chain16, 4096, 14))
    if "--skip-hommult" not in sys.argv:
        np.savez(os.path.join(HERE, "hommult_N4096_L2.npz"),
                 **hommult_fixture(arith, 12, pyoracle.gen_moduli(12, 2), 15))
        np.savez(os.path.join(HERE, "hommult_N2048_L8_chain16.npz"),
                 **hommult_fixture(arith, 11, chain16, 16))
        np.savez(os.path.join(HERE, "hommult_sampled_N65536_L8.npz"),
                 **hommult_sampled_fixture(arith, chain16, 16, 17, 48))
    print("wrote", sorted(f for f in os.listdir(HERE) if f.endswith(".npz")))


if __name__ == "__main__":
    main()
