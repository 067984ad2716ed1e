"""CPU tests of the CKKS canonical-embedding encoder (gpu-fhe_amd/fhecore/ckks.py, SURVEY.md §8(f)
row 3): round trip, slot-wise products from negacyclic polynomial products, and the Galois element
5 rotating the slots by one.  Host-side data boundary; no GPU."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gpu-fhe_amd"))
from fhecore.ckks import Encoder, from_rns, to_rns  # noqa: E402

import pyoracle  # noqa: E402


def _z(rng, k):
    return rng.uniform(-1, 1, k) + 1j * rng.uniform(-1, 1, k)


def test_round_trip():
    rng = np.random.default_rng(0)
    enc = Encoder(1 << 10)
    z = _z(rng, 512)
    assert np.abs(enc.decode(enc.encode(z, 2.0 ** 40), 2.0 ** 40) - z).max() < 1e-9


def test_product_is_slotwise():
    rng = np.random.default_rng(1)
    n = 64
    enc = Encoder(n)
    z1, z2 = _z(rng, n // 2), _z(rng, n // 2)
    d = 2.0 ** 20
    m1, m2 = enc.encode(z1, d), enc.encode(z2, d)
    prod = [0] * n  # exact integer negacyclic product
    for i in range(n):
        for j in range(n):
            k = i + j
            if k < n:
                prod[k] += int(m1[i]) * int(m2[j])
            else:
                prod[k - n] -= int(m1[i]) * int(m2[j])
    assert np.abs(enc.decode(np.array(prod, dtype=np.float64), d * d) - z1 * z2).max() < 1e-4


def test_galois_5_rotates_slots():
    rng = np.random.default_rng(2)
    n = 64
    enc = Encoder(n)
    z = _z(rng, n // 2)
    d = 2.0 ** 30
    q = pyoracle.gen_moduli(6, 1)[0]
    m = enc.encode(z, d)
    x = to_rns(m, [q])
    y = pyoracle.automorphism_coeff(x.astype(object), pyoracle.galois_elt(1, n), [q])
    got = enc.decode(from_rns(np.asarray(y, dtype=np.uint64), [q]), d)
    assert np.abs(got - np.roll(z, -1)).max() < 1e-6


def test_rns_round_trip():
    qs = pyoracle.gen_moduli(10, 3)
    c = np.array([-5, 0, 7, -(2 ** 61), 2 ** 61 - 1] + [3] * 1019, dtype=np.int64)
    assert (from_rns(to_rns(c, qs), qs) == c.astype(np.float64)).all()
