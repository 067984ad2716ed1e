"""GPU parity for sampling, key generation, encryption and decryption (SURVEY.md §8(f) row 3,
gpu-fhe_amd/csrc/keygen.hip) -- bit-exact against oracle/pyoracle.py's Philox4x32-10 restatement
(itself pinned by Random123's known-answer vectors, tests/test_oracle.py) -- and end-to-end CKKS:
encode -> encrypt -> multiply + relinearise + rescale / rotate -> decrypt -> decode."""
import numpy as np
import pytest

import coracle
import pyoracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fc():
    import fhecore

    return fhecore


@pytest.fixture(scope="module")
def small(fc):
    return fc.Context(10, L=3, K=2, dnum=3)


def H(fc, t):
    return fc.to_host(t).astype(object)


@pytest.mark.parametrize("kind", ["uniform", "ternary", "error"])
def test_sample_matches_oracle(fc, small, kind):
    got = H(fc, small.sample(kind, 2, seed=0x1234_5678_9abc, tag=77))
    lim = list(enumerate(small.all_moduli))
    for p in range(2):
        assert (got[p] == pyoracle.sample(kind, 0x1234_5678_9abc, 77, p, lim, 1 << 10)).all()


def test_keys_and_encryption_match_oracle(fc, small):
    ctx = small
    qs, ps, log_n = ctx.moduli, ctx.all_moduli[ctx.L:], 10
    sk = ctx.keygen_secret(11)
    sk_o = pyoracle.keygen_secret(11, ctx.all_moduli, log_n)
    assert (H(fc, sk) == sk_o).all()
    pk = ctx.keygen_public(sk, 12)
    pk_o = pyoracle.keygen_public(12, sk_o, qs, log_n)
    assert (H(fc, pk) == pk_o).all()
    kb, ka = ctx.keygen_relin(sk, 13)
    col = pyoracle._mods_col(ctx.all_moduli)
    key_o = pyoracle.keygen_switch(13, sk_o, sk_o * sk_o % col, qs, ps, ctx.dnum, log_n)
    assert (H(fc, kb) == key_o[0]).all() and (H(fc, ka) == key_o[1]).all()
    rng = np.random.default_rng(1)
    pt = np.stack([rng.integers(0, q, 1 << log_n, dtype=np.uint64) for q in qs])
    ct = ctx.encrypt(fc.to_device(pt), pk, 14)
    assert (H(fc, ct) == pyoracle.encrypt(14, pt.astype(object), pk_o, qs, log_n)).all()
    ct2 = ctx.encrypt_sk(fc.to_device(pt), sk, 15)
    assert (H(fc, ct2) == pyoracle.encrypt_sk(15, pt.astype(object), sk_o, qs, log_n)).all()
    assert (H(fc, ctx.decrypt(ct2, sk)) == pyoracle.decrypt(H(fc, ct2), sk_o, qs)).all()


def _ckks(fc, log_n=13, L=4, K=2, dnum=2):
    from fhecore.ckks import Encoder, from_rns, to_rns

    ctx = fc.Context(log_n, L=L, K=K, dnum=dnum)
    sk = ctx.keygen_secret(1)
    pk = ctx.keygen_public(sk, 2)
    enc = Encoder(1 << log_n)

    def encrypt(z, delta, seed):
        pt = fc.to_device(to_rns(enc.encode(z, delta), ctx.moduli))
        ctx.ntt_(pt)
        return ctx.encrypt(pt, pk, seed)

    def decrypt(ct, delta):
        pt = ctx.decrypt(ct, sk)
        ctx.intt_(pt)
        return enc.decode(from_rns(fc.to_host(pt), ctx.moduli[:ct.shape[-2]]), delta)

    return ctx, sk, encrypt, decrypt


def test_ckks_multiply_relin_rescale_end_to_end(fc):
    ctx, sk, encrypt, decrypt = _ckks(fc)
    rng = np.random.default_rng(3)
    z1 = rng.uniform(-1, 1, ctx.n // 2) + 1j * rng.uniform(-1, 1, ctx.n // 2)
    z2 = rng.uniform(-1, 1, ctx.n // 2) + 1j * rng.uniform(-1, 1, ctx.n // 2)
    # delta ~ 2^50 so the product's scale after dropping a 60-bit prime stays at 2^40
    delta = 2.0 ** 50
    c1, c2 = encrypt(z1, delta, 10), encrypt(z2, delta, 11)
    assert np.abs(decrypt(c1, delta) - z1).max() < 1e-9
    kb, ka = ctx.keygen_relin(sk, 4)
    out = ctx.mul_relin(c1, c2, kb, ka, rescale=True)
    got = decrypt(out, delta * delta / ctx.moduli[-1])
    assert np.abs(got - z1 * z2).max() < 1e-7


def test_ckks_rotation_end_to_end(fc):
    ctx, sk, encrypt, decrypt = _ckks(fc)
    rng = np.random.default_rng(4)
    z = rng.uniform(-1, 1, ctx.n // 2) + 1j * rng.uniform(-1, 1, ctx.n // 2)
    delta = 2.0 ** 50
    ct = encrypt(z, delta, 20)
    for step in (1, -3):
        k = ctx.galois_elt(step)
        rb, ra = ctx.keygen_rotation(sk, k, 5 + step)
        got = decrypt(ctx.rotate(ct, k, rb, ra), delta)
        assert np.abs(got - np.roll(z, -step)).max() < 1e-7
