"""GPU parity for SURVEY.md §8(f) row 1 -- rescale, Galois automorphisms and rotation
(gpu-fhe_amd/csrc/galois.hip through the C ABI) -- against oracle/pyoracle.py, bit-exact.

None of these exist in the reference (parity unpinned by the reference); the oracle restates the
standard RNS-CKKS definitions and tests/test_oracle.py checks it (CRT divide-and-round, NTT/coefficient
consistency, ring homomorphism, real-key rotation decryption)."""
import random

import numpy as np
import pytest

import coracle
import pyoracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fc():
    import fhecore

    return fhecore


def rand(mods, log_n, lead=(), seed=0):
    rng = np.random.default_rng(seed)
    n = 1 << log_n
    return np.stack([rng.integers(0, q, size=lead + (n,), dtype=np.uint64) for q in mods],
                    axis=len(lead))


@pytest.mark.parametrize("log_n,L", [(10, 3), (12, 2), (16, 4)])
@pytest.mark.parametrize("step", [1, -2, 7, "conj"])
def test_automorphism_matches_oracle(fc, log_n, L, step):
    ctx = fc.Context(log_n, L=L)
    n = 1 << log_n
    k = 2 * n - 1 if step == "conj" else ctx.galois_elt(step)
    assert k == (2 * n - 1 if step == "conj" else pyoracle.galois_elt(step, n))
    x = rand(ctx.moduli, log_n, (2,), seed=log_n)
    # NTT form: a gather by the oracle's index map
    got = fc.to_host(ctx.automorphism(fc.to_device(x), k, ntt_form=True))
    idx = pyoracle.automorphism_ntt_index(k, log_n)
    assert (got == x[..., idx]).all()
    # coefficient form: the signed permutation, and it commutes with the NTT
    xc = x[0]
    got = fc.to_host(ctx.automorphism(fc.to_device(xc), k, ntt_form=False))
    if log_n <= 12:
        want = pyoracle.automorphism_coeff(xc.astype(object), k, ctx.moduli)
        assert (got.astype(object) == want).all()
    assert (coracle.ntt_fwd(got[None], ctx.moduli)[0] ==
            coracle.ntt_fwd(xc[None], ctx.moduli)[0][..., idx]).all()


def test_automorphism_rejects_even_element_and_alias(fc):
    ctx = fc.Context(10, L=1)
    x = fc.to_device(rand(ctx.moduli, 10))
    with pytest.raises(fc.FheError):
        ctx.automorphism(x, 4)
    from fhecore._capi import load
    from fhecore.context import _ptr, _stream

    assert load().fhe_automorphism(ctx.handle, _ptr(x), _ptr(x), 1, 0, 1, 5, 1, _stream(x)) != 0


@pytest.mark.parametrize("log_n,L,polys", [(10, 2, 1), (12, 4, 3), (16, 8, 2)])
def test_rescale_coeff_matches_oracle(fc, log_n, L, polys):
    ctx = fc.Context(log_n, L=L)
    x = rand(ctx.moduli, log_n, (polys,), seed=L)
    got = fc.to_host(ctx.rescale(fc.to_device(x), ntt_form=False))
    assert got.shape == (polys, L - 1, 1 << log_n)
    for p in range(polys):
        want = pyoracle.rescale_coeff(x[p].astype(object), ctx.moduli)
        assert (got[p].astype(object) == want).all()


@pytest.mark.parametrize("log_n,L,polys", [(10, 3, 2), (14, 4, 1), (16, 8, 2)])
def test_rescale_ntt_matches_oracle(fc, log_n, L, polys):
    ctx = fc.Context(log_n, L=L)
    x = rand(ctx.moduli, log_n, (polys,), seed=L + 1)
    got = fc.to_host(ctx.rescale(fc.to_device(x), ntt_form=True))
    for p in range(polys):
        c = coracle.ntt_inv(x[p][None], ctx.moduli)[0]
        r = pyoracle.rescale_coeff(c.astype(object), ctx.moduli)
        want = coracle.ntt_fwd(np.asarray(r, dtype=np.uint64)[None], ctx.moduli[:-1])[0]
        assert (got[p] == want).all()


def test_rescale_partial_level_and_errors(fc):
    """Rescaling a ciphertext already at level l < L uses q_{l-1} as the dropped modulus."""
    ctx = fc.Context(12, L=4)
    x = rand(ctx.moduli[:3], 12, (1,), seed=9)
    got = fc.to_host(ctx.rescale(fc.to_device(x), ntt_form=False))
    assert (got[0].astype(object) == pyoracle.rescale_coeff(x[0].astype(object),
                                                             ctx.moduli[:3])).all()
    with pytest.raises(fc.FheError):
        ctx.rescale(fc.to_device(rand(ctx.moduli[:1], 12, (1,))), ntt_form=False)


def test_rotate_matches_oracle_and_decrypts(fc):
    """fhe_rotate = (sigma c0 + KS0(sigma c1), KS1(sigma c1)), bit-exact vs the oracle; with a real
    rotation key the result decrypts to the rotated message."""
    log_n, L, K, dnum = 10, 3, 2, 3
    n = 1 << log_n
    ctx = fc.Context(log_n, L=L, K=K, dnum=dnum)
    qs, ps = ctx.moduli, ctx.all_moduli[L:]
    rng = random.Random(3)
    s = [rng.randrange(-1, 2) for _ in range(n)]
    m = [rng.randrange(-1000, 1000) for _ in range(n)]
    col = pyoracle._mods_col(qs)
    s_n = coracle.ntt_fwd(np.asarray(pyoracle._to_rns(s, qs), dtype=np.uint64), qs).astype(object)
    a = np.stack([np.array([rng.randrange(q) for _ in range(n)], dtype=object) for q in qs])
    e = coracle.ntt_fwd(np.asarray(pyoracle._to_rns([rng.randrange(-3, 4) for _ in range(n)], qs),
                                   dtype=np.uint64), qs).astype(object)
    m_n = coracle.ntt_fwd(np.asarray(pyoracle._to_rns(m, qs), dtype=np.uint64), qs).astype(object)
    ct = np.stack([(-a * s_n + e + m_n) % col, a]).astype(np.uint64)
    k = ctx.galois_elt(1)
    rb, ra = pyoracle.gen_rot_key(s, k, qs, ps, dnum, rng)
    rb, ra = rb.astype(np.uint64), ra.astype(np.uint64)
    got = fc.to_host(ctx.rotate(fc.to_device(ct), k, fc.to_device(rb), fc.to_device(ra)))
    # oracle: automorphisms + the C key-switch restatement
    c0 = ct[0][..., pyoracle.automorphism_ntt_index(k, log_n)]
    c1 = ct[1][..., pyoracle.automorphism_ntt_index(k, log_n)]
    ks0, ks1 = coracle.keyswitch(c1, rb, ra, qs, ps, dnum)
    assert (got[1] == ks1).all()
    assert (got[0].astype(object) == (c0.astype(object) + ks0.astype(object)) % col).all()
    dec = pyoracle.crt_centered(
        coracle.ntt_inv(((got[0].astype(object) + got[1].astype(object) * s_n) % col)
                        .astype(np.uint64), qs).astype(object), qs)
    want = pyoracle.automorphism_coeff(np.array([[v % qs[0] for v in m]], dtype=object), k,
                                       [qs[0]])[0]
    want = [int(v) - qs[0] if int(v) > qs[0] // 2 else int(v) for v in want]
    assert max(abs(int(d) - w) for d, w in zip(dec, want)) < 1 << 20


def test_rotate_batch_matches_single(fc):
    log_n, L, K, dnum = 12, 4, 2, 2
    ctx = fc.Context(log_n, L=L, K=K, dnum=dnum)
    ct = rand(ctx.moduli, log_n, (3, 2), seed=1)
    allm = ctx.all_moduli
    rb = rand(allm, log_n, (dnum,), seed=2)
    ra = rand(allm, log_n, (dnum,), seed=3)
    k = ctx.galois_elt(5)
    d = lambda v: fc.to_device(np.ascontiguousarray(v))  # noqa: E731
    batched = fc.to_host(ctx.rotate(d(ct), k, d(rb), d(ra)))
    for b in range(3):
        assert (fc.to_host(ctx.rotate(d(ct[b]), k, d(rb), d(ra))) == batched[b]).all()


def _real_ct(ctx, log_n, rng):
    """A real encryption of a small message under a ternary secret (NTT form), as above."""
    n = 1 << log_n
    qs = ctx.moduli
    s = [rng.randrange(-1, 2) for _ in range(n)]
    m = [rng.randrange(-1000, 1000) for _ in range(n)]
    col = pyoracle._mods_col(qs)
    ntt = lambda v: coracle.ntt_fwd(np.asarray(pyoracle._to_rns(v, qs), dtype=np.uint64),  # noqa: E731
                                    qs).astype(object)
    s_n = ntt(s)
    a = np.stack([np.array([rng.randrange(q) for _ in range(n)], dtype=object) for q in qs])
    ct = np.stack([(-a * s_n + ntt([rng.randrange(-3, 4) for _ in range(n)]) + ntt(m)) % col, a])
    return ct.astype(np.uint64), s, s_n, m


@pytest.mark.parametrize("log_n,L,K,dnum", [
    (10, 3, 2, 3), (11, 4, 2, 2),
    # the branches with an unfused ModDown -- K > 4 (the separate sigma(c0) pass,
    # k_moddown_finish) and dnum > 4 (k_ks_inner's u128 sums with the gather)
    (10, 6, 5, 2), (10, 6, 2, 6)])
def test_rotate_hoisted_matches_oracle_and_decrypts(fc, log_n, L, K, dnum):
    """fhe_rotate_hoisted (one ModUp, the automorphism gathered inside the inner product) bit-exact
    vs pyoracle.rotate_hoisted for several Galois elements at once; every output decrypts to the
    rotated message."""
    n = 1 << log_n
    ctx = fc.Context(log_n, L=L, K=K, dnum=dnum)
    qs, ps = ctx.moduli, ctx.all_moduli[L:]
    rng = random.Random(log_n)
    ct, s, s_n, m = _real_ct(ctx, log_n, rng)
    ks = [ctx.galois_elt(1), ctx.galois_elt(-2), 2 * n - 1]
    keys = [pyoracle.gen_rot_key(s, k, qs, ps, dnum, rng) for k in ks]
    keys = [(rb.astype(np.uint64), ra.astype(np.uint64)) for rb, ra in keys]
    d = lambda v: fc.to_device(np.ascontiguousarray(v))  # noqa: E731
    got = fc.to_host(ctx.rotate_hoisted(d(ct), ks, [(d(rb), d(ra)) for rb, ra in keys]))
    want = pyoracle.rotate_hoisted(ct, ks, keys, qs, ps, dnum, log_n)
    assert got.shape == (len(ks), 2, L, n)
    assert (got.astype(object) == want).all()
    col = pyoracle._mods_col(qs)
    for k, out in zip(ks, got):
        dec = pyoracle.crt_centered(
            coracle.ntt_inv(((out[0].astype(object) + out[1].astype(object) * s_n) % col)
                            .astype(np.uint64), qs).astype(object), qs)
        mk = pyoracle.automorphism_coeff(np.array([[v % qs[0] for v in m]], dtype=object), k,
                                         [qs[0]])[0]
        mk = [int(v) - qs[0] if int(v) > qs[0] // 2 else int(v) for v in mk]
        assert max(abs(int(x) - w) for x, w in zip(dec, mk)) < 1 << 20


def test_rotate_hoisted_batch_matches_single_and_errors(fc):
    log_n, L, K, dnum = 12, 4, 2, 2
    ctx = fc.Context(log_n, L=L, K=K, dnum=dnum)
    ct = rand(ctx.moduli, log_n, (3, 2), seed=4)
    allm = ctx.all_moduli
    keys = [(rand(allm, log_n, (dnum,), seed=5 + 2 * r), rand(allm, log_n, (dnum,), seed=6 + 2 * r))
            for r in range(2)]
    ks = [ctx.galois_elt(3), ctx.galois_elt(-7)]
    d = lambda v: fc.to_device(np.ascontiguousarray(v))  # noqa: E731
    dk = [(d(rb), d(ra)) for rb, ra in keys]
    batched = fc.to_host(ctx.rotate_hoisted(d(ct), ks, dk))
    assert batched.shape == (2, 3, 2, L, 1 << log_n)
    for b in range(3):
        assert (fc.to_host(ctx.rotate_hoisted(d(ct[b]), ks, dk)) == batched[:, b]).all()
    # a single hoisted rotation: same pipeline, count 1
    assert (fc.to_host(ctx.rotate_hoisted(d(ct), ks[1:], dk[1:]))[0] == batched[1]).all()
    with pytest.raises(fc.FheError):
        ctx.rotate_hoisted(d(ct), [4], dk[:1])  # even Galois element
    # a caller-supplied out must be a HIP int64/uint64 tensor on the ct's device
    import torch

    shape = (2, 3, 2, L, 1 << log_n)
    with pytest.raises(TypeError):
        ctx.rotate_hoisted(d(ct), ks, dk, out=torch.empty(shape, dtype=torch.int64))  # on CPU
    with pytest.raises(TypeError):
        ctx.rotate_hoisted(d(ct), ks, dk, out=torch.empty(shape, dtype=torch.float64,
                                                          device="cuda"))
    with pytest.raises(ValueError):
        ctx.rotate_hoisted(d(ct), ks, dk, out=torch.empty((1,) + shape[1:], dtype=torch.int64,
                                                          device="cuda"))
    # ... and a null key pointer inside the per-rotation arrays is refused at the C ABI
    import ctypes

    from fhecore import _capi

    lib = _capi.load()
    ctd = d(ct)
    out = torch.empty(shape, dtype=torch.int64, device="cuda")
    g_arr = (ctypes.c_uint32 * 2)(*ks)
    b_arr = (ctypes.c_void_p * 2)(dk[0][0].data_ptr(), None)
    a_arr = (ctypes.c_void_p * 2)(dk[0][1].data_ptr(), dk[1][1].data_ptr())
    rc = lib.fhe_rotate_hoisted(ctx.handle, out.data_ptr(), ctd.data_ptr(), g_arr, b_arr, a_arr,
                                2, 3, None, None)
    assert rc == -1 and b"null key pointer" in lib.fhe_last_error()


def test_rotate_and_mul_relin_in_cache_sized_passes(fc):
    """fhe_rotate and fhe_mul_relin run a batch above 256 MiB of d2 in passes (N = 2^16, L = 16:
    32 ciphertexts per pass): 33 ciphertexts, each one equal to its own single-ciphertext call
    (ciphertexts 0 and 31 in the first pass, 32 alone in the second)."""
    import torch

    log_n, L, K, dnum, B = 16, 16, 4, 4, 33
    ctx = fc.Context(log_n, L=L, K=K, dnum=dnum)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(33)

    def rows(mods, lead):
        return torch.stack([torch.randint(0, q, lead + (1 << log_n,), generator=gen,
                                          dtype=torch.int64, device="cuda") for q in mods], len(lead))

    ct = rows(ctx.moduli, (B, 2))
    ct2 = rows(ctx.moduli, (B, 2))
    kb, ka = rows(ctx.all_moduli, (dnum,)), rows(ctx.all_moduli, (dnum,))
    k = ctx.galois_elt(3)
    rot = ctx.rotate(ct, k, kb, ka)
    mr = ctx.mul_relin(ct, ct2, kb, ka, rescale=True)
    for b in (0, 31, 32):
        assert torch.equal(ctx.rotate(ct[b:b + 1], k, kb, ka), rot[b:b + 1]), b
        assert torch.equal(ctx.mul_relin(ct[b:b + 1], ct2[b:b + 1], kb, ka, rescale=True),
                           mr[b:b + 1]), b
