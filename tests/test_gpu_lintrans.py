"""GPU parity for the baby-step / giant-step linear transform with both hoistings
(fhe_linear_transform, csrc/galois.hip launch_linear_transform) and its giant-step sum over
different ciphertexts (fhe_rotate_sum_multi, launch_rotate_sum_multi): CKKS bootstrapping's
CoeffToSlot / SlotToCoeff shape, the widening after SURVEY.md §8(f) rows 1 and 4.

Not in the reference (parity unpinned by the reference); oracle/pyoracle.py linear_transform and
rotate_sum_multi (checked by real-key decryption in tests/test_oracle.py) are the checkers,
bit-exact.  At the configs[3] shape, where the Python oracle is too slow, the transform is checked
word for word against its definition through the device's own primitives (each giant step's inner
sum = fhe_rotate_sum_hoisted, the outer sum = fhe_rotate_sum_multi), which the smaller cases and
tests/test_gpu_rotsum.py pin to the oracles."""
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


def dev(fc, v):
    return fc.to_device(np.ascontiguousarray(v))


def keys_for(fc, elts, allm, log_n, dnum, seed):
    """Uniform keys per rotated element (None for element 1): host and device forms."""
    host = [None if k == 1 else (rand(allm, log_n, (dnum,), seed + 2 * r),
                                 rand(allm, log_n, (dnum,), seed + 2 * r + 1))
            for r, k in enumerate(elts)]
    return host, [None if h is None else (dev(fc, h[0]), dev(fc, h[1])) for h in host]


@pytest.mark.parametrize("log_n,L,K,dnum", [
    (10, 3, 2, 3), (11, 4, 2, 2),
    # the unfused ModDown (K > 4) and dnum > 4 (the u128 k_rot_sum)
    (10, 6, 5, 2), (10, 6, 2, 6)])
def test_rotate_sum_multi_matches_oracle(fc, log_n, L, K, dnum):
    """Three different ciphertexts, one of them unrotated, one conjugated: bit-exact vs
    pyoracle.rotate_sum_multi."""
    ctx = fc.Context(log_n, L=L, K=K, dnum=dnum)
    qs, ps, allm = ctx.moduli, ctx.all_moduli[L:], ctx.all_moduli
    n = 1 << log_n
    elts = [ctx.galois_elt(1), 1, 2 * n - 1]
    cts = [rand(qs, log_n, (2,), seed=10 + r) for r in range(len(elts))]
    hk, dk = keys_for(fc, elts, allm, log_n, dnum, 20)
    got = fc.to_host(ctx.rotate_sum_multi([dev(fc, c) for c in cts], elts, dk))
    want = pyoracle.rotate_sum_multi(cts, elts, hk, qs, ps, dnum, log_n)
    assert got.shape == (2, L, n)
    assert (got.astype(object) == want).all()


@pytest.mark.parametrize("log_n,L,K,dnum", [(10, 3, 2, 3), (10, 6, 5, 2), (10, 6, 2, 6)])
def test_linear_transform_matches_oracle(fc, log_n, L, K, dnum):
    """n1 = 3 baby steps (the unrotated one first), n2 = 2 giant steps (one unrotated), batch 2:
    bit-exact vs pyoracle.linear_transform for each ciphertext of the batch."""
    ctx = fc.Context(log_n, L=L, K=K, dnum=dnum)
    qs, ps, allm = ctx.moduli, ctx.all_moduli[L:], ctx.all_moduli
    baby = [1, ctx.galois_elt(1), ctx.galois_elt(2)]
    giant = [ctx.galois_elt(3), 1]
    ct = rand(qs, log_n, (2, 2), seed=3)
    hb, db = keys_for(fc, baby, allm, log_n, dnum, 40)
    hg, dg = keys_for(fc, giant, allm, log_n, dnum, 60)
    pts = [[rand(allm, log_n, seed=80 + 3 * g + b) for b in range(len(baby))]
           for g in range(len(giant))]
    got = fc.to_host(ctx.linear_transform(dev(fc, ct), baby, db, giant, dg,
                                          [[dev(fc, p) for p in row] for row in pts]))
    assert got.shape == (2, 2, L, 1 << log_n)
    for b in range(2):
        want = pyoracle.linear_transform(ct[b], baby, hb, giant, hg, pts, qs, ps, dnum, log_n)
        assert (got[b].astype(object) == want).all(), b


def test_linear_transform_wide_moduli_match_oracle(fc):
    """A chain with 62/63-bit moduli (the WIDE k_rot_sum, unfused ModUp / ModDown) and 50-61-bit
    ones: the transform and its giant-step sum bit-exact vs the oracle."""
    log_n = 11
    g = lambda bits, count=1, skip=0: [int(q) for q in fc.gen_moduli(log_n, count, bits=bits,  # noqa: E731
                                                                     skip=skip)]
    qs = g(63) + g(60) + g(55) + g(62)
    ps = g(61) + g(50)
    ctx = fc.Context(log_n, moduli=qs, special=ps, dnum=2)
    allm = qs + ps
    baby = [ctx.galois_elt(1), 1]
    giant = [1, ctx.galois_elt(-2)]
    ct = rand(qs, log_n, (2,), seed=17)
    hb, db = keys_for(fc, baby, allm, log_n, 2, 500)
    hg, dg = keys_for(fc, giant, allm, log_n, 2, 600)
    pts = [[rand(allm, log_n, seed=700 + 2 * gg + b) for b in range(2)] for gg in range(2)]
    got = fc.to_host(ctx.linear_transform(dev(fc, ct), baby, db, giant, dg,
                                          [[dev(fc, p) for p in row] for row in pts]))
    want = pyoracle.linear_transform(ct, baby, hb, giant, hg, pts, qs, ps, 2, log_n)
    assert (got.astype(object) == want).all()


def test_linear_transform_decrypts_with_real_keys(fc):
    """Real rotation keys and a real encryption: the transform decrypts to
    sum_g sigma_G(sum_b pt_{g,b} sigma_B(m)) up to noise (and equals the oracle bit for bit)."""
    log_n, L, K, dnum = 10, 3, 2, 3
    n = 1 << log_n
    ctx = fc.Context(log_n, L=L, K=K, dnum=dnum)
    qs, ps, allm = ctx.moduli, ctx.all_moduli[L:], ctx.all_moduli
    rng = random.Random(91)
    s = [rng.randrange(-1, 2) for _ in range(n)]
    m = [rng.randrange(-1000, 1000) for _ in range(n)]
    col = pyoracle._mods_col(qs)
    ntt = lambda v, mods: coracle.ntt_fwd(np.asarray(pyoracle._to_rns(v, mods), dtype=np.uint64),  # noqa: E731
                                          mods).astype(object)
    s_n = ntt(s, qs)
    a = np.stack([np.array([rng.randrange(q) for _ in range(n)], dtype=object) for q in qs])
    ct = np.stack([(-a * s_n + ntt([rng.randrange(-3, 4) for _ in range(n)], qs) + ntt(m, qs))
                   % col, a]).astype(np.uint64)
    baby = [1, ctx.galois_elt(1)]
    giant = [1, ctx.galois_elt(2)]
    key = lambda k: None if k == 1 else pyoracle.gen_rot_key(s, k, qs, ps, dnum, rng)  # noqa: E731
    hb = [key(k) for k in baby]
    hg = [key(k) for k in giant]
    as_u64 = lambda kk: None if kk is None else (kk[0].astype(np.uint64), kk[1].astype(np.uint64))  # noqa: E731
    hb, hg = [as_u64(k) for k in hb], [as_u64(k) for k in hg]
    dk = lambda ks: [None if k is None else (dev(fc, k[0]), dev(fc, k[1])) for k in ks]  # noqa: E731
    pt_int = [[[rng.randrange(-3, 4) for _ in range(n)] for _ in baby] for _ in giant]
    pts = [[ntt(p, allm).astype(np.uint64) for p in row] for row in pt_int]
    got = fc.to_host(ctx.linear_transform(dev(fc, ct), baby, dk(hb), giant, dk(hg),
                                          [[dev(fc, p) for p in row] for row in pts]))
    want = pyoracle.linear_transform(ct, baby, hb, giant, hg, pts, qs, ps, dnum, log_n)
    assert (got.astype(object) == want).all()
    decd = pyoracle.crt_centered(
        coracle.ntt_inv(((got[0].astype(object) + got[1].astype(object) * s_n) % col)
                        .astype(np.uint64), qs).astype(object), qs)

    def sigma(v, k):
        r = pyoracle.automorphism_coeff(np.array([[x % qs[0] for x in v]], dtype=object), k,
                                        [qs[0]])[0]
        return [int(x) - qs[0] if int(x) > qs[0] // 2 else int(x) for x in r]

    def negacyclic(x, y):
        out = [0] * n
        for i, u in enumerate(x):
            if u:
                for j, w in enumerate(y):
                    k = i + j
                    if k < n:
                        out[k] += u * w
                    else:
                        out[k - n] -= u * w
        return out

    expect = [0] * n
    for G, row in zip(giant, pt_int):
        inner = [0] * n
        for B, p in zip(baby, row):
            inner = [w + v for w, v in zip(inner, negacyclic(p, sigma(m, B)))]
        expect = [w + v for w, v in zip(expect, sigma(inner, G))]
    assert max(abs(int(x) - w) for x, w in zip(decd, expect)) < 1 << 24


def test_linear_transform_configs3_shape_is_its_composition(fc):
    """configs[3]'s context (N = 2^16, L = 16, K = 4, dnum = 4: the fused hoisted ModUp, the lz16
    k_rot_sum) with 3 ciphertexts, n1 = 4 baby steps and n2 = 3 giant steps: the transform equals,
    word for word, fhe_rotate_sum_multi over the giant steps of fhe_rotate_sum_hoisted outputs."""
    import torch

    log_n, L, K, dnum, B = 16, 16, 4, 4, 3
    ctx = fc.Context(log_n, L=L, K=K, dnum=dnum)
    allm = ctx.all_moduli
    baby = [1, ctx.galois_elt(1), ctx.galois_elt(2), ctx.galois_elt(3)]
    giant = [1, ctx.galois_elt(4), ctx.galois_elt(8)]
    ct = dev(fc, rand(ctx.moduli, log_n, (B, 2), seed=5))
    _, db = keys_for(fc, baby, allm, log_n, dnum, 100)
    _, dg = keys_for(fc, giant, allm, log_n, dnum, 200)
    pts = [[dev(fc, rand(allm, log_n, seed=300 + 4 * g + b)) for b in range(len(baby))]
           for g in range(len(giant))]
    got = ctx.linear_transform(ct, baby, db, giant, dg, pts)
    inner = [ctx.rotate_sum_hoisted(ct, baby, db, row) for row in pts]
    ref = ctx.rotate_sum_multi(inner, giant, dg)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    # one ciphertext on its own gives the same words (batch independence)
    one = ctx.linear_transform(ct[1:2], baby, db, giant, dg, pts)
    assert torch.equal(one[0], got[1])


def test_linear_transform_and_multi_errors(fc):
    import ctypes

    import torch

    from fhecore import _capi

    log_n, L, K = 10, 3, 2
    ctx = fc.Context(log_n, L=L, K=K, dnum=3)
    allm = ctx.all_moduli
    ct = dev(fc, rand(ctx.moduli, log_n, (2,), seed=1))
    kb = dev(fc, rand(allm, log_n, (3,), seed=2))
    ka = dev(fc, rand(allm, log_n, (3,), seed=3))
    pt = dev(fc, rand(allm, log_n, seed=4))
    k3 = ctx.galois_elt(3)
    with pytest.raises(ValueError):  # a rotated giant step without a key
        ctx.linear_transform(ct, [1], [None], [k3], [None], [[pt]])
    with pytest.raises(ValueError):  # pts not n2 x n1
        ctx.linear_transform(ct, [1, k3], [None, (kb, ka)], [1], [None], [[pt]])
    with pytest.raises(fc.FheError):  # even Galois element
        ctx.rotate_sum_multi([ct], [4], [(kb, ka)])
    lib = _capi.load()
    out = torch.empty(tuple(ct.shape), dtype=torch.int64, device="cuda")
    c_arr = (ctypes.c_void_p * 2)(ct.data_ptr(), out.data_ptr())
    g_arr = (ctypes.c_uint32 * 2)(1, 1)
    rc = lib.fhe_rotate_sum_multi(ctx.handle, out.data_ptr(), c_arr, g_arr, None, None, 2, 1,
                                  None, None)
    assert rc == -1 and b"overlap" in lib.fhe_last_error()
    b1 = (ctypes.c_uint32 * 1)(1)
    p_arr = (ctypes.c_void_p * 1)(pt.data_ptr())
    rc = lib.fhe_linear_transform(ctx.handle, out.data_ptr(), ct.data_ptr(), 1, 17, b1, None,
                                  None, b1, None, None, p_arr, 1, None, None)
    assert rc == -1 and b"n1 and n2" in lib.fhe_last_error()
    rc = lib.fhe_linear_transform(ctx.handle, ct.data_ptr() + 8, ct.data_ptr(), 1, 1, b1, None,
                                  None, b1, None, None, p_arr, 1, None, None)
    assert rc == -1 and b"overlap" in lib.fhe_last_error()
    k_arr = (ctypes.c_uint32 * 1)(k3)
    rc = lib.fhe_linear_transform(ctx.handle, out.data_ptr(), ct.data_ptr(), 1, 1, k_arr, None,
                                  None, b1, None, None, p_arr, 1, None, None)
    assert rc == -1 and b"without its key" in lib.fhe_last_error()
    # unrotated only: out = pt ct exactly
    got = fc.to_host(ctx.linear_transform(ct, [1], [None], [1], [None], [[pt]]))
    col = np.array(ctx.moduli, dtype=object).reshape(-1, 1)
    want = fc.to_host(ct).astype(object) * fc.to_host(pt)[:L].astype(object) % col
    assert (got.astype(object) == want).all()
