"""GPU parity for the double-hoisted rotation sum (fhe_rotate_sum_hoisted, csrc/galois.hip
launch_rotate_sum_hoisted): out = sum_r pt_r rot_r(ct) with one ModUp and one ModDown, the inner
loop of a baby-step / giant-step linear transform (CKKS bootstrapping's CoeffToSlot / SlotToCoeff,
the step after SURVEY.md §8(f) rows 1 and 4).

Not in the reference (parity unpinned by the reference); oracle/pyoracle.py rotate_sum_hoisted and
its C restatement (oracle/fhe_oracle.c, checked against each other and against real-key decryption
in tests/test_oracle.py) are the checkers, bit-exact."""
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


def _real_ct(qs, log_n, rng):
    """A real encryption of a small message under a ternary secret (NTT form)."""
    n = 1 << log_n
    s = [rng.randrange(-1, 2) for _ in range(n)]
    m = [rng.randrange(-1000, 1000) for _ in range(n)]
    col = pyoracle._mods_col(qs)
    ntt = lambda v: coracle.ntt_fwd(np.asarray(pyoracle._to_rns(v, qs), dtype=np.uint64),  # noqa: E731
                                    qs).astype(object)
    s_n = ntt(s)
    a = np.stack([np.array([rng.randrange(q) for _ in range(n)], dtype=object) for q in qs])
    ct = np.stack([(-a * s_n + ntt([rng.randrange(-3, 4) for _ in range(n)]) + ntt(m)) % col, a])
    return ct.astype(np.uint64), s, s_n, m


def _negacyclic_int(a, b):
    n = len(a)
    out = [0] * n
    for i, x in enumerate(a):
        if x:
            for j, y in enumerate(b):
                k = i + j
                if k < n:
                    out[k] += x * y
                else:
                    out[k - n] -= x * y
    return out


@pytest.mark.parametrize("log_n,L,K,dnum", [
    (10, 3, 2, 3), (11, 4, 2, 2),
    # the unfused ModDown (K > 4: k_moddown_finish adds both addends) and dnum > 4
    (10, 6, 5, 2), (10, 6, 2, 6)])
def test_rotate_sum_matches_oracle_and_decrypts(fc, log_n, L, K, dnum):
    """Bit-exact vs pyoracle.rotate_sum_hoisted with the unrotated term and three rotations
    (one of them the conjugation); decrypts to sum_r pt_r sigma_r(m) under real keys."""
    n = 1 << log_n
    ctx = fc.Context(log_n, L=L, K=K, dnum=dnum)
    qs, ps = ctx.moduli, ctx.all_moduli[L:]
    allm = ctx.all_moduli
    rng = random.Random(100 + log_n + dnum)
    ct, s, s_n, m = _real_ct(qs, log_n, rng)
    ks = [1, ctx.galois_elt(1), ctx.galois_elt(-2), 2 * n - 1]
    keys = [None if k == 1 else pyoracle.gen_rot_key(s, k, qs, ps, dnum, rng) for k in ks]
    keys = [None if kk is None else (kk[0].astype(np.uint64), kk[1].astype(np.uint64))
            for kk in keys]
    pt_int = [[rng.randrange(-3, 4) for _ in range(n)] for _ in ks]
    pts = [coracle.ntt_fwd(np.asarray(pyoracle._to_rns(p, allm), dtype=np.uint64), allm)
           for p in pt_int]
    d = lambda v: fc.to_device(np.ascontiguousarray(v))  # noqa: E731
    got = fc.to_host(ctx.rotate_sum_hoisted(
        d(ct), ks, [None if kk is None else (d(kk[0]), d(kk[1])) for kk in keys],
        [d(p) for p in pts]))
    want = pyoracle.rotate_sum_hoisted(ct, ks, keys, pts, qs, ps, dnum, log_n)
    assert got.shape == (2, L, n)
    assert (got.astype(object) == want).all()
    col = pyoracle._mods_col(qs)
    dec = pyoracle.crt_centered(
        coracle.ntt_inv(((got[0].astype(object) + got[1].astype(object) * s_n) % col)
                        .astype(np.uint64), qs).astype(object), qs)
    expect = [0] * n
    for k, p in zip(ks, pt_int):
        mk = pyoracle.automorphism_coeff(np.array([[v % qs[0] for v in m]], dtype=object), k,
                                         [qs[0]])[0]
        mk = [int(v) - qs[0] if int(v) > qs[0] // 2 else int(v) for v in mk]
        expect = [w + v for w, v in zip(expect, _negacyclic_int(p, mk))]
    assert max(abs(int(x) - w) for x, w in zip(dec, expect)) < 1 << 24


def test_rotate_sum_wide_moduli_match_oracle(fc):
    """A chain with 62/63-bit moduli (the WIDE kernel: every product reduced) and 50-61-bit ones."""
    log_n = 11
    g = lambda bits, count=1, skip=0: [int(q) for q in fc.gen_moduli(log_n, count, bits=bits,  # noqa: E731
                                                                     skip=skip)]
    qs = g(63) + g(60) + g(55) + g(62)
    ps = g(61) + g(50)
    ctx = fc.Context(log_n, moduli=qs, special=ps, dnum=2)
    allm = qs + ps
    ct = rand(qs, log_n, (2,), seed=7)
    ks = [ctx.galois_elt(3), 1, ctx.galois_elt(-5)]
    keys = [(rand(allm, log_n, (2,), seed=8 + r), rand(allm, log_n, (2,), seed=18 + r))
            for r in range(len(ks))]
    keys[1] = None
    pts = [rand(allm, log_n, seed=30 + r) for r in range(len(ks))]
    d = lambda v: fc.to_device(np.ascontiguousarray(v))  # noqa: E731
    got = fc.to_host(ctx.rotate_sum_hoisted(
        d(ct), ks, [None if kk is None else (d(kk[0]), d(kk[1])) for kk in keys],
        [d(p) for p in pts]))
    want = pyoracle.rotate_sum_hoisted(ct, ks, keys, pts, qs, ps, 2, log_n)
    assert (got.astype(object) == want).all()


def test_rotate_sum_configs3_shape_matches_c_oracle(fc):
    """configs[3]'s context (N = 2^16, L = 16, K = 4, dnum = 4, the fused ModDown finish) with 5
    ciphertexts (a partial group of the kernel's 4-ciphertext blocks) and 4 terms: ciphertexts 0
    and 4 against the C restatement word for word, and every ciphertext of the batch equal to
    its own single-ciphertext call."""
    import torch

    log_n, L, K, dnum, B = 16, 16, 4, 4, 5
    ctx = fc.Context(log_n, L=L, K=K, dnum=dnum)
    qs, ps = ctx.moduli, ctx.all_moduli[L:]
    allm = ctx.all_moduli
    ct = rand(qs, log_n, (B, 2), seed=41)
    ks = [ctx.galois_elt(1), ctx.galois_elt(2), 1, ctx.galois_elt(-4)]
    kb = rand(allm, log_n, (len(ks), dnum), seed=42)
    ka = rand(allm, log_n, (len(ks), dnum), seed=43)
    pts = rand(allm, log_n, (len(ks),), seed=44)
    d = lambda v: fc.to_device(np.ascontiguousarray(v))  # noqa: E731
    dkeys = [None if k == 1 else (d(kb[r]), d(ka[r])) for r, k in enumerate(ks)]
    dpts = [d(pts[r]) for r in range(len(ks))]
    dct = d(ct)
    got = fc.to_host(ctx.rotate_sum_hoisted(dct, ks, dkeys, dpts))
    assert got.shape == (B, 2, L, 1 << log_n)
    for b in (0, 4):
        want = coracle.rotate_sum_hoisted(ct[b], ks, kb, ka, pts, qs, ps, dnum)
        assert (got[b] == want).all(), b
    for b in range(B):
        one = fc.to_host(ctx.rotate_sum_hoisted(dct[b:b + 1], ks, dkeys, dpts))
        assert (one[0] == got[b]).all(), b
    torch.cuda.synchronize()


def test_rotate_sum_unrotated_only_is_the_plaintext_product(fc):
    """Only the unrotated term: no ModUp, A = 0, so out = pt ct exactly (ModDown(0) = 0)."""
    log_n, L, K = 12, 4, 2
    ctx = fc.Context(log_n, L=L, K=K, dnum=2)
    qs, allm = ctx.moduli, ctx.all_moduli
    ct = rand(qs, log_n, (3, 2), seed=5)
    pt = rand(allm, log_n, seed=6)
    d = lambda v: fc.to_device(np.ascontiguousarray(v))  # noqa: E731
    got = fc.to_host(ctx.rotate_sum_hoisted(d(ct), [1], [None], [d(pt)]))
    col = np.array(qs, dtype=object).reshape(-1, 1)
    want = ct.astype(object) * pt[:L].astype(object) % col
    assert (got.astype(object) == want).all()


def test_rotate_sum_errors(fc):
    import ctypes

    import torch

    from fhecore import _capi

    log_n, L, K = 10, 3, 2
    ctx = fc.Context(log_n, L=L, K=K, dnum=3)
    allm = ctx.all_moduli
    ct = fc.to_device(rand(ctx.moduli, log_n, (2,), seed=1))
    kb = fc.to_device(rand(allm, log_n, (3,), seed=2))
    ka = fc.to_device(rand(allm, log_n, (3,), seed=3))
    pt = fc.to_device(rand(allm, log_n, seed=4))
    k3 = ctx.galois_elt(3)
    with pytest.raises(ValueError):  # a rotated term without a key
        ctx.rotate_sum_hoisted(ct, [k3], [None], [pt])
    with pytest.raises(ValueError):  # one plaintext per term
        ctx.rotate_sum_hoisted(ct, [k3, 1], [(kb, ka), None], [pt])
    with pytest.raises(fc.FheError):  # even Galois element
        ctx.rotate_sum_hoisted(ct, [4], [(kb, ka)], [pt])
    with pytest.raises(fc.FheError):  # 17 terms
        ctx.rotate_sum_hoisted(ct, [k3] * 17, [(kb, ka)] * 17, [pt] * 17)
    lib = _capi.load()
    out = torch.empty(tuple(ct.shape), dtype=torch.int64, device="cuda")
    g_arr = (ctypes.c_uint32 * 2)(k3, 1)
    b_arr = (ctypes.c_void_p * 2)(None, None)
    a_arr = (ctypes.c_void_p * 2)(ka.data_ptr(), None)
    p_arr = (ctypes.c_void_p * 2)(pt.data_ptr(), pt.data_ptr())
    rc = lib.fhe_rotate_sum_hoisted(ctx.handle, out.data_ptr(), ct.data_ptr(), g_arr, b_arr, a_arr,
                                    p_arr, 2, 1, None, None)
    assert rc == -1 and b"null plaintext or key pointer for term 0" in lib.fhe_last_error()
    # out overlapping in
    b_arr = (ctypes.c_void_p * 2)(kb.data_ptr(), None)
    rc = lib.fhe_rotate_sum_hoisted(ctx.handle, ct.data_ptr() + 8, ct.data_ptr(), g_arr, b_arr,
                                    a_arr, p_arr, 2, 1, None, None)
    assert rc == -1 and b"overlap" in lib.fhe_last_error()
    # count 0
    rc = lib.fhe_rotate_sum_hoisted(ctx.handle, out.data_ptr(), ct.data_ptr(), g_arr, b_arr,
                                    a_arr, p_arr, 0, 1, None, None)
    assert rc == -1
