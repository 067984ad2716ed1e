"""GPU parity across modulus widths: north_star's "60-63-bit primes" and the narrower primes CKKS
chains mix in (scaling primes of 40-55 bits).

libfhecore picks its butterfly arithmetic per context (csrc/ntt.hip, HD template argument):
  * every q < 2^60                      lazy forward up to 16q (HD = 16); the final reduction takes
                                        the one-step top-bits estimate only for q in
                                        [2^60 - 2^56, 2^60) and the halving subtractions otherwise;
  * some q in [2^60, 2^61)              lazy up to 8q (HD = 8);
  * some q in [2^61, 2^63) ("wide")     exact butterflies with values below 2q (HD = 2), and the
                                        unfused key-switch kernels (rns.hip) with per-product
                                        reductions (reduce128_wide).
Each chain below runs NTT, HomMult, vec ops, base conversion, key-switch, rescale and the
keygen/encrypt/decrypt path through the C ABI, bit-exact against the oracle.  The reference accepts
any MOD for vec_* (/root/reference/arithmetic.py:3-13); its NTT is the identity
(arithmetic.py:15-19), so the NTT-family rows are pinned by the oracle's math."""
import numpy as np
import pytest

import coracle
import pyoracle

pytestmark = pytest.mark.gpu

LOG_N, L, K, DNUM = 12, 4, 2, 2


@pytest.fixture(scope="module")
def fc():
    import fhecore

    return fhecore


def rand(mods, log_n, lead=(), seed=0):
    rng = np.random.default_rng(seed)
    n = 1 << log_n
    return np.stack([rng.integers(0, q, size=lead + (n,), dtype=np.uint64) for q in mods],
                    axis=len(lead))


def _chain(fc, name):
    """(Q moduli, P moduli) for a named width class, all q = 1 mod 2N at N = 2^12."""
    g = lambda bits, count, skip=0: fc.gen_moduli(LOG_N, count, bits=bits, skip=skip)  # noqa: E731
    if name.startswith("b"):
        m = g(int(name[1:]), L + K)
        return m[:L], m[L:]
    if name == "mixed-wide":  # 63, 60, 55, 62-bit Q; 61, 50-bit P
        return [g(63, 1)[0], g(60, 1)[0], g(55, 1)[0], g(62, 1)[0]], [g(61, 1)[0], g(50, 1)[0]]
    if name == "mixed-narrow":  # below 2^60 with and without the top-bits final reduction
        return [g(60, 1)[0], g(50, 1)[0], g(59, 1)[0], g(55, 1)[0]], [g(60, 1, 1)[0], g(45, 1)[0]]
    if name == "far":  # below 2^60 but not within 1/16 below a power of two: the 8q kernels
        fr = [0.70, 0.80, 0.90, 0.60, 0.75, 0.85]
        m = [_prime_below(int(f * (1 << b))) for f, b in zip(fr, [59, 56, 50, 58, 57, 52])]
        return m[:L], m[L:]
    raise ValueError(name)


def _prime_below(bound):
    """Largest prime q < bound with q = 1 mod 2N (N = 2^LOG_N)."""
    step = 2 << LOG_N
    q = (bound - 1) // step * step + 1
    while not pyoracle.is_prime(q):
        q -= step
    return q


# b33 / b34: the smallest lz16 moduli (top_bits works on the 32-bit halves, shift s - 32 = 1, 2);
# b32: below 2^32, so the context takes the 8q kernels
CHAINS = ["b32", "b33", "b34", "b50", "b55", "b60", "b61", "b62", "b63", "mixed-wide",
          "mixed-narrow", "far"]
_CTX = {}


def ctx_for(fc, name):
    if name not in _CTX:
        qs, ps = _chain(fc, name)
        _CTX[name] = fc.Context(LOG_N, moduli=qs, special=ps, dnum=DNUM)
    return _CTX[name]


@pytest.mark.parametrize("name,lz16", [("b32", False), ("b33", True), ("b34", True), ("b60", True),
                                       ("far", False)])
def test_chain_width_class(fc, name, lz16):
    """The chains above reach the kernel family they are meant to (fhe_ctx::lz16: every modulus
    in (2^32, 2^60) within 1/16 below a power of two)."""
    qs, ps = _chain(fc, name)
    in_class = all((1 << 32) < q < (1 << 60) and q >= (1 << q.bit_length()) - (1 << (q.bit_length() - 4))
                   for q in qs + ps)
    assert in_class == lz16


@pytest.mark.parametrize("name", CHAINS)
def test_chain_ntt_and_hommult(fc, name):
    ctx = ctx_for(fc, name)
    qs = ctx.moduli
    top = max(ctx.all_moduli).bit_length()
    assert top == {"b32": 32, "b33": 33, "b34": 34, "b50": 50, "b55": 55, "b60": 60, "b61": 61,
                   "b62": 62, "b63": 63,
                   "mixed-wide": 63, "mixed-narrow": 60, "far": 59}[name]
    x = rand(qs, LOG_N, (3,), seed=1)
    t = fc.to_device(x)
    ctx.ntt_(t)
    fwd = coracle.ntt_fwd(x, qs)
    assert (fc.to_host(t) == fwd).all()
    ctx.intt_(t)
    assert (fc.to_host(t) == x).all()
    # inverse of an arbitrary (non-NTT-image) input, and edge residues 0 / q - 1
    y = rand(qs, LOG_N, (2,), seed=2)
    y[0, :, :64] = 0
    y[1, :, :64] = np.array(qs, dtype=np.uint64)[:, None] - 1
    u = fc.to_device(y)
    ctx.intt_(u)
    assert (fc.to_host(u) == coracle.ntt_inv(y, qs)).all()
    a = rand(qs, LOG_N, (2, 2), seed=3)
    b = rand(qs, LOG_N, (2, 2), seed=4)
    a[0, :, :, :32] = np.array(qs, dtype=np.uint64)[:, None] - 1
    b[0, :, :, :32] = np.array(qs, dtype=np.uint64)[:, None] - 1
    d = fc.to_host(ctx.hommult(fc.to_device(a), fc.to_device(b)))
    for i in range(2):
        assert (d[i] == coracle.hommult(a[i], b[i], qs)).all(), i


@pytest.mark.parametrize("name", CHAINS)
def test_chain_vec_baseconv_keyswitch(fc, name):
    ctx = ctx_for(fc, name)
    qs, allm = ctx.moduli, ctx.all_moduli
    a = rand(qs, LOG_N, (2,), seed=5)
    b = rand(qs, LOG_N, (2,), seed=6)
    rows = np.array(qs * 2, dtype=np.uint64)
    for op in ("add", "sub", "mul"):
        got = fc.to_host(ctx.vec(op, fc.to_device(a), fc.to_device(b)))
        want = coracle.vec_op(op, a.reshape(-1, 1 << LOG_N), b.reshape(-1, 1 << LOG_N), rows)
        assert (got.reshape(-1, 1 << LOG_N) == want).all(), op
    x = rand(allm[:L], LOG_N, seed=7)
    out = fc.to_host(ctx.baseconv(fc.to_device(x), 0, L, K))
    assert (out == coracle.baseconv(x, allm[:L], allm[L:])).all()
    d2 = rand(qs, LOG_N, (2,), seed=8)
    eb = rand(allm, LOG_N, (DNUM,), seed=9)
    ea = rand(allm, LOG_N, (DNUM,), seed=10)
    ks0, ks1 = ctx.keyswitch(fc.to_device(d2), fc.to_device(eb), fc.to_device(ea))
    h0, h1 = fc.to_host(ks0), fc.to_host(ks1)
    for i in range(2):
        r0, r1 = coracle.keyswitch(d2[i], eb, ea, qs, ctx.special, DNUM)
        assert (h0[i] == r0).all() and (h1[i] == r1).all(), i


@pytest.mark.parametrize("name", ["b55", "b62", "b63", "mixed-wide", "far"])
def test_chain_rescale_and_keys(fc, name):
    ctx = ctx_for(fc, name)
    qs, ps = ctx.moduli, ctx.special
    x = rand(qs, LOG_N, (1,), seed=11)
    got = fc.to_host(ctx.rescale(fc.to_device(x), ntt_form=False))
    assert (got[0].astype(object) == pyoracle.rescale_coeff(x[0].astype(object), qs)).all()
    got = fc.to_host(ctx.rescale(fc.to_device(x), ntt_form=True))
    c = coracle.ntt_inv(x[0][None], qs)[0]
    want = coracle.ntt_fwd(np.asarray(pyoracle.rescale_coeff(c.astype(object), qs),
                                      dtype=np.uint64)[None], qs[:-1])[0]
    assert (got[0] == want).all()
    # keys, encryption and decryption: Philox samples and every product bit-exact
    sk = ctx.keygen_secret(21)
    sk_o = pyoracle.keygen_secret(21, ctx.all_moduli, LOG_N)
    assert (fc.to_host(sk).astype(object) == sk_o).all()
    pk = ctx.keygen_public(sk, 22)
    pk_o = pyoracle.keygen_public(22, sk_o, qs, LOG_N)
    assert (fc.to_host(pk).astype(object) == pk_o).all()
    kb, ka = ctx.keygen_relin(sk, 23)
    col = pyoracle._mods_col(ctx.all_moduli)
    key_o = pyoracle.keygen_switch(23, sk_o, sk_o * sk_o % col, qs, ps, DNUM, LOG_N)
    assert (fc.to_host(kb).astype(object) == key_o[0]).all()
    assert (fc.to_host(ka).astype(object) == key_o[1]).all()
    pt = rand(qs, LOG_N, seed=12)
    ct = ctx.encrypt(fc.to_device(pt), pk, 24)
    ct_o = pyoracle.encrypt(24, pt.astype(object), pk_o, qs, LOG_N)
    assert (fc.to_host(ct).astype(object) == ct_o).all()
    dec = fc.to_host(ctx.decrypt(ct, sk)).astype(object)
    assert (dec == pyoracle.decrypt(ct_o, sk_o, qs)).all()


@pytest.mark.parametrize("bits", [62, 63])
def test_wide_hommult_at_config3_size(fc, bits):
    """BASELINE configs[2]'s shape (N = 2^16, 8 limbs) on a 62- / 63-bit chain."""
    mods = fc.gen_moduli(16, 8, bits=bits)
    ctx = fc.Context(16, moduli=mods)
    a = rand(mods, 16, (1, 2), seed=bits)
    b = rand(mods, 16, (1, 2), seed=bits + 1)
    d = fc.to_host(ctx.hommult(fc.to_device(a), fc.to_device(b)))
    assert (d[0] == coracle.hommult(a[0], b[0], mods)).all()
    x = rand(mods, 16, (2,), seed=bits + 2)
    t = fc.to_device(x)
    ctx.ntt_(t)
    assert (fc.to_host(t) == coracle.ntt_fwd(x, mods)).all()


@pytest.mark.parametrize("bits", [62, 63])
def test_reference_shim_ntt_wide_mod(fc, bits):
    """arithmetic.NTT / iNTT with an explicit 62- or 63-bit MOD (the reference takes any MOD)."""
    import arithmetic

    q = fc.gen_moduli(10, 1, bits=bits)[0]
    x = rand([q], 10, seed=bits)[0]
    y = arithmetic.NTT(x, MOD=q)
    assert (y == coracle.ntt_fwd(x[None, None], [q])[0, 0]).all()
    assert (arithmetic.iNTT(y, MOD=q) == x).all()
    naive = pyoracle.ntt_naive([int(v) for v in x], q)
    assert [int(v) for v in y] == list(naive)


@pytest.mark.parametrize("name", CHAINS)
def test_chain_rotate_hoisted(fc, name):
    """Hoisted rotations on every width class: the wide contexts take the exact unfused kernels
    end to end, the others the gathered inner product with the fused ModDown."""
    ctx = ctx_for(fc, name)
    qs, allm = ctx.moduli, ctx.all_moduli
    ct = rand(qs, LOG_N, (2, 2), seed=11)
    ct[0, 0, :, :16] = np.array(qs, dtype=np.uint64)[:, None] - 1
    keys = [(rand(allm, LOG_N, (DNUM,), seed=12 + 2 * r), rand(allm, LOG_N, (DNUM,), seed=13 + 2 * r))
            for r in range(2)]
    ks = [ctx.galois_elt(1), (2 << LOG_N) - 1]
    got = fc.to_host(ctx.rotate_hoisted(fc.to_device(ct), ks,
                                        [(fc.to_device(b), fc.to_device(a)) for b, a in keys]))
    for i in range(2):
        want = pyoracle.rotate_hoisted(ct[i], ks, keys, qs, ctx.special, DNUM, LOG_N)
        assert (got[:, i].astype(object) == want).all(), i
