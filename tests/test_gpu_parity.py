"""GPU parity tests: libfhecore (hand-written gfx950 kernels, called through the C ABI via ctypes)
against the exact CPU oracle and the reference-derived golden fixtures.  Bit-exact everywhere:
all outputs are canonical residues.  Full BASELINE sizes are covered by direct oracle comparison
(the C restatement finishes them in seconds) plus size-independent properties."""
import os

import numpy as np
import pytest

import coracle
import pyoracle

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def fc():
    import fhecore

    return fhecore


def rand(mods, log_n, lead=(), seed=0):
    rng = np.random.default_rng(seed)
    n = 1 << log_n
    return np.stack([rng.integers(0, q, size=lead + (n,), dtype=np.uint64) for q in mods],
                    axis=len(lead))


_CTX = {}


def ctx_for(fc, log_n, L, K=0, dnum=1):
    key = (log_n, L, K, dnum)
    if key not in _CTX:
        _CTX[key] = fc.Context(log_n, L=L, K=K, dnum=dnum)
    return _CTX[key]


# ------------------------------------------------------------------------------------ NTT

@pytest.mark.parametrize("log_n,L,polys", [(10, 3, 2), (11, 2, 1), (12, 1, 3), (13, 2, 1),
                                           (14, 4, 2), (15, 2, 1), (16, 8, 2), (17, 4, 1),
                                           # many limbs (XCD placement walks limbs in runs),
                                           # incl. the BASELINE configs[4] shape (N=2^17, 32 limbs)
                                           (13, 24, 3), (14, 12, 2), (16, 16, 1), (17, 32, 1)])
def test_ntt_matches_oracle(fc, log_n, L, polys):
    ctx = ctx_for(fc, log_n, L)
    x = rand(ctx.moduli, log_n, (polys,), seed=log_n)
    t = fc.to_device(x)
    ctx.ntt_(t)
    got = fc.to_host(t)
    assert (got == coracle.ntt_fwd(x, ctx.moduli)).all()
    ctx.intt_(t)
    assert (fc.to_host(t) == x).all()


def test_ntt_golden_naive_fixture(fc):
    d = np.load(os.path.join(GOLDEN, "ntt_N4096_L1.npz"))
    ctx = fc.Context(12, moduli=[int(q) for q in d["moduli"]])
    assert ctx.psi[0] == int(d["psi"])
    t = fc.to_device(d["x"])
    ctx.ntt_(t)
    assert (fc.to_host(t) == d["y"]).all()
    ctx.intt_(t)
    assert (fc.to_host(t) == d["x"]).all()


def test_ntt_inverse_of_arbitrary_input(fc):
    """iNTT is applied to data that was never a forward output (bit-reversed inputs)."""
    ctx = ctx_for(fc, 14, 4)
    y = rand(ctx.moduli, 14, (2,), seed=3)
    t = fc.to_device(y)
    ctx.intt_(t)
    assert (fc.to_host(t) == coracle.ntt_inv(y, ctx.moduli)).all()


def test_ntt_edge_values_and_limb_window(fc):
    ctx = ctx_for(fc, 16, 8)
    qs = ctx.moduli
    n = 1 << 16
    x = np.zeros((3, 4, n), dtype=np.uint64)
    for li in range(4):
        q = qs[2 + li]
        x[0, li] = q - 1                       # all max
        x[1, li, ::2] = q - 1                  # alternating
        x[2, li, n - 1] = 1                    # single monomial X^(N-1)
    t = fc.to_device(x)
    ctx.ntt_(t, limb0=2)
    got = fc.to_host(t)
    assert (got == coracle.ntt_fwd(x, qs[2:6])).all()
    ctx.intt_(t, limb0=2)
    assert (fc.to_host(t) == x).all()


def test_ntt_linearity_full_size(fc):
    """NTT(a + b) = NTT(a) + NTT(b) at N = 2^17 (size-independent property)."""
    ctx = ctx_for(fc, 17, 4)
    a = fc.to_device(rand(ctx.moduli, 17, (1,), seed=1))
    b = fc.to_device(rand(ctx.moduli, 17, (1,), seed=2))
    s = ctx.vec("add", a, b)
    ctx.ntt_(a)
    ctx.ntt_(b)
    ctx.ntt_(s)
    assert (fc.to_host(ctx.vec("add", a, b)) == fc.to_host(s)).all()


# ----------------------------------------------------------------------------- vec ops

@pytest.mark.parametrize("op", ["add", "sub", "mul"])
def test_vec_ctx_golden(fc, op):
    d = np.load(os.path.join(GOLDEN, "vec_N16384_L4.npz"))
    ctx = fc.Context(14, moduli=[int(q) for q in d["moduli"]])
    out = ctx.vec(op, fc.to_device(d["a"]), fc.to_device(d["b"]))
    assert (fc.to_host(out) == d[op]).all()


@pytest.mark.parametrize("fx", ["vec_N4096_L1.npz", "vec_N16384_L4.npz"])
@pytest.mark.parametrize("op", ["add", "sub", "mul"])
def test_reference_shim_golden(fc, fx, op):
    import arithmetic

    d = np.load(os.path.join(GOLDEN, fx))
    col = np.array([int(q) for q in d["moduli"]], dtype=np.uint64).reshape(-1, 1)
    fn = getattr(arithmetic, "vec_" + op)
    got = fn(d["a"], d["b"], col)
    assert got.dtype == np.uint64 and (got == d[op]).all()
    got_obj = fn(d["a"].astype(object), d["b"].astype(object), col.astype(object))
    assert got_obj.dtype == object and (got_obj.astype(np.uint64) == d[op]).all()


def test_reference_shim_generic_moduli(fc):
    import arithmetic

    rng = np.random.default_rng(9)
    a = rng.integers(0, 2**64 - 1, (3, 500), dtype=np.uint64, endpoint=True)
    b = rng.integers(0, 2**64 - 1, (3, 500), dtype=np.uint64, endpoint=True)
    for mod in [7, 2**31 - 1, 2**61 - 1, 2**63 + 29, 2**64 - 59,
                np.array([[3], [2**40 + 15], [2**62 + 135]], dtype=object),
                np.arange(2, 502, dtype=np.uint64)]:
        for op in ("add", "sub", "mul"):
            got = getattr(arithmetic, "vec_" + op)(a, b, mod)
            want = getattr(pyoracle, "vec_" + op)(a, b, np.asarray(mod, dtype=object))
            assert (got.astype(object) == want).all(), (op, mod)
    # signed operands (Python floor-mod semantics)
    x = rng.integers(-2**62, 2**62, (2, 64), dtype=np.int64)
    y = rng.integers(-2**62, 2**62, (2, 64), dtype=np.int64)
    for op in ("add", "sub", "mul"):
        got = getattr(arithmetic, "vec_" + op)(x, y, 1000003)
        want = getattr(pyoracle, "vec_" + op)(x, y, 1000003)
        assert (got.astype(object) == want).all(), op
    with pytest.raises(AssertionError):
        arithmetic.vec_add(a, b[:, :10], 7)


def test_reference_shim_ntt_and_poly_add(fc):
    import arithmetic
    import polynomial

    d = np.load(os.path.join(GOLDEN, "ntt_N4096_L1.npz"))
    y = arithmetic.NTT(d["x"])  # default modulus chain = the fixture's modulus
    assert (y == d["y"]).all()
    assert (arithmetic.iNTT(y) == d["x"]).all()
    y1 = arithmetic.NTT(d["x"][0], MOD=int(d["moduli"][0]))
    assert (y1 == d["y"][0]).all()
    v = np.load(os.path.join(GOLDEN, "vec_N16384_L4.npz"))
    col = v["moduli"].reshape(-1, 1)
    r = polynomial.poly_add((v["a"], v["b"]), (v["b"], v["a"]), col)
    assert isinstance(r, tuple) and (r[0] == v["add"]).all() and (r[1] == v["add"]).all()


def test_reference_import_line_unchanged(fc):
    """The reference's caller line, verbatim: importlib.import_module(" polynomial") with
    gpu-fhe_amd/ on sys.path (/root/reference/ polynomial.py:1-5) gets this package's module, whose
    poly_add runs on the HIP path and matches the reference-made vec_N4096_L1 fixture."""
    import importlib

    import fhecore

    poly = importlib.import_module(" polynomial")
    assert os.path.dirname(os.path.abspath(poly.__file__)) == os.path.dirname(
        os.path.abspath(fhecore.__path__[0]))
    v = np.load(os.path.join(GOLDEN, "vec_N4096_L1.npz"))
    col = v["moduli"].reshape(-1, 1)
    r = poly.poly_add((v["a"], v["b"]), (v["b"], v["a"]), col)
    assert isinstance(r, tuple) and len(r) == 2
    assert (r[0] == v["add"]).all() and (r[1] == v["add"]).all()
    assert bool(v["ref_poly_add_returns_none"])  # the reference's own return (divergence)


# ------------------------------------------------------------------------------- HomMult

@pytest.mark.parametrize("fx", ["hommult_N4096_L2.npz", "hommult_N2048_L8_chain16.npz"])
def test_hommult_reference_composed_golden(fc, fx):
    """HomMult vs the reference's own arithmetic: (d0, d1, d2) in the fixture are schoolbook
    negacyclic products built only from /root/reference/arithmetic.py:3-13 (vec_mul / vec_add /
    vec_sub on exact object arrays; tests/golden/make_golden.py).  The N = 2048 case runs on the
    8-limb BASELINE configs[2] modulus chain."""
    d = np.load(os.path.join(GOLDEN, fx))
    log_n = int(d["log_n"])
    ctx = fc.Context(log_n, moduli=[int(q) for q in d["moduli"]])
    a = np.stack([d["a"], d["b"][::-1]])  # two ciphertext pairs: (a, b) and (a, b swapped)
    b = np.stack([d["b"], d["a"][::-1]])
    got = fc.to_host(ctx.hommult(fc.to_device(a), fc.to_device(b)))
    assert (got[0] == d["d"]).all()
    # second pair: (b1, b0) x (a1, a0) -> d0' = b1 a1 = d2, d1' = b1 a0 + b0 a1 = d1, d2' = d0
    assert (got[1] == d["d"][::-1]).all()


def test_hommult_config3_full_size_reference_sampled(fc):
    """BASELINE configs[2] at its full size -- N = 2^16, the 8-limb chain, the bench's batch of 64
    through the bench's kernels -- against the reference's own arithmetic: 48 output coefficients
    of d0, d1, d2 of one ciphertext pair (at batch index 37), each computed by
    tests/golden/make_golden.py with only /root/reference/arithmetic.py:3-13 (one vec_mul of a
    against b's signed reversal, a vec_add halving tree).  The pair is regenerated from the
    fixture's seed and checked by sha256 before the comparison; the other 63 pairs are random.
    The whole batch is also checked against the C oracle on two more pairs."""
    import hashlib
    import sys

    sys.path.insert(0, GOLDEN)
    from make_golden import sampled_inputs  # data generation only (seeded numpy)

    d = np.load(os.path.join(GOLDEN, "hommult_sampled_N65536_L8.npz"))
    log_n, qs = int(d["log_n"]), [int(q) for q in d["moduli"]]
    n = 1 << log_n
    pa, pb = sampled_inputs(qs, n, int(d["seed"]))
    assert hashlib.sha256(pa.tobytes() + pb.tobytes()).hexdigest() == str(d["inputs_sha256"])
    ctx = fc.Context(log_n, moduli=qs)
    B, at = 64, 37
    a = rand(qs, log_n, (B, 2), seed=98)
    b = rand(qs, log_n, (B, 2), seed=99)
    a[at], b[at] = pa, pb
    got = fc.to_host(ctx.hommult(fc.to_device(a), fc.to_device(b)))
    assert (got[at][:, :, d["index"]].transpose(2, 0, 1) == d["d"]).all()
    for i in (0, B - 1):
        assert (got[i] == coracle.hommult(a[i], b[i], qs)).all()


@pytest.mark.parametrize("op", ["add", "sub", "mul"])
def test_vec_config3_chain_golden(fc, op):
    """vec_* on the configs[2] chain: the first 4096 coefficients of each N = 2^16 limb are the
    reference's golden vectors, through the context kernel (k_vec_ctx) and the reference-shaped
    shim (fhe_vec_op_mod)."""
    import arithmetic

    d = np.load(os.path.join(GOLDEN, "vec_N65536_L8.npz"))
    ctx = ctx_for(fc, 16, 8)
    assert [int(q) for q in d["moduli"]] == ctx.moduli
    a = rand(ctx.moduli, 16, (1,), seed=31)
    b = rand(ctx.moduli, 16, (1,), seed=32)
    a[0, :, :4096], b[0, :, :4096] = d["a"], d["b"]
    got = fc.to_host(ctx.vec(op, fc.to_device(a), fc.to_device(b)))
    assert (got[0, :, :4096] == d[op]).all()
    assert (got == coracle.vec_op(op, a, b, ctx.moduli)).all()
    shim = getattr(arithmetic, "vec_" + op)(d["a"], d["b"], d["moduli"].reshape(-1, 1))
    assert (shim == d[op]).all()


def test_hommult_config3_matches_oracle(fc):
    ctx = ctx_for(fc, 16, 8)
    a = rand(ctx.moduli, 16, (2, 2), seed=21)
    b = rand(ctx.moduli, 16, (2, 2), seed=22)
    d = fc.to_host(ctx.hommult(fc.to_device(a), fc.to_device(b)))
    assert (d == coracle.hommult(a, b, ctx.moduli)).all()


@pytest.mark.parametrize("log_n,L,B", [(12, 16, 3), (13, 24, 2)])
def test_hommult_many_limbs_matches_oracle(fc, log_n, L, B):
    """More limbs than XCDs: the fused row kernel walks each XCD's limbs one after another."""
    ctx = ctx_for(fc, log_n, L)
    a = rand(ctx.moduli, log_n, (B, 2), seed=23)
    b = rand(ctx.moduli, log_n, (B, 2), seed=24)
    d = fc.to_host(ctx.hommult(fc.to_device(a), fc.to_device(b)))
    assert (d == coracle.hommult(a, b, ctx.moduli)).all()


@pytest.mark.parametrize("log_n", [10, 11, 12, 13, 14, 15, 16, 17])
def test_row_layouts_every_log_n(fc, log_n):
    """Every transform size's row geometry (rows of 2^5 .. 2^9 points, the lane-major twiddle
    segments of context.cpp lane_major_rows, the linear row stores): HomMult and the fused
    key-switch (k_ks_row_inner, k_moddown_row) against the C oracle."""
    ctx = ctx_for(fc, log_n, 4, K=2, dnum=2)
    a = rand(ctx.moduli, log_n, (2, 2), seed=80 + log_n)
    b = rand(ctx.moduli, log_n, (2, 2), seed=90 + log_n)
    d = fc.to_host(ctx.hommult(fc.to_device(a), fc.to_device(b)))
    assert (d == coracle.hommult(a, b, ctx.moduli)).all()
    allm = ctx.all_moduli
    d2 = rand(ctx.moduli, log_n, seed=100 + log_n)
    eb = rand(allm, log_n, (2,), seed=101)
    ea = rand(allm, log_n, (2,), seed=102)
    ks0, ks1 = ctx.keyswitch(fc.to_device(d2), fc.to_device(eb), fc.to_device(ea))
    r0, r1 = coracle.keyswitch(d2, eb, ea, ctx.moduli, ctx.special, 2)
    assert (fc.to_host(ks0) == r0).all() and (fc.to_host(ks1) == r1).all()


def test_hommult_small_schoolbook(fc):
    ctx = ctx_for(fc, 10, 2)
    a = rand(ctx.moduli, 10, (2,), seed=4)
    b = rand(ctx.moduli, 10, (2,), seed=5)
    d = fc.to_host(ctx.hommult(fc.to_device(a), fc.to_device(b)))
    for li, q in enumerate(ctx.moduli):
        assert (d[0, li].astype(object) == pyoracle.negacyclic_mul(a[0, li], b[0, li], q)).all()


def test_hommult_identity_ciphertext(fc):
    """b = (1, 0): d0 = a0, d1 = a1, d2 = 0 at N = 2^16 (property, no oracle)."""
    ctx = ctx_for(fc, 16, 8)
    a = rand(ctx.moduli, 16, (3, 2), seed=30)
    b = np.zeros_like(a)
    b[:, 0, :, 0] = 1
    d = fc.to_host(ctx.hommult(fc.to_device(a), fc.to_device(b)))
    assert (d[:, 0] == a[:, 0]).all() and (d[:, 1] == a[:, 1]).all() and (d[:, 2] == 0).all()


def test_hommult_limb_window(fc):
    ctx = ctx_for(fc, 14, 4)
    a = rand(ctx.moduli[1:3], 14, (1, 2), seed=40)
    b = rand(ctx.moduli[1:3], 14, (1, 2), seed=41)
    d = fc.to_host(ctx.hommult(fc.to_device(a), fc.to_device(b), limb0=1))
    assert (d == coracle.hommult(a, b, ctx.moduli[1:3])).all()


@pytest.mark.parametrize("L,limb0,nl,B", [(8, 3, 3, 2), (16, 0, 16, 1), (8, 7, 1, 3), (12, 2, 9, 1)])
def test_hommult_split9_limb_windows(fc, L, limb0, nl, B):
    """N = 2^16 takes the 9 + 7 forward split (k_hm_col9 + the 7-stage rows with d_tw_fwd9): limb
    windows off 0 (the second twiddle table's per-limb offset), limb counts below, above and not a
    multiple of the 8 XCDs (the row kernel's limb placement), against the C oracle."""
    ctx = ctx_for(fc, 16, L)
    mods = ctx.moduli[limb0:limb0 + nl]
    a = rand(mods, 16, (B, 2), seed=50 + nl)
    b = rand(mods, 16, (B, 2), seed=60 + nl)
    d = fc.to_host(ctx.hommult(fc.to_device(a), fc.to_device(b), limb0=limb0))
    assert (d == coracle.hommult(a, b, mods)).all()


# ------------------------------------------------------------------ base conversion / key-switch

def test_baseconv_matches_oracle(fc):
    ctx = ctx_for(fc, 16, 16, K=4, dnum=4)
    mods = ctx.all_moduli
    x = rand(mods[2:6], 16, seed=50)
    out = fc.to_host(ctx.baseconv(fc.to_device(x), 2, 10, 10))
    assert (out == coracle.baseconv(x, mods[2:6], mods[10:20])).all()


@pytest.mark.parametrize("L,K,dnum", [(16, 4, 4), (8, 2, 3)])
def test_keyswitch_matches_oracle(fc, L, K, dnum):
    ctx = ctx_for(fc, 16, L, K=K, dnum=dnum)
    allm = ctx.all_moduli
    d2 = rand(ctx.moduli, 16, seed=60)
    eb = rand(allm, 16, (dnum,), seed=61)
    ea = rand(allm, 16, (dnum,), seed=62)
    ks0, ks1 = ctx.keyswitch(fc.to_device(d2), fc.to_device(eb), fc.to_device(ea))
    r0, r1 = coracle.keyswitch(d2, eb, ea, ctx.moduli, ctx.special, dnum)
    assert (fc.to_host(ks0) == r0).all() and (fc.to_host(ks1) == r1).all()


@pytest.mark.parametrize("L,K,dnum,batch", [
    (10, 2, 2, 2),   # digits of 5 limbs: fused row kernel, unfused ModUp (k_baseconv + column pass)
    (12, 3, 6, 1),   # dnum 6 > 4: the fully unfused path (full NTTs + k_ks_inner + k_moddown_finish)
    (16, 4, 4, 3),   # batched, the fused path end to end
    (7, 2, 3, 2),    # a ragged last digit (7 = 3 + 3 + 1)
])
def test_keyswitch_paths_match_oracle(fc, L, K, dnum, batch):
    """Every key-switch code path (fused / partly fused / unfused, ragged digits, batches) against
    the C oracle at N = 2^12."""
    ctx = ctx_for(fc, 12, L, K=K, dnum=dnum)
    allm = ctx.all_moduli
    d2 = rand(ctx.moduli, 12, (batch,), seed=70 + L)
    eb = rand(allm, 12, (dnum,), seed=71)
    ea = rand(allm, 12, (dnum,), seed=72)
    ks0, ks1 = ctx.keyswitch(fc.to_device(d2), fc.to_device(eb), fc.to_device(ea))
    h0, h1 = fc.to_host(ks0), fc.to_host(ks1)
    for b in range(batch):
        r0, r1 = coracle.keyswitch(d2[b], eb, ea, ctx.moduli, ctx.special, dnum)
        assert (h0[b] == r0).all() and (h1[b] == r1).all(), b


@pytest.mark.parametrize("log_n", [10, 11, 13, 14, 15, 17])
def test_keyswitch_every_ring_degree(fc, log_n):
    """The fused key-switch (row kernel with the inner product and ModDown's INTT row pass, the
    stage-0-folded conversions, P^-1 in the constants) at every other supported N: the row-kernel
    geometries differ (32 rows per workgroup at N = 2^10, too few tiles for the XCD placement
    below 2^14, a row group spanning two wavefronts at 2^17)."""
    L, K, dnum, batch = 4, 2, 2, 2
    ctx = ctx_for(fc, log_n, L, K=K, dnum=dnum)
    allm = ctx.all_moduli
    d2 = rand(ctx.moduli, log_n, (batch,), seed=80 + log_n)
    eb = rand(allm, log_n, (dnum,), seed=81)
    ea = rand(allm, log_n, (dnum,), seed=82)
    ks0, ks1 = ctx.keyswitch(fc.to_device(d2), fc.to_device(eb), fc.to_device(ea))
    h0, h1 = fc.to_host(ks0), fc.to_host(ks1)
    for b in range(batch):
        r0, r1 = coracle.keyswitch(d2[b], eb, ea, ctx.moduli, ctx.special, dnum)
        assert (h0[b] == r0).all() and (h1[b] == r1).all(), b


@pytest.mark.parametrize("G", [2, 4, 8])
def test_keyswitch_sharded_equals_unsharded(fc, G):
    """the G-way limb-sharded key-switch (one all-gather of INTT(d2)) concatenates to
    the single-device result bit for bit.  G shards run one after another on this one GPU."""
    L, K, dnum = 16, 4, 4
    ctx = ctx_for(fc, 16, L, K=K, dnum=dnum)
    d2 = rand(ctx.moduli, 16, seed=70)
    eb = rand(ctx.all_moduli, 16, (dnum,), seed=71)
    ea = rand(ctx.all_moduli, 16, (dnum,), seed=72)
    full0, full1 = ctx.keyswitch(fc.to_device(d2), fc.to_device(eb), fc.to_device(ea))
    c_all = fc.to_device(d2)
    ctx.intt_(c_all)
    nl = L // G
    parts0, parts1 = [], []
    for r in range(G):
        lo = r * nl
        own = np.concatenate([np.arange(lo, lo + nl), np.arange(L, L + K)])
        k0, k1 = ctx.keyswitch_shard(c_all, fc.to_device(d2[lo:lo + nl]),
                                     fc.to_device(np.ascontiguousarray(eb[:, own])),
                                     fc.to_device(np.ascontiguousarray(ea[:, own])), lo)
        parts0.append(fc.to_host(k0))
        parts1.append(fc.to_host(k1))
    assert (np.concatenate(parts0) == fc.to_host(full0)).all()
    assert (np.concatenate(parts1) == fc.to_host(full1)).all()


def test_keyswitch_decrypts_with_real_keys_on_gpu(fc):
    import random

    log_n, L, K, dnum = 10, 4, 2, 2
    n = 1 << log_n
    ctx = fc.Context(log_n, L=L, K=K, dnum=dnum)
    qs, ps = ctx.moduli, ctx.special
    rng = random.Random(5)
    s = [rng.randrange(-1, 2) for _ in range(n)]
    evk_b, evk_a = pyoracle.gen_relin_key(s, qs, ps, dnum, rng)
    d2 = np.stack([np.array([rng.randrange(q) for _ in range(n)], dtype=np.uint64) for q in qs])
    ks0, ks1 = ctx.keyswitch(fc.to_device(d2), fc.to_device(evk_b.astype(np.uint64)),
                             fc.to_device(evk_a.astype(np.uint64)))
    ks0, ks1 = fc.to_host(ks0).astype(object), fc.to_host(ks1).astype(object)
    col = pyoracle._mods_col(qs)
    sn = pyoracle.rns_ntt_fwd(pyoracle._to_rns(s, qs), qs)
    err = (ks0 + ks1 * sn - d2.astype(object) * sn * sn) % col
    e = pyoracle.crt_centered(pyoracle.rns_ntt_inv(err, qs), qs)
    assert max(abs(int(v)) for v in e) < 1 << 20


def test_bad_window_is_rejected(fc):
    ctx = ctx_for(fc, 12, 1)
    t = fc.to_device(np.zeros((1, 2, 4096), np.uint64))
    with pytest.raises(fc.FheError):
        ctx.ntt_(t)  # 2 limbs on a 1-limb context


def test_dist_sharded_keyswitch_single_rank_on_gpu(fc):
    """fhecore.dist driving the HIP Context (world 1: the all-gather is the identity)."""
    from fhecore.dist import LimbShard, sharded_keyswitch

    L, K, dnum = 8, 2, 3
    ctx = ctx_for(fc, 14, L, K=K, dnum=dnum)
    d2 = rand(ctx.moduli, 14, seed=80)
    eb = rand(ctx.all_moduli, 14, (dnum,), seed=81)
    ea = rand(ctx.all_moduli, 14, (dnum,), seed=82)
    k0, k1 = sharded_keyswitch(ctx, fc.to_device(d2), fc.to_device(eb), fc.to_device(ea),
                               LimbShard(L, 1, 0))
    r0, r1 = coracle.keyswitch(d2, eb, ea, ctx.moduli, ctx.special, dnum)
    assert (fc.to_host(k0) == r0).all() and (fc.to_host(k1) == r1).all()


@pytest.mark.parametrize("bits", [60, 61])
def test_lazy_headroom_variants_match_oracle(fc, bits):
    """Contexts whose moduli are all below 2^60 run the forward NTTs lazy up to 16q; 61-bit primes
    take the 8q variant (ntt.hip fwd_range).  Both must be bit-exact (NTT and HomMult)."""
    log_n = 12
    mods = fc.gen_moduli(log_n, 3, bits=bits)
    assert (max(mods) >= 1 << 60) == (bits == 61)
    ctx = fc.Context(log_n, moduli=mods)
    x = rand(mods, log_n, (2,), seed=bits)
    t = fc.to_device(x)
    ctx.ntt_(t)
    assert (fc.to_host(t) == coracle.ntt_fwd(x, mods)).all()
    a = rand(mods, log_n, (2, 2), seed=bits + 1)
    b = rand(mods, log_n, (2, 2), seed=bits + 2)
    d = fc.to_host(ctx.hommult(fc.to_device(a), fc.to_device(b)))
    for i in range(2):
        assert (d[i] == coracle.hommult(a[i], b[i], mods)).all()


def test_keyswitch_batch_in_cache_sized_passes(fc):
    """fhe_keyswitch runs a batch above 256 MiB of d2 in passes (N = 2^16, L = 16: 32 ciphertexts
    per pass): 33 ciphertexts = a full pass + a one-ciphertext pass.  The whole batch equals the
    one-pass distributed path (fhe_keyswitch_dist, one rank, one chunk) word for word, and the
    first and last ciphertexts equal the C oracle."""
    from fhecore.dist import RcclComm

    L, K, dnum, B = 16, 4, 4, 33
    ctx = ctx_for(fc, 16, L, K=K, dnum=dnum)
    allm = ctx.all_moduli
    d2 = rand(ctx.moduli, 16, (B,), seed=90)
    eb = rand(allm, 16, (dnum,), seed=91)
    ea = rand(allm, 16, (dnum,), seed=92)
    dd, db, da = fc.to_device(d2), fc.to_device(eb), fc.to_device(ea)
    ks0, ks1 = ctx.keyswitch(dd, db, da)
    comm = RcclComm()
    try:
        w0, w1 = ctx.keyswitch_dist(comm, dd, db, da, chunks=1)
    finally:
        comm.close()
    h0, h1 = fc.to_host(ks0), fc.to_host(ks1)
    assert (h0 == fc.to_host(w0)).all() and (h1 == fc.to_host(w1)).all()
    for b in (0, B - 1):
        r0, r1 = coracle.keyswitch(d2[b], eb, ea, ctx.moduli, ctx.special, dnum)
        assert (h0[b] == r0).all() and (h1[b] == r1).all(), b
