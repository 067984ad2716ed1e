"""The key-switch aliasing contract (include/fhecore.h, "Aliasing"): an output may be d2 itself (the
in-place call) or lie wholly outside it; any other overlap -- and any overlap of fhe_rotate's output
with its input -- is refused with FHE_EINVAL before anything is launched.

The in-place calls run the lz16 fused path end to end (k_ks_row_fin reads each d2 word at the
position it later overwrites) and are compared word for word with the C oracle at the BASELINE
configs[3] shape (N = 2^16, L = 16, K = 4, dnum = 4), including a batch that straddles the 256 MiB
pass boundary of fhe_keyswitch.  The reference has no key-switch (SURVEY.md §8a'); the pointwise
products it feeds are /root/reference/arithmetic.py:11-13."""
import numpy as np
import pytest

import coracle

pytestmark = pytest.mark.gpu

LOG_N, L, K, DNUM = 16, 16, 4, 4


@pytest.fixture(scope="module")
def fc():
    import fhecore

    return fhecore


@pytest.fixture(scope="module")
def ks_ctx(fc):
    return fc.Context(LOG_N, L=L, K=K, dnum=DNUM)


def rand(mods, lead, seed):
    rng = np.random.default_rng(seed)
    n = 1 << LOG_N
    return np.stack([rng.integers(0, q, size=lead + (n,), dtype=np.uint64) for q in mods],
                    axis=len(lead))


@pytest.fixture(scope="module")
def keys(fc, ks_ctx):
    eb = rand(ks_ctx.all_moduli, (DNUM,), 201)
    ea = rand(ks_ctx.all_moduli, (DNUM,), 202)
    return eb, ea, fc.to_device(eb), fc.to_device(ea)


def oracle(ctx, d2, eb, ea):
    return coracle.keyswitch(d2, eb, ea, ctx.moduli, ctx.special, DNUM)


@pytest.mark.parametrize("which", [0, 1])
def test_keyswitch_output_in_place_on_d2(fc, ks_ctx, keys, which):
    """ks0 (which = 0) or ks1 (which = 1) is d2 itself: batch 3 at the configs[3] shape."""
    eb, ea, db, da = keys
    d2 = rand(ks_ctx.moduli, (3,), 210 + which)
    buf = fc.to_device(d2)
    other = ks_ctx.empty(*buf.shape)
    out = (buf, other) if which == 0 else (other, buf)
    k0, k1 = ks_ctx.keyswitch(buf, db, da, out=out)
    assert k0.data_ptr() == out[0].data_ptr() and k1.data_ptr() == out[1].data_ptr()
    h0, h1 = fc.to_host(k0), fc.to_host(k1)
    for b in range(3):
        r0, r1 = oracle(ks_ctx, d2[b], eb, ea)
        assert (h0[b] == r0).all() and (h1[b] == r1).all(), b


def test_keyswitch_in_place_straddling_a_pass(fc, ks_ctx, keys):
    """33 ciphertexts at L = 16 (8 MiB each): fhe_keyswitch runs a 32-ciphertext pass and a
    1-ciphertext pass.  With ks0 == d2 the first pass must not touch the second pass's input: the
    in-place result equals the out-of-place one word for word, and its first and last ciphertexts
    equal the oracle."""
    eb, ea, db, da = keys
    B = 33
    assert fc.load().fhe_keyswitch_pass_batch(ks_ctx.handle, B) == 32
    d2 = rand(ks_ctx.moduli, (B,), 220)
    ref0, ref1 = ks_ctx.keyswitch(fc.to_device(d2), db, da)
    buf = fc.to_device(d2)
    k1 = ks_ctx.empty(*buf.shape)
    ks_ctx.keyswitch(buf, db, da, out=(buf, k1))
    h0, h1 = fc.to_host(buf), fc.to_host(k1)
    assert (h0 == fc.to_host(ref0)).all() and (h1 == fc.to_host(ref1)).all()
    for b in (0, B - 1):
        r0, r1 = oracle(ks_ctx, d2[b], eb, ea)
        assert (h0[b] == r0).all() and (h1[b] == r1).all(), b


def _refused(fc, fn):
    with pytest.raises(fc.FheError) as e:
        fn()
    assert "FHE_EINVAL" in str(e.value)


def test_keyswitch_partial_overlaps_are_refused(fc, ks_ctx, keys):
    """Outputs shifted onto d2 (by one ciphertext, by one limb), ks0 == ks1: FHE_EINVAL, and the
    buffers are untouched (nothing was launched)."""
    _, _, db, da = keys
    B = 2
    d2 = rand(ks_ctx.moduli, (B + 1,), 230)
    buf = fc.to_device(d2)
    other = ks_ctx.empty(B, L, 1 << LOG_N)
    lin = buf.view(-1)
    words = B * L << LOG_N
    shifted_limb = lin[(1 << LOG_N):(1 << LOG_N) + words].view(B, L, 1 << LOG_N)
    for out in ((buf[1:], other), (other, buf[1:]), (shifted_limb, other), (other, other)):
        _refused(fc, lambda: ks_ctx.keyswitch(buf[:B], db, da, out=out))
    assert (fc.to_host(buf) == d2).all()


def test_rotate_overlap_is_refused(fc, ks_ctx, keys):
    """fhe_rotate reads c0 through sigma while other workgroups write out: an output overlapping the
    input by one ciphertext is refused, not only out == in."""
    _, _, db, da = keys
    B = 2
    ct = rand(ks_ctx.moduli, (B + 1, 2), 240)
    buf = fc.to_device(ct)
    g = ks_ctx.galois_elt(1)
    for out in (buf[1:], buf[:B]):
        _refused(fc, lambda: ks_ctx.rotate(buf[:B], g, db, da, out=out))
    assert (fc.to_host(buf) == ct).all()
