"""GPU parity of the batched key-switch (one key read per batch) and its limb shards."""
import numpy as np
import pytest

import coracle

pytestmark = pytest.mark.gpu


def rand(mods, log_n, lead=(), seed=0):
    rng = np.random.default_rng(seed)
    n = 1 << log_n
    return np.stack([rng.integers(0, q, size=lead + (n,), dtype=np.uint64) for q in mods],
                    axis=len(lead))


@pytest.fixture(scope="module")
def ks_setup():
    import fhecore as fc

    L, K, dnum, log_n, B = 16, 4, 4, 16, 3
    ctx = fc.Context(log_n, L=L, K=K, dnum=dnum)
    d2 = rand(ctx.moduli, log_n, (B,), seed=90)
    eb = rand(ctx.all_moduli, log_n, (dnum,), seed=91)
    ea = rand(ctx.all_moduli, log_n, (dnum,), seed=92)
    ref = [coracle.keyswitch(d2[i], eb, ea, ctx.moduli, ctx.special, dnum) for i in range(B)]
    return fc, ctx, d2, eb, ea, ref


def test_batched_keyswitch_matches_oracle(ks_setup):
    fc, ctx, d2, eb, ea, ref = ks_setup
    k0, k1 = ctx.keyswitch(fc.to_device(d2), fc.to_device(eb), fc.to_device(ea))
    k0, k1 = fc.to_host(k0), fc.to_host(k1)
    for i, (r0, r1) in enumerate(ref):
        assert (k0[i] == r0).all() and (k1[i] == r1).all()


@pytest.mark.parametrize("G", [2, 8])
def test_batched_shards_concatenate(ks_setup, G):
    from fhecore.dist import LimbShard

    fc, ctx, d2, eb, ea, ref = ks_setup
    L, K = ctx.L, ctx.K
    c_all = fc.to_device(d2)
    ctx.intt_(c_all)
    parts0, parts1 = [], []
    for r in range(G):
        sh = LimbShard(L, G, r)
        rows = sh.evk_rows(K)
        k0, k1 = ctx.keyswitch_shard(c_all, fc.to_device(np.ascontiguousarray(d2[:, sh.lo:sh.hi])),
                                     fc.to_device(np.ascontiguousarray(eb[:, rows])),
                                     fc.to_device(np.ascontiguousarray(ea[:, rows])), sh.lo)
        parts0.append(fc.to_host(k0))
        parts1.append(fc.to_host(k1))
    g0, g1 = np.concatenate(parts0, axis=1), np.concatenate(parts1, axis=1)
    for i, (r0, r1) in enumerate(ref):
        assert (g0[i] == r0).all() and (g1[i] == r1).all()


def test_pass_batch_and_pass_sized_workspaces(ks_setup):
    """fhe_keyswitch_pass_batch: the pass size the single-device key-switch, rotate and mul-relin
    split a batch into (256 MiB of L limbs: 32 ciphertexts at N = 2^16, L = 16), and the Python
    wrappers size their workspaces for one pass, not for the whole batch."""
    fc, ctx, d2, eb, ea, ref = ks_setup
    lib = fc.load()
    p = lambda b: lib.fhe_keyswitch_pass_batch(ctx.handle, b)  # noqa: E731
    assert (p(0), p(1), p(31), p(32), p(33), p(1000)) == (0, 1, 31, 32, 32, 32)
    sized = []
    orig = ctx.workspace

    def spy(nbytes):
        sized.append(nbytes)
        return orig(nbytes)

    ctx.workspace = spy
    try:
        big = np.concatenate([d2] * 11 + [d2[:1]])  # 34 ciphertexts: two passes
        k0, k1 = ctx.keyswitch(fc.to_device(big), fc.to_device(eb), fc.to_device(ea))
    finally:
        del ctx.workspace
    assert sized == [lib.fhe_keyswitch_workspace(ctx.handle, ctx.L, 32)]
    k0, k1 = fc.to_host(k0), fc.to_host(k1)
    for i in range(big.shape[0]):
        r0, r1 = ref[i % d2.shape[0]]
        assert (k0[i] == r0).all() and (k1[i] == r1).all(), i
