"""Edge cases of the HIP path (GPU): empty batches, ragged reference-shim shapes, the largest limb
count and transform size, all-maximum residues, and the bench's own HomMult shape checked
bit-exact against the C oracle.  Everything goes through the C ABI (ctypes); the oracle is only
the checker."""
import numpy as np
import pytest

import coracle

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


def test_empty_batches_are_noops(fc):
    """Zero polynomials / ciphertexts: every entry point returns at once, shapes preserved."""
    import torch

    ctx = fc.Context(12, L=2)
    n = 1 << 12
    t = torch.empty(0, 2, n, dtype=torch.int64, device="cuda")
    ctx.ntt_(t)
    ctx.intt_(t)
    assert tuple(t.shape) == (0, 2, n)
    assert tuple(ctx.vec("add", t, t).shape) == (0, 2, n)
    a = torch.empty(0, 2, 2, n, dtype=torch.int64, device="cuda")
    d = ctx.hommult(a, a)
    assert tuple(d.shape) == (0, 3, 2, n)


@pytest.mark.parametrize("shape", [(7,), (3, 5), (2, 3, 5), (1, 1), (0,), (4, 0)])
@pytest.mark.parametrize("op", ["vec_add", "vec_sub", "vec_mul"])
def test_reference_shim_ragged_shapes(fc, shape, op):
    """arithmetic.vec_* on shapes no kernel tiles evenly (odd lengths, empty axes), exact values
    (the reference's semantics on object-dtype input, /root/reference/arithmetic.py:3-13)."""
    import arithmetic

    q = (1 << 60) - 93  # any modulus: the generic vec_op_mod path
    rng = np.random.default_rng(len(shape) * 10 + sum(shape))
    a = rng.integers(0, q, size=shape, dtype=np.uint64)
    b = rng.integers(0, q, size=shape, dtype=np.uint64)
    got = np.asarray(getattr(arithmetic, op)(a, b, q))
    f = {"vec_add": lambda x, y: (x + y) % q, "vec_sub": lambda x, y: (x - y) % q,
         "vec_mul": lambda x, y: (x * y) % q}[op]
    want = np.array([f(int(x), int(y)) for x, y in zip(a.reshape(-1), b.reshape(-1))],
                    dtype=object).reshape(shape)
    assert got.shape == shape
    assert all(int(x) == int(y) for x, y in zip(got.reshape(-1), want.reshape(-1)))


def test_ntt_many_limbs_round_trip(fc):
    """64 RNS limbs (the most a context takes) at N = 2^11: forward vs oracle, inverse back."""
    ctx = fc.Context(11, L=64)
    x = rand(ctx.moduli, 11, (1,), seed=64)
    t = fc.to_device(x)
    ctx.ntt_(t)
    assert (fc.to_host(t) == coracle.ntt_fwd(x, ctx.moduli)).all()
    ctx.intt_(t)
    assert (fc.to_host(t) == x).all()


def test_ntt_all_max_residues_largest_n(fc):
    """q - 1 in every coefficient at N = 2^17 (the deepest lazy ranges), 2 limbs."""
    ctx = fc.Context(17, L=2)
    n = 1 << 17
    x = np.stack([np.full(n, q - 1, dtype=np.uint64) for q in ctx.moduli])[None]
    t = fc.to_device(x)
    ctx.ntt_(t)
    assert (fc.to_host(t) == coracle.ntt_fwd(x, ctx.moduli)).all()
    ctx.intt_(t)
    assert (fc.to_host(t) == x).all()


def test_hommult_bench_shape_matches_oracle(fc):
    """bench.py's default HomMult shape (N = 2^16, 8 limbs, 64 ciphertext pairs per GPU), every
    output word compared with the C oracle."""
    ctx = fc.Context(16, L=8)
    a = rand(ctx.moduli, 16, (64, 2), seed=640)
    b = rand(ctx.moduli, 16, (64, 2), seed=641)
    d = fc.to_host(ctx.hommult(fc.to_device(a), fc.to_device(b)))
    assert (d == coracle.hommult(a, b, ctx.moduli)).all()


@pytest.mark.parametrize("log_n,L", [(12, 3), (16, 8)])
def test_out_of_place_ntt_leaves_source(fc, log_n, L):
    """fhe_ntt_fwd_to / fhe_ntt_inv_to (Context.ntt / intt): dst = NTT(src), src untouched."""
    ctx = fc.Context(log_n, L=L)
    x = rand(ctx.moduli, log_n, (2,), seed=log_n + L)
    src = fc.to_device(x)
    y = ctx.ntt(src)
    assert (fc.to_host(src) == x).all()
    assert (fc.to_host(y) == coracle.ntt_fwd(x, ctx.moduli)).all()
    z = ctx.intt(y)
    assert (fc.to_host(z) == x).all() and (fc.to_host(y) == coracle.ntt_fwd(x, ctx.moduli)).all()


@pytest.mark.parametrize("world", [2, 8])
def test_hommult_rank_shapes_of_the_scaling_bench(fc, world):
    """The per-rank shape bench.py runs at N = 2 / 8 GPUs (L = 8 limbs sharded, 64 N ciphertext
    pairs, the last rank's limb window): the whole batch on the GPU, the first and last pairs
    checked bit-exact against the C oracle."""
    import torch
    from fhecore import dist as fdist

    ctx = fc.Context(16, L=8)
    shard = fdist.LimbShard(8, world, world - 1)
    mods = ctx.moduli[shard.lo:shard.hi]
    B = 64 * world
    gen = torch.Generator(device="cuda")
    gen.manual_seed(world)
    a = torch.stack([torch.randint(0, q, (B, 2, 1 << 16), generator=gen, dtype=torch.int64,
                                   device="cuda") for q in mods], 2)
    b = torch.stack([torch.randint(0, q, (B, 2, 1 << 16), generator=gen, dtype=torch.int64,
                                   device="cuda") for q in mods], 2)
    d = fdist.sharded_hommult(ctx, a, b, shard)
    for sl in (slice(0, 2), slice(B - 2, B)):
        want = coracle.hommult(fc.to_host(a[sl]), fc.to_host(b[sl]), mods)
        assert (fc.to_host(d[sl]) == want).all()


def test_configs4_full_batch_round_trip(fc):
    """BASELINE configs[4] at its full size on one GPU: 1024 polynomials x 32 limbs x N = 2^17
    (2^32 residues, 32 GiB) -- the whole batch through the forward NTT (first and last
    polynomial compared with the C oracle) and back through the inverse (every word compared
    with a device copy of the input)."""
    import torch

    log_n, L, P = 17, 32, 1024
    n = 1 << log_n
    ctx = fc.Context(log_n, L=L)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(1024)
    x = torch.empty(P, L, n, dtype=torch.int64, device="cuda")
    for l, q in enumerate(ctx.moduli):  # uniform residues, one limb at a time (bounded temporaries)
        x[:, l, :] = torch.randint(0, q, (P, n), generator=gen, dtype=torch.int64, device="cuda")
    keep = x.clone()
    ctx.ntt_(x)
    for p in (0, P - 1):
        assert (fc.to_host(x[p]) == coracle.ntt_fwd(fc.to_host(keep[p]), ctx.moduli)).all()
    ctx.intt_(x)
    torch.cuda.synchronize()
    assert torch.equal(x, keep)
    del x, keep
    torch.cuda.empty_cache()


def test_oversize_launch_is_refused(fc):
    """Launch sizes are checked before any kernel is launched (csrc/internal.hpp check_grid): a
    grid dimension the dispatch cannot hold returns FHE_EINVAL instead of being truncated.  Here
    70000 polynomials at N = 2^10 put 70000 workgroups on the automorphism's z dimension (at most
    65535); the buffers are real, so nothing could fault even if the check were missing."""
    import torch

    ctx = fc.Context(10, L=1)
    x = torch.zeros(70000, 1, 1 << 10, dtype=torch.int64, device="cuda")
    with pytest.raises(fc.FheError, match="launch too large"):
        ctx.automorphism(x, 5)
    # one poly fewer than the limit still runs
    y = ctx.automorphism(x[:65535], 5)
    assert tuple(y.shape) == (65535, 1, 1 << 10)


def test_internal_workspace_shared_across_streams(fc):
    """workspace == NULL on alternating streams (include/fhecore.h conventions): every call uses
    the context's one internal buffer, so a call on another stream must not start before the
    previous call has finished with it.  Two different HomMult batches on two streams, issued
    back to back several times, each still equal to the same product computed alone."""
    import torch
    from fhecore._capi import check, load

    lib = load()
    log_n, L, B = 14, 4, 8
    ctx = fc.Context(log_n, L=L)
    n = 1 << log_n
    mods = list(ctx.moduli)
    ins = [tuple(fc.to_device(rand(mods, log_n, (B, 2), seed=s + k)) for k in (0, 1))
           for s in (11, 23)]
    want = [ctx.hommult(a, b).cpu() for a, b in ins]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [torch.empty(B, 3, L, n, dtype=torch.int64, device="cuda") for _ in ins]
    torch.cuda.synchronize()
    for _ in range(4):
        for o in outs:
            o.zero_()
        torch.cuda.synchronize()
        for (a, b), o, s in zip(ins, outs, streams):  # back to back, no host sync in between
            check(lib.fhe_hommult(ctx.handle, o.data_ptr(), a.data_ptr(), b.data_ptr(), B, 0, L,
                                  None, s.cuda_stream), "fhe_hommult")
        torch.cuda.synchronize()
        for o, w in zip(outs, want):
            assert torch.equal(o.cpu(), w)
