"""GPU tests of the native multi-GPU key-switch (gpu-fhe_amd/csrc/dist.cpp):
the rank-major all-gather layout that the local key-switch reads without a reorder copy (every
rank of an even or uneven G-way sharding, run one after another on this GPU), and the full
fhe_keyswitch_dist path over a one-rank RCCL communicator (INTT + ncclAllGather + key-switch, in
chunks) -- all bit-exact against the single-device key-switch and the C oracle.  Multi-rank
orchestration runs over gloo on the CPU (tests/test_dist_cpu.py); N > 1 GPUs are not available to
these tests."""
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


@pytest.mark.parametrize("log_n,L,K,dnum,G,batch", [
    (16, 16, 4, 4, 8, 2),   # configs[3]: 2 limbs per rank, the fused kernels
    (12, 16, 4, 4, 6, 3),   # uneven: 3,3,3,3,3,1 limbs
    (12, 10, 2, 2, 4, 2),   # uneven digits and shards: 3,3,3,1
    (12, 10, 2, 3, 8, 1),   # ranks without limbs: 2,2,2,2,2,0,0,0
])
def test_ranked_gather_layout_shards(fc, log_n, L, K, dnum, G, batch):
    from fhecore.dist import LimbShard

    ctx = fc.Context(log_n, L=L, K=K, dnum=dnum)
    d2 = rand(ctx.moduli, log_n, (batch,), seed=L + G)
    eb = rand(ctx.all_moduli, log_n, (dnum,), seed=1)
    ea = rand(ctx.all_moduli, log_n, (dnum,), seed=2)
    full0, full1 = ctx.keyswitch(fc.to_device(d2), fc.to_device(eb), fc.to_device(ea))
    c = coracle.ntt_inv(d2, ctx.moduli)  # coefficient form of every limb
    width = -(-L // G)
    ranked = np.zeros((G, batch, width, 1 << log_n), dtype=np.uint64)
    for r in range(G):  # what the all-gather leaves on every rank
        sh = LimbShard(L, G, r)
        ranked[r, :, :sh.nlimbs] = c[:, sh.lo:sh.hi]
    ranked_d = fc.to_device(ranked)
    parts0, parts1 = [], []
    for r in range(G):
        sh = LimbShard(L, G, r)
        if sh.nlimbs == 0:
            continue
        rows = sh.evk_rows(K)
        k0, k1 = ctx.keyswitch_shard(ranked_d, fc.to_device(np.ascontiguousarray(d2[:, sh.lo:sh.hi])),
                                     fc.to_device(np.ascontiguousarray(eb[:, rows])),
                                     fc.to_device(np.ascontiguousarray(ea[:, rows])), sh.lo,
                                     ranks=G)
        parts0.append(fc.to_host(k0))
        parts1.append(fc.to_host(k1))
    assert (np.concatenate(parts0, axis=1) == fc.to_host(full0)).all()
    assert (np.concatenate(parts1, axis=1) == fc.to_host(full1)).all()
    # a window that is not a rank's shard is refused
    with pytest.raises(fc.FheError):
        ctx.keyswitch_shard(ranked_d, fc.to_device(np.ascontiguousarray(d2[:, 1:2])),
                            fc.to_device(np.ascontiguousarray(eb[:, [1] + list(range(L, L + K))])),
                            fc.to_device(np.ascontiguousarray(ea[:, [1] + list(range(L, L + K))])),
                            1, ranks=G)


@pytest.mark.parametrize("log_n,L,K,dnum,G,batch,chunks", [
    (16, 16, 4, 4, 8, 4, 4),   # configs[3] at 8 ranks, the bench's chunking (1 ciphertext each)
    (16, 16, 4, 4, 2, 5, 4),   # 2 ranks, uneven chunks (2, 2, 1)
    (14, 16, 4, 4, 4, 6, 0),   # default chunking
    (12, 16, 4, 4, 6, 3, 2),   # uneven shards 3,3,3,3,3,1
    (12, 10, 2, 3, 8, 2, 2),   # ranks without limbs
    (12, 10, 2, 2, 3, 7, 16),  # more chunks asked than ciphertexts
])
def test_keyswitch_dist_loopback_g_ranks(fc, log_n, L, K, dnum, G, batch, chunks):
    """fhe_keyswitch_dist's G-rank plan executed on this GPU (fhe_keyswitch_dist_loopback: every
    virtual rank's INTT writes its block of one gather region -- what the in-place all-gather
    leaves on each rank -- then every rank's chunked key-switch reads it through CAll::ranked):
    the G > 1 offsets, chunking and rank blocks of the native multi-GPU path, bit-exact against
    the single-device key-switch."""
    from fhecore.dist import LimbShard

    ctx = fc.Context(log_n, L=L, K=K, dnum=dnum)
    d2 = rand(ctx.moduli, log_n, (batch,), seed=G + batch)
    eb = rand(ctx.all_moduli, log_n, (dnum,), seed=5)
    ea = rand(ctx.all_moduli, log_n, (dnum,), seed=6)
    full0, full1 = ctx.keyswitch(fc.to_device(d2), fc.to_device(eb), fc.to_device(ea))
    parts = [[], [], []]
    for r in range(G):
        sh = LimbShard(L, G, r)
        if sh.nlimbs == 0:
            for p in parts:
                p.append(None)
            continue
        rows = sh.evk_rows(K)
        parts[0].append(fc.to_device(np.ascontiguousarray(d2[:, sh.lo:sh.hi])))
        parts[1].append(fc.to_device(np.ascontiguousarray(eb[:, rows])))
        parts[2].append(fc.to_device(np.ascontiguousarray(ea[:, rows])))
    k0, k1 = ctx.keyswitch_dist_loopback(*parts, chunks=chunks)
    got0 = np.concatenate([fc.to_host(t) for t in k0 if t is not None], axis=1)
    got1 = np.concatenate([fc.to_host(t) for t in k1 if t is not None], axis=1)
    assert (got0 == fc.to_host(full0)).all() and (got1 == fc.to_host(full1)).all()


@pytest.mark.parametrize("batch,chunks", [(1, 0), (4, 0), (5, 4), (3, 8), (6, 2)])
def test_keyswitch_dist_one_rank_rccl(fc, batch, chunks):
    """fhe_keyswitch_dist through a real RCCL communicator (world 1): INTT into the gather buffer,
    ncclAllGather on the communicator's stream, chunked key-switch; equals fhe_keyswitch and the
    oracle."""
    from fhecore.dist import RcclComm

    L, K, dnum, log_n = 16, 4, 4, 14
    ctx = fc.Context(log_n, L=L, K=K, dnum=dnum)
    comm = RcclComm()
    assert (comm.world, comm.rank) == (1, 0) and comm.shard(L).nlimbs == L
    d2 = rand(ctx.moduli, log_n, (batch,), seed=batch)
    eb = rand(ctx.all_moduli, log_n, (dnum,), seed=3)
    ea = rand(ctx.all_moduli, log_n, (dnum,), seed=4)
    k0, k1 = ctx.keyswitch_dist(comm, fc.to_device(d2), fc.to_device(eb), fc.to_device(ea),
                                chunks=chunks)
    r0, r1 = ctx.keyswitch(fc.to_device(d2), fc.to_device(eb), fc.to_device(ea))
    assert (fc.to_host(k0) == fc.to_host(r0)).all() and (fc.to_host(k1) == fc.to_host(r1)).all()
    o0, o1 = coracle.keyswitch(d2[0], eb, ea, ctx.moduli, ctx.special, dnum)
    assert (fc.to_host(k0)[0] == o0).all() and (fc.to_host(k1)[0] == o1).all()
    # one timed all-gather per chunk of the plan
    from fhecore.dist import dist_plan

    ms = comm.gather_ms()
    assert len(ms) == dist_plan(L, log_n, 1, 0, batch, chunks).chunks
    assert all(v >= 0 for v in ms)
    comm.close()


@pytest.mark.parametrize("chunks", [1, 4])
def test_bench_dist_check_native_world1(fc, chunks):
    """bench.py's dist_check on the GPU (world 1): the native RCCL key-switch and the limb-sharded
    HomMult against the single-device calls count zero mismatched words, and a corrupted shard is
    counted -- the check that makes the driver's multi-GPU runs fail loudly on a wrong answer."""
    import os
    import sys

    import torch

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from fhecore.dist import LimbShard, RcclComm

    L, K, dnum, log_n = 16, 4, 4, 13
    ctx = fc.Context(log_n, L=L, K=K, dnum=dnum)
    comm = RcclComm()
    shard = LimbShard(L, 1, 0)
    d2 = fc.to_device(rand(ctx.moduli, log_n, (2 * chunks,), seed=11))
    eb = fc.to_device(rand(ctx.all_moduli, log_n, (dnum,), seed=12))
    ea = fc.to_device(rand(ctx.all_moduli, log_n, (dnum,), seed=13))
    native = lambda d, kb, ka: ctx.keyswitch_dist(comm, d, kb, ka, chunks=chunks)  # noqa: E731
    assert bench.check_keyswitch_shard(ctx, shard, K, d2, eb, ea, native) == 0

    def corrupted(d, kb, ka):
        k0, k1 = native(d, kb, ka)
        k1.view(-1)[7] ^= 1
        return k0, k1

    assert bench.check_keyswitch_shard(ctx, shard, K, d2, eb, ea, corrupted) == 1
    hctx = fc.Context(log_n, L=4)
    a = fc.to_device(rand(hctx.moduli, log_n, (2, 2), seed=14))
    b = fc.to_device(rand(hctx.moduli, log_n, (2, 2), seed=15))
    assert bench.check_hommult_shard(hctx, LimbShard(4, 1, 0), a, b) == 0
    torch.cuda.synchronize()
    comm.close()


def test_bench_default_line_end_to_end():
    """bench.py as the driver runs it (one GPU, a short run): one JSON line carrying the headline,
    the roofline, the key-switch leg and a bit-exact dist_check, and exit status 0."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "3", "--warmup",
                        "1", "--batch", "8", "--ks-batch", "8", "--no-cpu-baseline", "--no-pmc"],
                       capture_output=True, text=True, timeout=110, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["value"] > 0 and line["unit"] == "HomMult/s" and line["n_gpus"] == 1
    assert line["roofline"]["kernel"] == "hm_row_tensor" and line["roofline"]["frac"] > 0
    assert line["keyswitch_leg"]["value"] > 0
    assert line["dist_check"]["result"] == "bit-exact"


@pytest.mark.parametrize("log_n,G,groups,batch,chunks", [
    (16, 8, 4, 8, 2),   # g = 2 limb shards x 4 ciphertext groups (configs[3] key shape)
    (16, 8, 2, 6, 0),   # g = 4 x 2 groups, default chunking
    (16, 8, 8, 8, 1),   # g = 1: every rank key-switches whole ciphertexts, no gather
    (12, 8, 4, 5, 2),   # uneven groups: 2, 2, 1, 0 ciphertexts
    (12, 6, 2, 7, 4),   # g = 3: uneven shards 6, 6, 4 of L = 16
])
def test_keyswitch_dist_hybrid_loopback(fc, log_n, G, groups, batch, chunks):
    """The hybrid partition (fhe_dist_hybrid: `groups` ciphertext groups x g = G / groups limb
    shards, the all-gather inside each group) executed for all G virtual ranks on this GPU: rank r's
    outputs are fhe_keyswitch's rows of its group's ciphertexts and its shard's limbs, bit for bit
    (DESIGN.md §7 models its rates)."""
    from fhecore.dist import LimbShard, hybrid_plan

    L, K, dnum = 16, 4, 4
    ctx = fc.Context(log_n, L=L, K=K, dnum=dnum)
    d2 = rand(ctx.moduli, log_n, (batch,), seed=31 + G * groups)
    eb = rand(ctx.all_moduli, log_n, (dnum,), seed=32)
    ea = rand(ctx.all_moduli, log_n, (dnum,), seed=33)
    full0, full1 = (fc.to_host(t) for t in ctx.keyswitch(fc.to_device(d2), fc.to_device(eb),
                                                          fc.to_device(ea)))
    g = G // groups
    plans = [hybrid_plan(L, log_n, G, groups, r, batch, chunks) for r in range(G)]
    d2p, ebp, eap = [], [], []
    for r, h in enumerate(plans):
        assert (h.g, h.group, h.shard) == (g, r // g, r % g)
        sh = LimbShard(L, g, h.shard)
        assert (h.plan.limb0, h.plan.nlimbs, h.plan.batch) == (sh.lo, sh.nlimbs, h.batch)
        rows = sh.evk_rows(K)
        d2p.append(fc.to_device(np.ascontiguousarray(d2[h.batch0:h.batch0 + h.batch, sh.lo:sh.hi]))
                   if sh.nlimbs else None)
        ebp.append(fc.to_device(np.ascontiguousarray(eb[:, rows])) if sh.nlimbs else None)
        eap.append(fc.to_device(np.ascontiguousarray(ea[:, rows])) if sh.nlimbs else None)
    ks0, ks1 = ctx.keyswitch_dist_hybrid_loopback(groups, d2p, ebp, eap, chunks=chunks)
    covered = np.zeros((batch, L), dtype=int)
    for r, h in enumerate(plans):
        if ks0[r] is None:
            continue
        sh = LimbShard(L, g, h.shard)
        sl = (slice(h.batch0, h.batch0 + h.batch), slice(sh.lo, sh.hi))
        assert (fc.to_host(ks0[r]) == full0[sl]).all(), r
        assert (fc.to_host(ks1[r]) == full1[sl]).all(), r
        covered[sl] += 1
    assert (covered == 1).all()  # every (ciphertext, limb) row exactly once
