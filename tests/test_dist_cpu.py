"""Multi-rank (gloo, world_size 2 and 4, CPU) tests of the RNS-limb sharding orchestration in
fhecore/dist.py: the same code drives the HIP Context on MI355X ranks over RCCL.  The engine here
is a CPU restatement (oracle/, test infrastructure) with the Context's method signatures."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import coracle
import pyoracle
from fhecore.dist import (LimbShard, all_gather_limbs, ranked_to_limbs, sharded_hommult,
                          sharded_keyswitch)

LOG_N, L, K, DNUM = 6, 4, 2, 2


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64))


def _a(t):
    return t.contiguous().numpy().view(np.uint64)


class CpuEngine:
    """Context-shaped CPU engine over the oracle (torch int64 CPU tensors)."""

    def __init__(self, qs, ps):
        self.qs, self.ps = list(qs), list(ps)

    def intt_(self, t, limb0=0):
        nl = t.shape[-2]
        if nl == 0:
            return t
        t.copy_(_t(coracle.ntt_inv(_a(t), self.qs[limb0:limb0 + nl])))
        return t

    def hommult(self, a, b, out=None, limb0=0, workspace=None):
        nl = a.shape[-2]
        if nl == 0:  # a rank without limbs (uneven shards)
            return torch.empty(a.shape[:-3] + (3, 0, a.shape[-1]), dtype=torch.int64)
        return _t(coracle.hommult(_a(a), _a(b), self.qs[limb0:limb0 + nl]))

    def keyswitch(self, d2, evk_b, evk_a):
        """The single-device key-switch of the whole [batch, L, N] input (bench.dist_check's
        reference side)."""
        outs = [coracle.keyswitch(d, _a(evk_b), _a(evk_a), self.qs, self.ps, DNUM)
                for d in _a(d2).reshape(-1, L, 1 << LOG_N)]
        k0 = np.stack([o[0] for o in outs]).astype(np.uint64).reshape(d2.shape)
        k1 = np.stack([o[1] for o in outs]).astype(np.uint64).reshape(d2.shape)
        return _t(k0), _t(k1)

    def keyswitch_shard(self, c_all, d2_own, evk_b, evk_a, limb0, ranks=None):
        nl = d2_own.shape[-2]
        if nl == 0:
            return torch.empty_like(d2_own), torch.empty_like(d2_own)
        if ranks is not None:  # the rank-major all-gather output [ranks, batch, width, N]
            c_all = ranked_to_limbs(c_all, LimbShard(L, ranks, 0))
        ca, da = _a(c_all).reshape(-1, L, 1 << LOG_N), _a(d2_own).reshape(-1, nl, 1 << LOG_N)
        outs = [pyoracle.keyswitch_shard(c, d, _a(evk_b), _a(evk_a), self.qs, self.ps, DNUM, limb0,
                                         limb0 + nl) for c, d in zip(ca, da)]
        k0 = np.stack([o[0] for o in outs]).astype(np.uint64).reshape(d2_own.shape)
        k1 = np.stack([o[1] for o in outs]).astype(np.uint64).reshape(d2_own.shape)
        return _t(k0), _t(k1)


def _data(seed=0):
    mods = pyoracle.gen_moduli(LOG_N, L + K)
    qs, ps = mods[:L], mods[L:]
    rng = np.random.default_rng(seed)
    n = 1 << LOG_N
    rand = lambda ms, lead: np.stack([rng.integers(0, q, lead + (n,), dtype=np.uint64) for q in ms],  # noqa: E731
                                     axis=len(lead))
    d2 = rand(qs, (2,))  # a batch of two ciphertexts sharing one key
    eb, ea = rand(mods, (DNUM,)), rand(mods, (DNUM,))
    a, b = rand(qs, (3, 2)), rand(qs, (3, 2))
    return qs, ps, d2, eb, ea, a, b


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        qs, ps, d2, eb, ea, a, b = _data()
        shard = LimbShard.from_env(L)
        eng = CpuEngine(qs, ps)
        rows = shard.evk_rows(K)
        k0, k1 = sharded_keyswitch(eng, _t(d2[:, shard.lo:shard.hi]), _t(eb[:, rows]),
                                   _t(ea[:, rows]), shard)
        d = sharded_hommult(eng, _t(a[:, :, shard.lo:shard.hi]), _t(b[:, :, shard.lo:shard.hi]),
                            shard)
        g0 = all_gather_limbs(k0, shard)
        g1 = all_gather_limbs(k1, shard)
        gd = all_gather_limbs(d, shard)
        if rank == 0:
            q.put((_a(g0).copy(), _a(g1).copy(), _a(gd).copy()))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3, 4])
def test_sharded_keyswitch_and_hommult_gloo(world):
    """world 3 over L = 4 limbs: uneven shards (2, 2, 0 limbs; the idle rank still joins the
    all-gather with a padded block)."""
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    g0, g1, d = q.get()
    qs, ps, d2, eb, ea, a, b = _data()
    for i in range(2):
        r0, r1 = coracle.keyswitch(d2[i], eb, ea, qs, ps, DNUM)
        assert (g0[i] == r0).all() and (g1[i] == r1).all()
    assert (d == coracle.hommult(a, b, qs)).all()


def test_limb_shard_ranges():
    s = LimbShard(16, 8, 3)
    assert (s.lo, s.hi, s.nlimbs, s.width) == (6, 8, 2, 2)
    assert s.evk_rows(4) == [6, 7, 16, 17, 18, 19]
    # uneven: ceil(L / G) per rank, the remainder on the last ranks
    assert [(LimbShard(10, 4, r).lo, LimbShard(10, 4, r).nlimbs) for r in range(4)] == \
        [(0, 3), (3, 3), (6, 3), (9, 1)]
    assert [LimbShard(10, 8, r).nlimbs for r in range(8)] == [2, 2, 2, 2, 2, 0, 0, 0]
    with pytest.raises(ValueError):
        LimbShard(10, 4, 4)
    x = torch.arange(16 * 3).reshape(16, 3)
    assert s.own(x).tolist() == x[6:8].tolist()


def test_ranked_layout_round_trip():
    """Rank-major padded blocks (what gather_ranked's all-gather produces) map back to limb
    order exactly, for even and uneven shards; a single rank's gather is its padded block."""
    from fhecore.dist import gather_ranked

    x = torch.arange(2 * 10 * 4).reshape(2, 10, 4)
    assert (gather_ranked(x, LimbShard(10, 1, 0)) == x[None]).all()
    for world in (2, 3, 4, 8):
        sh0 = LimbShard(10, world, 0)
        buf = torch.zeros(world, 2, sh0.width, 4, dtype=x.dtype)
        for r in range(world):  # single-process emulation of the all-gather
            sh = LimbShard(10, world, r)
            buf[r, :, :sh.nlimbs] = sh.own(x)
        assert (ranked_to_limbs(buf, sh0) == x).all()


def test_single_rank_shard_is_identity():
    qs, ps, d2, eb, ea, a, b = _data(1)
    shard = LimbShard(L, 1, 0)
    eng = CpuEngine(qs, ps)
    k0, k1 = sharded_keyswitch(eng, _t(d2), _t(eb), _t(ea), shard)
    for i in range(2):
        r0, r1 = coracle.keyswitch(d2[i], eb, ea, qs, ps, DNUM)
        assert (_a(k0)[i] == r0).all() and (_a(k1)[i] == r1).all()


def _hybrid_worker(rank, world, groups, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fhecore.dist import hybrid_groups, hybrid_plan

        qs, ps, d2, eb, ea, _, _ = _data(seed=3)
        B = d2.shape[0]
        grp = hybrid_groups(world, groups)  # every rank creates every group's sub-group
        h = hybrid_plan(L, LOG_N, world, groups, rank, B, 1)
        shard = LimbShard(L, h.g, h.shard)
        assert shard.world == (dist.get_world_size(grp) if grp is not None else 1)
        eng = CpuEngine(qs, ps)
        rows = shard.evk_rows(K)
        mine = d2[h.batch0:h.batch0 + h.batch, shard.lo:shard.hi]
        k0, k1 = sharded_keyswitch(eng, _t(mine), _t(eb[:, rows]), _t(ea[:, rows]), shard,
                                   group=grp)
        q.put((rank, h.batch0, h.batch, shard.lo, shard.hi, _a(k0).copy(), _a(k1).copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,groups", [(4, 2), (2, 2)])
def test_hybrid_partition_gloo(world, groups):
    """The hybrid partition's torch.distributed form (fhe_dist_hybrid): `groups`
    ciphertext groups of world / groups limb shards, the all-gather inside each group's
    sub-group only; every rank's rows equal the oracle key-switch of its group's ciphertexts."""
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_hybrid_worker, args=(r, world, groups, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    qs, ps, d2, eb, ea, _, _ = _data(seed=3)
    refs = [coracle.keyswitch(d2[i], eb, ea, qs, ps, DNUM) for i in range(d2.shape[0])]
    covered = np.zeros((d2.shape[0], L), dtype=int)
    for _ in range(world):
        rank, b0, bn, lo, hi, k0, k1 = q.get()
        for i in range(bn):
            assert (k0[i] == refs[b0 + i][0][lo:hi]).all(), (rank, i)
            assert (k1[i] == refs[b0 + i][1][lo:hi]).all(), (rank, i)
            covered[b0 + i, lo:hi] += 1
    assert (covered == 1).all()


def test_hybrid_groups_must_divide_world():
    """fhecore.dist.hybrid_groups refuses a group count that does not divide the ranks (before any
    collective), and needs no process group for one rank or one-rank groups."""
    from fhecore.dist import hybrid_groups

    with pytest.raises(ValueError):
        hybrid_groups(8, 3)
    with pytest.raises(ValueError):
        hybrid_groups(4, 0)
    assert hybrid_groups(1, 1) is None
    assert hybrid_groups(4, 4) is None  # g = 1: every group is one rank
