"""CPU checks of fhe_keyswitch_dist's placement plan (gpu-fhe_amd/csrc/dist.cpp, exported as
fhe_dist_plan_*; host code, no GPU): for every rank count G = 1..8 with even and uneven limb
splits, every batch / chunk combination the bench and tests use, the plan that the native
multi-GPU key-switch follows must
  * give each Q-limb to exactly one rank (contiguous windows in rank order);
  * cut the batch into non-empty chunks that cover it exactly;
  * put every (rank, ciphertext, own limb) row that a rank's INTT writes at exactly the offset
    the key-switch kernels read that limb from (CAll::ranked, the same code path), inside that
    rank's block of that chunk, with no two rows overlapping and everything inside the gather
    region the workspace size is computed from;
  * be the same on every rank (the all-gather's block geometry must agree).
The single-device G-rank execution of the same plan is tests/test_gpu_dist.py (loopback)."""
import ctypes
import itertools

import pytest

from fhecore import _capi
from fhecore.dist import LimbShard, dist_plan

BAD = (1 << 64) - 1
LOG_N = 4  # row length 16: offsets stay small, the arithmetic is the same for any N


def rows_of(p, n):
    lib = _capi.load()
    out = []
    for b in range(p.batch):
        for j in range(p.nlimbs):
            w = lib.fhe_dist_plan_send_word(ctypes.byref(p), b, j)
            assert w != BAD
            out.append((b, p.limb0 + j, w))
    return out


@pytest.mark.parametrize("G", range(1, 9))
@pytest.mark.parametrize("L", [1, 3, 8, 10, 16, 17, 32])
def test_plan_places_every_row_where_it_is_read(G, L):
    lib = _capi.load()
    n = 1 << LOG_N
    for batch, chunks in itertools.product([1, 3, 5, 16], [0, 1, 2, 3, 4, 8, 16, 40]):
        plans = [dist_plan(L, LOG_N, G, r, batch, chunks) for r in range(G)]
        geo = {(p.width, p.chunks, p.chunk_batch, p.block_words, p.gather_words) for p in plans}
        assert len(geo) == 1, "ranks disagree on the gather geometry"
        p0 = plans[0]
        assert p0.width == -(-L // G)
        assert 1 <= p0.chunks <= 16 and p0.chunks <= batch
        assert p0.block_words == p0.chunk_batch * p0.width * n
        assert p0.gather_words == p0.chunks * G * p0.block_words
        # limb windows: LimbShard's, contiguous, disjoint, covering [0, L)
        lo = 0
        for r, p in enumerate(plans):
            sh = LimbShard(L, G, r)
            assert (p.limb0, p.nlimbs) == (sh.lo, sh.nlimbs)
            assert p.limb0 == lo or p.nlimbs == 0
            lo += p.nlimbs
        assert lo == L
        # chunks cover the batch exactly, none empty
        seen = []
        for k in range(p0.chunks):
            b0, bn = ctypes.c_uint32(), ctypes.c_uint32()
            _capi.check(lib.fhe_dist_plan_chunk(ctypes.byref(p0), k, ctypes.byref(b0),
                                                ctypes.byref(bn)), "chunk")
            assert bn.value >= 1 and b0.value == len(seen)
            seen += list(range(b0.value, b0.value + bn.value))
        assert seen == list(range(batch))
        assert lib.fhe_dist_plan_chunk(ctypes.byref(p0), p0.chunks, ctypes.byref(b0),
                                       ctypes.byref(bn)) == -1
        # rows: written where read, inside the writer's block of its chunk, disjoint
        spans = []
        for r, p in enumerate(plans):
            for b, l, w in rows_of(p, n):
                k = b // p.chunk_batch
                assert lib.fhe_dist_plan_read_word(ctypes.byref(p0), b, l) == w
                # every rank reads the same place
                assert lib.fhe_dist_plan_read_word(ctypes.byref(plans[-1]), b, l) == w
                blk0 = (k * G + r) * p.block_words
                assert blk0 <= w and w + n <= blk0 + p.block_words
                # the INTT writes a chunk's rows at poly stride width N from its first row
                b0 = k * p.chunk_batch
                first = lib.fhe_dist_plan_send_word(ctypes.byref(p), b0, 0)
                assert w == first + ((b - b0) * p.width + (l - p.limb0)) * n
                spans.append((w, w + n))
        spans.sort()
        assert len(spans) == batch * L
        assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:])), "rows overlap"
        assert spans[-1][1] <= p0.gather_words
        # out-of-range arguments are refused, not wrapped
        assert lib.fhe_dist_plan_read_word(ctypes.byref(p0), batch, 0) == BAD
        assert lib.fhe_dist_plan_read_word(ctypes.byref(p0), 0, L) == BAD
        assert lib.fhe_dist_plan_send_word(ctypes.byref(p0), 0, p0.nlimbs) == BAD


def test_plan_rejects_bad_ranks():
    lib = _capi.load()
    p = _capi.DistPlan()
    assert lib.fhe_dist_plan_make(ctypes.byref(p), 16, 16, 4, 4, 1, 0) == -1
    assert lib.fhe_dist_plan_make(ctypes.byref(p), 16, 16, 0, 0, 1, 0) == -1
    assert lib.fhe_dist_plan_make(ctypes.byref(p), 0, 16, 1, 0, 1, 0) == -1


def test_bench_default_plans():
    """The shapes bench.py's key-switch leg runs: configs[3] (L = 16) at G = 1, 2, 4, 8 with the
    default chunking (1 chunk at G = 1, 4 above) and batch 16."""
    for G in (1, 2, 4, 8):
        chunks = 1 if G == 1 else 4
        p = dist_plan(16, 16, G, G - 1, 16, chunks)
        assert (p.nlimbs, p.chunks, p.chunk_batch) == (16 // G, chunks, 16 // chunks)
        assert p.block_words * 8 == 16 // chunks * (16 // G) * 8 << 16


@pytest.mark.parametrize("G", range(1, 9))
@pytest.mark.parametrize("L", [1, 7, 16, 17])
def test_hybrid_partition_plan(G, L):
    """fhe_dist_hybrid_make for every divisor `groups` of G: rank r is limb shard r % g of group
    r // g; the groups' ciphertext ranges partition the job's batch in rank order; each rank's plan
    is exactly the limb plan of its group (g ranks, its ciphertexts); within a group the shards
    cover every limb once.  Bad shapes (groups not dividing G, rank out of range) are refused."""
    from fhecore.dist import hybrid_plan

    lib = _capi.load()
    for groups in [d for d in range(1, G + 1) if G % d == 0]:
        g = G // groups
        for batch, chunks in itertools.product([0, 1, 3, 5, 16, 32], [0, 1, 4]):
            hs = [hybrid_plan(L, LOG_N, G, groups, r, batch, chunks) for r in range(G)]
            start = 0
            for k in range(groups):
                grp = hs[k * g:(k + 1) * g]
                assert {(h.batch0, h.batch) for h in grp} == {(grp[0].batch0, grp[0].batch)}
                assert grp[0].batch0 == min(start, batch)
                start = grp[0].batch0 + grp[0].batch
                lo = 0
                for s, h in enumerate(grp):
                    assert (h.ranks, h.groups, h.g, h.group, h.shard) == (G, groups, g, k, s)
                    ref = dist_plan(L, LOG_N, g, s, h.batch, chunks)
                    for f, _ in _capi.DistPlan._fields_:
                        assert getattr(h.plan, f) == getattr(ref, f), f
                    assert h.plan.limb0 == lo or h.plan.nlimbs == 0
                    lo += h.plan.nlimbs
                assert lo == L
            assert start == batch
    bad = _capi.DistHybrid()
    for args in ((G, G + 1, 0), (G, 0, 0), (G, 1, G)):
        if args[1] and G % args[1] == 0 and args[2] < G:
            continue
        assert lib.fhe_dist_hybrid_make(ctypes.byref(bad), L, LOG_N, args[0], args[1], args[2],
                                        4, 0) == -1
