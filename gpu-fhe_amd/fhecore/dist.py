"""RNS-limb sharding across GPUs: one process per GPU, torch.distributed over RCCL.

Every coefficient-wise op, NTT/INTT and the HomMult tensor is independent per RNS limb, so rank r
of G simply owns a contiguous block of Q-limbs and runs those -- no collective.  The hybrid
key-switch has exactly one exchange: each rank INTTs its own limbs of d2, one all-gather makes the
full coefficient-form d2 available everywhere (ModUp needs every limb of a digit), and each rank
then finishes ModUp / NTT / inner product / ModDown for its own Q-limbs plus a replicated copy of
the K special limbs (so ModDown needs no second collective).  Outputs stay limb-sharded and
concatenate to the single-device result bit for bit.

Shards: rank r owns Q-limbs [r c, min((r + 1) c, L)), c = ceil(L / G) -- any L and G (the last
ranks may own fewer limbs, or none).  The all-gather output stays rank-major, [G, batch, c, N]
with the short blocks padded (gather_ranked), and the key-switch reads that layout directly
(Context.keyswitch_shard(..., ranks=G)): no reorder copy.

Two drivers run the same algorithm:
  * sharded_keyswitch -- torch.distributed all-gather + the engine's local step; written against
    an "engine" (``intt`` / ``intt_`` and ``keyswitch_shard``), so fhecore.Context (HIP) and the
    CPU restatement of the gloo tests share it;
  * RcclComm + Context.keyswitch_dist -- the whole exchange inside libfhecore
    (fhe_keyswitch_dist: its own RCCL communicator and stream, chunked so each chunk's transfer
    overlaps the previous chunk's key-switch).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass(frozen=True)
class LimbShard:
    """Rank `rank` of `world` owns Q-limbs [lo, hi) of an L-limb modulus chain."""

    L: int
    world: int
    rank: int

    def __post_init__(self):
        if self.world < 1 or not 0 <= self.rank < self.world or self.L < 1:
            raise ValueError("bad rank/world")

    @property
    def width(self) -> int:
        """Limbs per rank block (the last blocks may hold fewer): ceil(L / world)."""
        return -(-self.L // self.world)

    @property
    def lo(self) -> int:
        return min(self.L, self.rank * self.width)

    @property
    def hi(self) -> int:
        return min(self.L, self.lo + self.width)

    @property
    def nlimbs(self) -> int:
        return self.hi - self.lo

    def own(self, x, limb_dim: int = -2):
        """This rank's slice of a full-limb tensor/array along `limb_dim`."""
        idx = [slice(None)] * x.dim() if hasattr(x, "dim") else [slice(None)] * x.ndim
        idx[limb_dim] = slice(self.lo, self.hi)
        return x[tuple(idx)]

    def evk_rows(self, K: int):
        """Row indices of an evk [dnum, L + K, N] this rank keeps: its Q-limbs, then all P-limbs."""
        return list(range(self.lo, self.hi)) + list(range(self.L, self.L + K))

    @classmethod
    def from_env(cls, L: int, group=None):
        if dist.is_available() and dist.is_initialized():
            return cls(L, dist.get_world_size(group), dist.get_rank(group))
        return cls(L, 1, 0)


def dist_plan(L: int, log_n: int, ranks: int, rank: int, batch: int, chunks: int = 0):
    """libfhecore's placement plan of fhe_keyswitch_dist for one rank (fhe_dist_plan_make; host
    only, no GPU needed): limb window, chunking and the gather region's geometry."""
    from ._capi import DistPlan, check, load

    p = DistPlan()
    check(load().fhe_dist_plan_make(ctypes.byref(p), L, log_n, ranks, rank, batch, chunks),
          "fhe_dist_plan_make")
    return p


def hybrid_plan(L: int, log_n: int, ranks: int, groups: int, rank: int, batch: int,
                chunks: int = 0):
    """The hybrid partition (fhe_dist_hybrid_make; host only): rank `rank` of `ranks` is limb shard
    rank % g of ciphertext group rank // g (g = ranks / groups), which key-switches the job's
    ciphertexts [batch0, batch0 + batch) among its g ranks (``plan``: its limb plan)."""
    from ._capi import DistHybrid, check, load

    h = DistHybrid()
    lib = load()
    if groups == 1 and not hasattr(lib, "fhe_dist_hybrid_make"):
        # an older A/B library (FHECORE_LIB): the limb-only plan is the whole job's
        h.ranks, h.groups, h.g, h.group, h.shard, h.batch0, h.batch = ranks, 1, ranks, 0, rank, 0, batch
        h.plan = dist_plan(L, log_n, ranks, rank, batch, chunks)
        return h
    check(lib.fhe_dist_hybrid_make(ctypes.byref(h), L, log_n, ranks, groups, rank, batch, chunks),
          "fhe_dist_hybrid_make")
    return h


def hybrid_groups(world: int, groups: int):
    """torch.distributed sub-groups of the hybrid partition: ranks [k g, (k + 1) g) for each
    ciphertext group k (every rank must call this, in the same order); returns this rank's group
    (None at world 1 or groups == world, where a group is one rank)."""
    if groups < 1 or world % groups:
        raise ValueError(f"{groups} ciphertext groups do not divide {world} ranks")
    g = world // groups
    if world == 1 or g == 1:
        return None
    mine = None
    me = dist.get_rank()
    for k in range(groups):
        ranks = list(range(k * g, (k + 1) * g))
        grp = dist.new_group(ranks=ranks)
        if me in ranks:
            mine = grp
    return mine


def gather_ranked(x_own, shard: LimbShard, group=None):
    """[..., nlimbs, N] per rank -> [world, batch, width, N] on every rank (batch = the flattened
    leading dims; blocks shorter than `width` padded): one all_gather_into_tensor, no reorder."""
    n = x_own.shape[-1]
    lead = 1
    for d in x_own.shape[:-2]:
        lead *= d
    x = x_own.reshape(lead, shard.nlimbs, n)
    if shard.nlimbs != shard.width:
        pad = torch.zeros(lead, shard.width, n, dtype=x.dtype, device=x.device)
        pad[:, :shard.nlimbs] = x
        x = pad
    x = x.contiguous()
    if shard.world == 1:
        return x.reshape(1, lead, shard.width, n)
    if x.is_cuda and dist.get_backend(group) == "gloo":
        # gloo gathers host tensors only: the multi-rank rehearsal on one GPU (several ranks
        # sharing a device, where RCCL refuses duplicate GPUs) stages through the host
        buf = torch.empty((shard.world * lead, shard.width, n), dtype=x.dtype)
        dist.all_gather_into_tensor(buf, x.cpu(), group=group)
        return buf.to(x.device).view(shard.world, lead, shard.width, n)
    buf = torch.empty((shard.world * lead, shard.width, n), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(buf, x, group=group)
    return buf.view(shard.world, lead, shard.width, n)


def ranked_to_limbs(buf, shard: LimbShard):
    """[world, batch, width, N] (gather_ranked) -> [batch, L, N] in limb order."""
    w, lead, width, n = buf.shape
    return buf.permute(1, 0, 2, 3).reshape(lead, w * width, n)[:, :shard.L].contiguous()


def all_gather_limbs(x_own, shard: LimbShard, group=None):
    """[..., nlimbs, N] per rank -> [..., L, N] on every rank (rank order = limb order)."""
    full = ranked_to_limbs(gather_ranked(x_own, shard, group), shard)
    return full.reshape(tuple(x_own.shape[:-2]) + (shard.L, x_own.shape[-1]))


def sharded_hommult(engine, a_own, b_own, shard: LimbShard, out=None, workspace=None):
    """ct x ct tensor on this rank's limbs: a_own/b_own [batch, 2, nlimbs, N]. No collective."""
    return engine.hommult(a_own, b_own, out=out, limb0=shard.lo, workspace=workspace)


def sharded_keyswitch(engine, d2_own, evk_b_own, evk_a_own, shard: LimbShard, group=None):
    """Hybrid key-switch of this rank's limbs (SURVEY.md §8a', §8e).

    d2_own: [..., nlimbs, N] NTT form (limbs [lo, hi), any leading batch shape); evk_*_own:
    [dnum, nlimbs + K, N] (own Q-limbs then the K P-limbs, see LimbShard.evk_rows), one key for the
    batch.  Returns (ks0_own, ks1_own) shaped like d2_own, NTT form."""
    if hasattr(engine, "intt"):  # out of place: no copy of d2 (the HIP Context)
        c_own = engine.intt(d2_own, limb0=shard.lo)
    else:
        c_own = d2_own.clone()
        engine.intt_(c_own, limb0=shard.lo)
    c_ranked = gather_ranked(c_own, shard, group)  # the only collective of the whole path
    return engine.keyswitch_shard(c_ranked, d2_own, evk_b_own, evk_a_own, shard.lo,
                                  ranks=shard.world)


class RcclComm:
    """libfhecore's own RCCL communicator for fhe_keyswitch_dist (include/fhecore.h).  Rank 0
    makes the unique id; torch.distributed (any backend) carries it to the others.  One per
    process/GPU; every rank of `group` must construct it together."""

    def __init__(self, device: int = None, group=None, local: bool = False):
        """local: a one-rank communicator whatever the process group (a hybrid partition's
        ciphertext group of one rank, fhe_dist_hybrid with g = 1)."""
        from ._capi import check, load

        lib = load()
        if dist.is_available() and dist.is_initialized() and not local:
            self.world, self.rank = dist.get_world_size(group), dist.get_rank(group)
        else:
            self.world, self.rank = 1, 0
        self.device = torch.cuda.current_device() if device is None else int(device)
        uid = ctypes.create_string_buffer(128)
        if self.rank == 0:
            check(lib.fhe_comm_get_unique_id(uid), "fhe_comm_get_unique_id")
        if self.world > 1:
            box = [uid.raw if self.rank == 0 else None]
            dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group else 0,
                                       group=group)
            uid = ctypes.create_string_buffer(box[0], 128)
        self._c = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib.fhe_comm_create(ctypes.byref(self._c), uid, self.world, self.rank,
                                      self.device), "fhe_comm_create")

    @property
    def handle(self):
        return self._c

    def gather_ms(self):
        """Per-chunk all-gather durations (ms, on the communicator's stream) of the last
        keyswitch_dist call (fhe_comm_gather_ms; waits for those gathers)."""
        from ._capi import check, load

        ms = (ctypes.c_float * 16)()
        cnt = ctypes.c_uint32()
        check(load().fhe_comm_gather_ms(self._c, ms, 16, ctypes.byref(cnt)), "fhe_comm_gather_ms")
        return [float(v) for v in ms[:cnt.value]]

    def shard(self, L: int) -> LimbShard:
        return LimbShard(L, self.world, self.rank)

    def close(self):
        if getattr(self, "_c", None) and self._c.value:
            from ._capi import load

            load().fhe_comm_destroy(self._c)
            self._c = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass
