"""RNS-limb sharding across GPUs: one process per GPU, torch.distributed over RCCL.

Every coefficient-wise op, NTT/INTT and the HomMult tensor is independent per RNS limb, so rank r
of G simply owns a contiguous block of Q-limbs and runs those -- no collective.  The hybrid
key-switch has exactly one exchange: each rank INTTs its own limbs of d2, one all-gather makes the
full coefficient-form d2 available everywhere (ModUp needs every limb of a digit), and each rank
then finishes ModUp / NTT / inner product / ModDown for its own Q-limbs plus a replicated copy of
the K special limbs (so ModDown needs no second collective).  Outputs stay limb-sharded and
concatenate to the single-device result bit for bit.

The orchestration is written against an "engine" with two methods -- ``intt_(t, limb0)`` and
``keyswitch_shard(c_all, d2_own, evk_b, evk_a, limb0)``, plus an optional out-of-place
``intt(t, limb0)`` that saves the copy of d2 -- so fhecore.Context (the HIP path) and a CPU
restatement used by the gloo tests run the same code.
"""
from __future__ import annotations

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
        if self.world < 1 or not 0 <= self.rank < self.world:
            raise ValueError("bad rank/world")
        if self.L % self.world:
            raise ValueError(f"L = {self.L} limbs do not divide evenly over {self.world} ranks")

    @property
    def nlimbs(self) -> int:
        return self.L // self.world

    @property
    def lo(self) -> int:
        return self.rank * self.nlimbs

    @property
    def hi(self) -> int:
        return self.lo + self.nlimbs

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


def all_gather_limbs(x_own, shard: LimbShard, group=None):
    """[..., nlimbs, N] per rank -> [..., L, N] on every rank (rank order = limb order).  One
    all_gather_into_tensor into a [world, ..., nlimbs, N] buffer, then a limb-major reorder."""
    if shard.world == 1:
        return x_own.contiguous()
    flat = (shard.world * x_own.shape[0],) + tuple(x_own.shape[1:])
    buf = torch.empty(flat, dtype=x_own.dtype, device=x_own.device)
    dist.all_gather_into_tensor(buf, x_own.contiguous(), group=group)
    if x_own.dim() == 2:
        return buf  # [world * nlimbs, N] is already limb order
    buf = buf.view((shard.world,) + tuple(x_own.shape))
    lead = x_own.dim() - 2
    perm = list(range(1, lead + 1)) + [0, lead + 1, lead + 2]
    return buf.permute(perm).reshape(tuple(x_own.shape[:-2]) + (shard.L, x_own.shape[-1])).contiguous()


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
    c_all = all_gather_limbs(c_own, shard, group)  # the only collective of the whole path
    return engine.keyswitch_shard(c_all, d2_own, evk_b_own, evk_a_own, shard.lo)
