"""D-sharding ("tensor parallel" for one huge instance): each rank owns a column slice.

Medians, consensus and moments are column-local (math.cairo:152-165, 365-398); only the per-oracle
quadratic risk qr_i = sum_d (x_id - c1_d)^2 (math.cairo:225-238) couples columns.  So a round is:

    pass 1 on the local columns  -> c1 (local), qr partials [B, N]      (HIP kernel, mode=1)
    all_reduce(SUM) of the qr partials over the shard group            (RCCL over xGMI; B*N*4 bytes)
    pass 2 on the local columns from the global qr                      (HIP kernel, mode=2)

Every rank then computes the identical rank mask from the identical reduced qr (deterministic,
no broadcast needed).  The constrained reliability divides by the GLOBAL dimension (rel_dim).
One all-reduce per round, batched over all B local instances -- sized for xGMI, where a few-KB
message is latency-bound (survey §5.8 b).

Per-instance atomicity across shards (survey §2.6; contract.cairo:588-603 reverts the whole tx): the
zero-variance check of pass 2 sees only the local columns, so pass 2 writes into shadow outputs, the
[B] status words are all-reduced (MAX: any shard's failure code wins, OK = 0), and only instances
whose reduced status is OK commit -- on every rank, or on none.

Exact (wsad) engines split the same way (the i128 kernel / CPU golden engine, modes 1 and 2): qr is
a sum of per-column integer terms (each truncated on its own, math.cairo:225-238), so the int64
all-reduce of the shards' partials IS the contract's qr and a successful sharded round is bit-identical
to the unsharded one.  Differences, by construction: a shard's partial must stay below 2^58 (else the
round reverts with OVERFLOW; the contract's i128 sum would only overflow near 2^127), and a reverted
round reports the largest of the shards' codes, not the contract's first error in evaluation order.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..status import Status


# exact mode: a shard's qr partial is < 2^58, so the int64 sum of at most 2^5 partials cannot wrap
MAX_EXACT_SHARDS = 32


def shard_bounds(D: int, rank: int, world: int):
    per = (D + world - 1) // world
    lo = min(D, rank * per)
    return lo, min(D, lo + per)


class _Shadow:
    """Scratch outputs of one sharded round (allocated once per engine)."""

    def __init__(self, e):
        self.qr = torch.zeros_like(e.qr)
        self.c1 = torch.zeros_like(e.c1)
        self.consensus = torch.zeros_like(e.consensus)
        self.skew = torch.zeros_like(e.skew)
        self.kurt = torch.zeros_like(e.kurt)
        self.rel = torch.zeros_like(e.rel)
        self.reliable = torch.zeros_like(e.reliable)


def run_round_sharded(engine, d_global: int, group=None, world: int = 1) -> None:
    """Consensus round for an engine holding a column shard of every instance."""
    e = engine
    sh = getattr(e, "_dshard_shadow", None)
    if sh is None:
        sh = e._dshard_shadow = _Shadow(e)
    e._ops.round_prologue(e.n_active, e.touched, e.N, True, e._active)
    lg = e.cfg.legacy
    if e.mode == "fast":
        mx = float(e.cfg.unconstrained_max_spread)
        w = e.work()                                     # window kernel: pass 1 -> pass 2 state
        head = (e.values, e._active, e.D, e.cfg.n_failing_oracles, e.cfg.constrained, mx, sh.c1)
        # pass 1: local c1 + qr partials (into the shadow qr: the committed qr stays intact)
        e._ops.fast_round(*head, sh.consensus, sh.skew, sh.kurt, sh.rel, sh.qr, sh.reliable, e.status,
                          e.wave_hint, 1, d_global, lg, w)
        if world > 1:
            dist.all_reduce(sh.qr, op=dist.ReduceOp.SUM, group=group)
        # pass 2 from the global qr, into the shadow outputs; status = this shard's verdict
        e._ops.fast_round(*head, sh.consensus, sh.skew, sh.kurt, sh.rel, sh.qr, sh.reliable, e.status,
                          e.wave_hint, 2, d_global, lg, w)
    else:
        if world > MAX_EXACT_SHARDS:
            # each shard's int64 qr partial is bounded below 2^58 (status.hpp kExactQrPartialMax); the SUM
            # all-reduce of more than 32 of them could wrap int64 and silently change the rank mask
            raise ValueError(f"exact D-sharding supports at most {MAX_EXACT_SHARDS} shards (got {world})")
        head = (e.values, e._active, e.cfg.n_failing_oracles, e.cfg.constrained, e.cfg.max_spread_wsad, sh.c1)
        # first half: c1 + int64 qr partials; a shard that fails here (overflow) fails the round
        e._ops.exact_round(*head, sh.consensus, sh.skew, sh.kurt, sh.rel, sh.qr, sh.reliable, e.status, lg,
                           1, d_global)
        if world > 1:
            dist.all_reduce(sh.qr, op=dist.ReduceOp.SUM, group=group)
            dist.all_reduce(e.status, op=dist.ReduceOp.MAX, group=group)
        # second half on the instances every shard passed (the kernel skips non-OK statuses)
        e._ops.exact_round(*head, sh.consensus, sh.skew, sh.kurt, sh.rel, sh.qr, sh.reliable, e.status, lg,
                           2, d_global)
    if world > 1:
        dist.all_reduce(e.status, op=dist.ReduceOp.MAX, group=group)
    ok = (e._active != 0) & (e.status == int(Status.OK))
    ok1 = ok[:, None]
    e.consensus.copy_(torch.where(ok1, sh.consensus, e.consensus))
    e.skew.copy_(torch.where(ok1, sh.skew, e.skew))
    e.kurt.copy_(torch.where(ok1, sh.kurt, e.kurt))
    e.rel.copy_(torch.where(ok1, sh.rel, e.rel))
    e.qr.copy_(torch.where(ok1, sh.qr, e.qr))
    e.reliable.copy_(torch.where(ok1, sh.reliable, e.reliable))
    e.c1.copy_(torch.where(ok1, sh.c1, e.c1))
    e._ops.round_epilogue(e._active, e.status, e.rel, e.consensus_active, e.touched, e.metrics_fx)
    e.rounds += 1
