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
        # a deferred round's (active, local pass-2 status, global qr, c1): persistent buffers, so a HIP graph
        # that captures a deferred round commits what the previous replay left here
        self.p_active = torch.zeros_like(e._active)
        self.p_status = torch.zeros_like(e.status)
        self.p_qr = torch.zeros_like(e.qr)
        self.p_c1 = torch.zeros_like(e.c1)


def _pack(qr: torch.Tensor, prev: torch.Tensor, cur: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    """[B, N + 2 * world] all-reduce buffer: the qr partials, then this rank's previous-round (deferred)
    pass-2 status and this round's pass-1 status in its own slots (zeros elsewhere).  A SUM of it is the
    global qr AND every rank's status codes exactly (x + 0 = x; codes < 64 are exact in fp32), so one
    collective replaces the separate status MAX reductions."""
    B, N = qr.shape
    buf = torch.zeros((B, N + 2 * world), dtype=qr.dtype, device=qr.device)
    buf[:, :N] = qr
    buf[:, N + rank] = prev.to(qr.dtype)
    buf[:, N + world + rank] = cur.to(qr.dtype)
    return buf


def _commit(e, sh, active: torch.Tensor, status: torch.Tensor, qr=None, c1=None) -> None:
    """Shadow outputs -> state for the instances whose (globally reduced) status is OK, then the epilogue.
    (A deferred round passes its own qr / c1: the next round's pass 1 rewrites those shadows.)"""
    qr = sh.qr if qr is None else qr
    c1 = sh.c1 if c1 is None else c1
    ok1 = ((active != 0) & (status == int(Status.OK)))[:, None]
    e.consensus.copy_(torch.where(ok1, sh.consensus, e.consensus))
    e.skew.copy_(torch.where(ok1, sh.skew, e.skew))
    e.kurt.copy_(torch.where(ok1, sh.kurt, e.kurt))
    e.rel.copy_(torch.where(ok1, sh.rel, e.rel))
    e.qr.copy_(torch.where(ok1, qr, e.qr))
    e.reliable.copy_(torch.where(ok1, sh.reliable, e.reliable))
    e.c1.copy_(torch.where(ok1, c1, e.c1))
    e._ops.round_epilogue(active, status, e.rel, e.consensus_active, e.touched, e.metrics_fx)


def run_round_sharded(engine, d_global: int, group=None, world: int = 1, defer: bool = False) -> None:
    """Consensus round for an engine holding a column shard of every instance.

    Collectives per round (world > 1): one SUM of the packed buffer (qr partials + status slots, _pack),
    then one status MAX after pass 2 -- or, with ``defer=True``, none: the round's pass-2 verdicts ride
    in the NEXT round's packed buffer, which commits this round before its own pass 2 (one collective
    per round).  A deferred round is pending until that next round or :func:`flush_sharded`; its
    instances' ``touched`` flags are cleared at once (the epilogue clears them anyway), so the next
    round's selection is unchanged."""
    e = engine
    sh = getattr(e, "_dshard_shadow", None)
    if sh is None:
        sh = e._dshard_shadow = _Shadow(e)
    rank = dist.get_rank(group) if world > 1 else 0
    if getattr(e, "_dshard_pending", None) is not None and getattr(e, "_dshard_pending_rows", None):
        # a deferred transactional round still holds saved rows: its verdict and restore come before this
        # round's pass 1 reads the rows (an instance selected again -- e.g. by touched.fill_(1) -- would
        # otherwise compute from rows that are rolled back right after).  Without saved rows
        # the verdict keeps riding in this round's packed buffer.
        flush_sharded(e, group, world)
    pend = getattr(e, "_dshard_pending", None)
    e._ops.round_prologue(e.n_active, e.touched, e.N, True, e._active)
    lg = e.cfg.legacy
    if e.mode == "fast":
        mx = float(e.cfg.unconstrained_max_spread)
        w = e.work()                                     # window kernel: pass 1 -> pass 2 state
        head = (e.values, e._active, e.D, e.cfg.n_failing_oracles, e.cfg.constrained, mx, sh.c1)

        def half(mode):
            e._ops.fast_round(*head, sh.consensus, sh.skew, sh.kurt, sh.rel, sh.qr, sh.reliable, e.status,
                              e.wave_hint, mode, d_global, lg, w)
    else:
        if world > MAX_EXACT_SHARDS:
            # each shard's int64 qr partial is bounded below 2^58 (status.hpp kExactQrPartialMax); the SUM
            # all-reduce of more than 32 of them could wrap int64 and silently change the rank mask
            raise ValueError(f"exact D-sharding supports at most {MAX_EXACT_SHARDS} shards (got {world})")
        head = (e.values, e._active, e.cfg.n_failing_oracles, e.cfg.constrained, e.cfg.max_spread_wsad, sh.c1)

        def half(mode):
            e._ops.exact_round(*head, sh.consensus, sh.skew, sh.kurt, sh.rel, sh.qr, sh.reliable, e.status, lg,
                               mode, d_global)
    # pass 1: local c1 + qr partials into the shadow qr (the committed qr stays intact); status = this
    # shard's pass-1 verdict (exact: a partial past 2^58 fails the round)
    half(1)
    if world > 1:
        prev = pend[1] if pend is not None else torch.zeros_like(e.status)
        buf = _pack(sh.qr, prev, e.status, rank, world)
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
        N = sh.qr.shape[1]
        sh.qr.copy_(buf[:, :N])
        if pend is not None:     # the previous (deferred) round: every rank's pass-2 verdict, then commit
            pst = buf[:, N:N + world].amax(1).to(e.status.dtype)
            _commit(e, sh, pend[0], pst, pend[2], pend[3])
            # (no saved rows can be pending here: they were flushed before pass 1)
            e._dshard_pending_rows = None
            e._dshard_pending = pend = None
        e.status.copy_(buf[:, N + world:].amax(1).to(e.status.dtype))
    # pass 2 from the global qr on the instances every shard passed, into the shadow outputs
    half(2)
    if defer and world > 1:
        # (active, local pass-2 status, global qr, c1): pass 1 of the next round rewrites the qr / c1 shadows.
        # Transactional fast engines keep the round's update batches (saved rows) until the verdict: the
        # next apply_updates flushes first (engine.apply_updates -> pipeline_join -> flush_sharded), so a
        # reverted instance's rows, enabled flags and n_active are restored before any new row lands.
        if e.mode == "fast":
            from ..engine import _PendingBatches
            e._dshard_pending_rows, e._pending = e._pending, _PendingBatches(e)
        sh.p_active.copy_(e._active)
        sh.p_status.copy_(e.status)
        sh.p_qr.copy_(sh.qr)
        sh.p_c1.copy_(sh.c1)
        e._dshard_pending = (sh.p_active, sh.p_status, sh.p_qr, sh.p_c1)
        e._dshard_ctx = (group, world)   # engine.pipeline_join (every state reader) commits it
        e.touched.zero_()
        e.rounds += 1
        return
    if world > 1:
        dist.all_reduce(e.status, op=dist.ReduceOp.MAX, group=group)
    _commit(e, sh, e._active, e.status)
    if e.mode == "fast":
        e._restore_pending()    # every rank rolls back its column slice of the reverted instances' updates
    e.rounds += 1


def flush_sharded(engine, group=None, world: int = 1) -> None:
    """Commit a deferred sharded round (one status MAX all-reduce); no-op when none is pending."""
    e = engine
    pend = getattr(e, "_dshard_pending", None)
    if pend is None:
        return
    st = pend[1].clone()
    if world > 1:
        dist.all_reduce(st, op=dist.ReduceOp.MAX, group=group)
    _commit(e, e._dshard_shadow, pend[0], st, pend[2], pend[3])
    e.status.copy_(st)
    rows = getattr(e, "_dshard_pending_rows", None)
    if rows:   # every rank rolls back its column slice of the reverted instances' update batches
        rows.restore(st, pend[0])
    e._dshard_pending_rows = None
    e._dshard_pending = None
