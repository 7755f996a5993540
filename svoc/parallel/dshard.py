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
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..status import Status


def shard_bounds(D: int, rank: int, world: int):
    per = (D + world - 1) // world
    lo = min(D, rank * per)
    return lo, min(D, lo + per)


def run_round_sharded(engine, d_global: int, group=None, world: int = 1) -> None:
    """Consensus round for an engine holding a column shard of every instance."""
    if engine.mode != "fast":
        raise NotImplementedError("D-sharding is implemented for the fast (float) engine")
    e = engine
    e._ops.round_prologue(e.n_active, e.touched, e.N, True, e._active)
    mx = float(e.cfg.unconstrained_max_spread)
    args = (e.values, e._active, e.D, e.cfg.n_failing_oracles, e.cfg.constrained, mx, e.c1, e.consensus,
            e.skew, e.kurt, e.rel, e.qr, e.reliable, e.status, e.wave_hint)
    lg = e.cfg.legacy
    w = e.work()                                     # window kernel: pass 1 -> pass 2 state
    e._ops.fast_round(*args, 1, d_global, lg, w)   # pass 1: local c1 + qr partials
    if world > 1:
        dist.all_reduce(e.qr, op=dist.ReduceOp.SUM, group=group)
    e._ops.fast_round(*args, 2, d_global, lg, w)   # pass 2 from the global qr
    e._ops.round_epilogue(e._active, e.status, e.rel, e.consensus_active, e.touched, e.metrics_fx)
    e.rounds += 1
