"""Data parallelism over independent consensus instances (one process per GPU, RCCL over xGMI).

The reference has no distribution at all: one contract, transactions serialised by the Starknet
sequencer (survey §2.5/§2.6).  Instances are independent, so the MI355X design shards them:
rank r owns global instances [r*B, (r+1)*B) and steady-state steps need no communication.
Collectives are only used for (a) the per-step health metrics, one tiny all-reduce batched over all
local instances (xGMI is point-to-point, 7 links; a few bytes are latency-bound, so ONE call per
step, never one per instance), and (b) reporting: all-gather of per-instance summaries.

Backend: ``torch.distributed`` "nccl" (= RCCL on ROCm) on GPUs; "gloo" for the CPU test rig.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.distributed as dist

from ..status import Status


class DataParallelConsensus:
    def __init__(self, engine, rank: int = 0, world: int = 1, group=None):
        self.engine = engine
        self.rank = rank
        self.world = world
        self.group = group
        dev = engine.device
        # [rel2 sum over committed rounds, committed rounds, processed rounds, reverted rounds]
        self._fx = torch.zeros(4, dtype=torch.int64, device=dev)
        self._global = torch.zeros(4, dtype=torch.float64, device=dev)
        # fixed-point scale of the rel2 sum (fast: 2^-32, exact: 1e-6); the other counters are integers
        fx_scale = (2.0 ** -32) if getattr(engine, "mode", "fast") == "fast" else 1e-6
        self._scale = torch.tensor([fx_scale, 1.0, 1.0, 1.0], dtype=torch.float64, device=dev)

    # -- sharding ---------------------------------------------------------------------------------
    def global_ids(self) -> torch.Tensor:
        B = self.engine.B
        return torch.arange(self.rank * B, (self.rank + 1) * B, device=self.engine.device)

    def owner(self, global_id: int) -> int:
        return global_id // self.engine.B

    # -- metrics ----------------------------------------------------------------------------------
    def accumulate(self) -> None:
        """Kept for API compatibility: every round's epilogue kernel already folds its outcome into
        ``engine.metrics_fx`` (integer counters, device-only, capturable)."""

    def reduce(self) -> torch.Tensor:
        """One all-reduce of the integer counters (RCCL on GPU), then float64 metrics:
        [sum rel2 of committed rounds, committed, processed, reverted]."""
        e = self.engine
        e.pipeline_join()
        src = e.metrics_fx
        if self.world > 1:
            self._fx.copy_(src)
            dist.all_reduce(self._fx, op=dist.ReduceOp.SUM, group=self.group)
            src = self._fx
        # one elementwise kernel: int64 counters -> float64, rel2 sum scaled (the 4-element tail of a step)
        torch.mul(src, self._scale, out=self._global)
        return self._global

    def step_metrics(self) -> None:
        self.accumulate()
        self.reduce()

    def global_ok_fraction(self) -> float:
        g = self.reduce()
        return float(g[1] / g[2]) if float(g[2]) > 0 else 0.0

    def mean_rel2(self) -> float:
        g = self.reduce()
        return float(g[0] / g[1]) if float(g[1]) > 0 else 0.0

    # -- reporting --------------------------------------------------------------------------------
    def all_gather_summaries(self, k: int = 4) -> Optional[Dict[str, torch.Tensor]]:
        """Gather [world*B] summaries (first k consensus components, rel, status) to every rank."""
        e = self.engine
        e.pipeline_join()
        local = torch.cat([e.consensus[:, :k].double(), e.rel.double(), e.status[:, None].double()], dim=1)
        if self.world == 1:
            full = local
        else:
            parts = [torch.empty_like(local) for _ in range(self.world)]
            dist.all_gather(parts, local.contiguous(), group=self.group)
            full = torch.cat(parts, 0)
        return dict(consensus=full[:, :k], rel=full[:, k:k + 2], status=full[:, k + 2].to(torch.int32))
