"""Streaming update sources and queues.

* :class:`SyntheticUpdateStream`: a device-resident pool of synthetic prediction batches (the
  stochastic oracles of client/oracle_scheduler.py:73-92 at scale): every step, ``U`` distinct oracles
  of every instance publish a new prediction; failing oracles (a fixed random subset per instance,
  survey §5.3 fault injection) publish U(0,1)^D noise, honest ones Beta(a, a) draws.  The pool is
  generated once and cycled, so the timed loop measures the engine, not the RNG.
* :class:`UpdateQueue`: host-side accumulation of (instance, oracle, prediction) triples from any
  producer (CLI, sentiment path, tests) flushed to the engine as one batched step.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch

from .models.oracle_gen import failing_mask


class SyntheticUpdateStream:
    def __init__(self, B: int, N: int, D: int, U: int, f: int, pool: int = 2, device="cuda", seed: int = 0,
                 a: float = 20.0, dtype=torch.bfloat16, failing: Optional[torch.Tensor] = None):
        self.B, self.N, self.D, self.U, self.pool = B, N, D, U, pool
        dev = torch.device(device)
        g = torch.Generator(device=dev).manual_seed(seed)
        # [B, N] fixed per instance: the engine's own failing set (ConsensusEngine.failing_mask) when given,
        # so a state and its stream agree on which f oracles fail (an extra noisy oracle per update would
        # stay among the reliable rows)
        self.failing = (failing.to(dev, torch.bool) if failing is not None else failing_mask(B, N, f, g, dev))
        self.batches: List[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]] = []
        inst = torch.arange(B, device=dev).repeat_interleave(U)
        for _ in range(pool):
            orc = torch.rand(B, N, generator=g, device=dev).argsort(1)[:, :U].reshape(-1)
            fail = self.failing[inst, orc]
            vals = torch.empty(B * U, D, dtype=dtype, device=dev)
            chunk = max(1, (1 << 26) // max(1, D))            # bound the fp32 temporaries
            for s in range(0, B * U, chunk):
                e = min(B * U, s + chunk)
                ga = torch._standard_gamma(torch.full((e - s, D), a, device=dev), generator=g)
                gb = torch._standard_gamma(torch.full((e - s, D), a, device=dev), generator=g)
                hon = ga / (ga + gb)
                uni = torch.rand(e - s, D, generator=g, device=dev)
                x = torch.where(fail[s:e, None], uni, hon)
                vals[s:e] = (x.double() * 1_000_000).to(torch.int64) if dtype == torch.int64 else x.to(dtype)
            self.batches.append((inst.contiguous(), orc.contiguous(), vals))

    def batch(self, i: int):
        return self.batches[i % self.pool]


class UpdateQueue:
    def __init__(self):
        self.inst: List[int] = []
        self.orc: List[int] = []
        self.vals: List[torch.Tensor] = []

    def push(self, instance: int, oracle: int, prediction) -> None:
        self.inst.append(int(instance))
        self.orc.append(int(oracle))
        self.vals.append(torch.as_tensor(prediction))

    def __len__(self) -> int:
        return len(self.inst)

    def flush(self, engine) -> Optional[torch.Tensor]:
        if not self.inst:
            return None
        st = engine.step(torch.tensor(self.inst), torch.tensor(self.orc), torch.stack(self.vals))
        self.inst, self.orc, self.vals = [], [], []
        return st


def governance_stream(B: int, n_oracles: int, admin_addresses, device, seed: int = 0, frac: float = 0.01,
                      pairs: int = 4):
    """Synthetic admin-replacement traffic (contract.cairo:661-738 -> :547-580), ``2 * pairs``
    batches for ``Governance.submit_tensors``: batch 2k = a proposition by admin 0 on ``frac`` of the
    instances (replace a random oracle by a fresh address), batch 2k+1 = admin 1's supporting vote on
    the SAME instances -- with majority 2 every pair completes a replacement.  Cycle them in order."""
    from .codec import address_to_limbs
    dev = torch.device(device)
    K = max(1, int(B * frac))
    g = torch.Generator(device=dev).manual_seed(7919 + seed)
    a0 = torch.tensor(address_to_limbs(int(admin_addresses[0])), device=dev).expand(K, 4).contiguous()
    a1 = torch.tensor(address_to_limbs(int(admin_addresses[1])), device=dev).expand(K, 4).contiguous()
    out = []
    for _ in range(pairs):
        inst = torch.randperm(B, generator=g, device=dev)[:K].contiguous()
        which = torch.randint(0, n_oracles, (K,), generator=g, device=dev)
        addr = torch.randint(10 ** 6, 10 ** 15, (K, 4), generator=g, device=dev)
        out.append((inst, a0, torch.zeros(K, dtype=torch.int32, device=dev),
                    torch.ones(K, dtype=torch.int32, device=dev), which, addr))          # propose(Some(idx, addr))
        out.append((inst, a1, torch.ones(K, dtype=torch.int32, device=dev),
                    torch.zeros(K, dtype=torch.int32, device=dev), torch.ones(K, dtype=torch.int64, device=dev),
                    addr))                                                              # vote(admin 0, yes)
    return out

