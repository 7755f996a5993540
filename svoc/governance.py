"""Admin replacement voting for B instances (contract/src/contract.cairo:547-580, 661-738).

Device state (see csrc/include/svoc/governance.hpp): admin / oracle addresses as 4 x int64 limbs,
the A x A vote matrix column-packed into one uint64 per receiving admin, and one optional
proposition per admin.  ``submit`` (a list of action tuples) and ``submit_batch`` (action tensors) run
actions with per-instance sequential semantics: the batch is sorted stably by instance on the device
and one launch applies each instance's run of actions in order (the CPU engine processes the list in
order).

Reference quirks kept: ``update_proposition(None)`` does not clear votes (§2.8-7); a proposal needs
a vote call to be applied even with required_majority = 1 (§2.8-9); a majority on a None
proposition reverts (§2.8-7); replacement keeps the oracle's value / enabled / reliable flags
(§2.8-6).  Hardening (documented deviation): ``which_admin >= n_admins`` reverts with
WRONG_ADMIN_INDEX instead of writing an unchecked storage key (§2.8-8).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import ops as svops
from .codec import address_to_limbs, limbs_to_address
from .status import ConsensusRevert, Status

PROPOSE, VOTE = 0, 1


class Governance:
    def __init__(self, B: int, n_admins: int, n_oracles: int, device, enable: bool = True, majority: int = 2):
        if n_admins > 64:
            raise ValueError("at most 64 admins")
        self.B, self.A, self.N = B, n_admins, n_oracles
        self.enable = bool(enable)
        self.majority = int(majority)
        self.device = torch.device(device)
        d = self.device
        self.admins = torch.zeros(B, n_admins, 4, dtype=torch.int64, device=d)
        self.oracle_addr = torch.zeros(B, n_oracles, 4, dtype=torch.int64, device=d)
        self.votes = torch.zeros(B, n_admins, dtype=torch.int64, device=d)   # uint64 bit columns
        self.prop_tag = torch.zeros(B, n_admins, dtype=torch.int8, device=d)
        self.prop_idx = torch.zeros(B, n_admins, dtype=torch.int32, device=d)
        self.prop_addr = torch.zeros(B, n_admins, 4, dtype=torch.int64, device=d)
        self._ops = svops.ops()
        self._oracle_cache: Optional[List[Dict[int, int]]] = None
        self.replacements = 0

    # ------------------------------------------------------------------ addresses
    def set_addresses(self, admins: Sequence[Sequence[int]], oracles: Sequence[Sequence[int]]) -> None:
        """admins[b] / oracles[b]: address ints per instance (or one list broadcast to all)."""
        def pack(lst, n):
            if lst and isinstance(lst[0], (list, tuple)):
                t = torch.tensor([[address_to_limbs(int(a)) for a in r] for r in lst], dtype=torch.int64)
            else:   # one list for every instance: [n, 4] broadcast (no B-long host list)
                t = torch.tensor([address_to_limbs(int(a)) for a in lst], dtype=torch.int64)[None].expand(self.B, -1, -1)
            assert t.shape[1] == n
            return t.to(self.device)
        if self.A:
            self.admins.copy_(pack(list(admins), self.A))
        self.oracle_addr.copy_(pack(list(oracles), self.N))
        self._oracle_cache = None

    def oracle_index(self, b: int, addr: int) -> Optional[int]:
        """find_oracle_index (contract.cairo:505-518) with a host-side hash map cache."""
        if self._oracle_cache is None:
            host = self.oracle_addr.cpu().tolist()
            self._oracle_cache = [{limbs_to_address(l): i for i, l in reversed(list(enumerate(r)))} for r in host]
        return self._oracle_cache[b].get(int(addr))

    def admin_index(self, b: int, addr: int) -> Optional[int]:
        for i, l in enumerate(self.admins[b].cpu().tolist()):
            if limbs_to_address(l) == int(addr):
                return i
        return None

    def oracle_list(self, b: int) -> List[int]:
        return [limbs_to_address(l) for l in self.oracle_addr[b].cpu().tolist()]

    def admin_list(self, b: int) -> List[int]:
        return [limbs_to_address(l) for l in self.admins[b].cpu().tolist()]

    # ------------------------------------------------------------------ actions
    def submit(self, actions: Sequence[Tuple]) -> Tuple[torch.Tensor, torch.Tensor]:
        """actions: ("propose", inst, caller, proposition | None) or ("vote", inst, caller, which, support).

        Returns (status[K], applied[K]) in submission order."""
        K = len(actions)
        inst = np.zeros(K, np.int64); kind = np.zeros(K, np.int32); a0 = np.zeros(K, np.int32)
        a1 = np.zeros(K, np.int64); caller = np.zeros((K, 4), np.int64); addr = np.zeros((K, 4), np.int64)
        for k, act in enumerate(actions):
            inst[k] = act[1]
            caller[k] = address_to_limbs(int(act[2]))
            if act[0] == "propose":
                kind[k] = PROPOSE
                if act[3] is not None:
                    a0[k] = 1
                    a1[k] = int(act[3][0])
                    addr[k] = address_to_limbs(int(act[3][1]))
            elif act[0] == "vote":
                kind[k] = VOTE
                a0[k] = int(act[3]) if 0 <= int(act[3]) < 2 ** 31 else -1
                a1[k] = 1 if act[4] else 0
            else:
                raise ValueError(act[0])
        d = self.device
        t = lambda x, dt: torch.as_tensor(x, dtype=dt).to(d)  # noqa: E731
        status, applied = self.submit_batch(t(inst, torch.int64), t(caller, torch.int64), t(kind, torch.int32),
                                            t(a0, torch.int32), t(a1, torch.int64), t(addr, torch.int64))
        if K and bool(applied.any()):
            self.replacements += int(applied.sum())
        return status, applied

    def submit_batch(self, inst: torch.Tensor, caller: torch.Tensor, kind: torch.Tensor, arg0: torch.Tensor,
                     arg1: torch.Tensor, addr: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """Device path for an ordered batch of K actions (tensors, submission order; any number per instance):
        inst [K] int64, caller [K, 4] int64 limbs, kind [K] int32 (PROPOSE / VOTE), arg0 [K] int32 (propose:
        1 = Some / 0 = None; vote: which_admin), arg1 [K] int64 (propose: oracle index; vote: support 0/1),
        addr [K, 4] int64 limbs (propose: new address).  Each instance's actions apply in submission order
        (contract.cairo:661-738 transactions, serialised per contract): on the GPU the batch is sorted stably by
        instance on the device and ONE launch applies every instance's run (no host wave split, no sync);
        the CPU applies the list in order.  Returns (status [K] int32, applied [K] uint8), submission order."""
        d = self.device
        K = int(inst.numel())
        c = lambda x, dt: x.to(d, dt).contiguous()  # noqa: E731
        inst, caller, kind, arg0, arg1, addr = (c(inst, torch.int64), c(caller, torch.int64).reshape(K, 4),
                                                c(kind, torch.int32), c(arg0, torch.int32), c(arg1, torch.int64),
                                                c(addr, torch.int64).reshape(K, 4))
        status = torch.empty(K, dtype=torch.int32, device=d)
        applied = torch.zeros(K, dtype=torch.uint8, device=d)
        if K == 0:
            return status, applied
        order = (torch.sort(inst, stable=True).indices if d.type != "cpu"
                 else torch.arange(K, dtype=torch.int64))
        self._ops.governance_seq(self.admins, self.oracle_addr, self.votes, self.prop_tag, self.prop_idx,
                                 self.prop_addr, inst, caller, kind, arg0, arg1, addr, self.enable, self.majority,
                                 order, status, applied)
        self._oracle_cache = None
        return status, applied

    def submit_tensors(self, inst, caller, kind, arg0, arg1, addr):
        """Low-level device path: one action per instance (instances must be unique), no host work."""
        K = inst.numel()
        st = torch.empty(K, dtype=torch.int32, device=self.device)
        ap = torch.zeros(K, dtype=torch.uint8, device=self.device)
        self._ops.governance(self.admins, self.oracle_addr, self.votes, self.prop_tag, self.prop_idx,
                             self.prop_addr, inst, caller, kind, arg0, arg1, addr, self.enable, self.majority, st, ap)
        self._oracle_cache = None
        return st, ap

    # ------------------------------------------------------------------ getters
    def propositions(self, b: int) -> List[Optional[Tuple[int, int]]]:
        tag = self.prop_tag[b].cpu().tolist()
        idx = self.prop_idx[b].cpu().tolist()
        addr = self.prop_addr[b].cpu().tolist()
        return [(idx[i], limbs_to_address(addr[i])) if tag[i] else None for i in range(self.A)]

    def vote_matrix(self, b: int) -> List[List[bool]]:
        """vote_matrix[emitter][receiver] (contract.cairo:94)."""
        cols = [int(v) & 0xFFFFFFFFFFFFFFFF for v in self.votes[b].cpu().tolist()]
        return [[bool((cols[r] >> e) & 1) for r in range(self.A)] for e in range(self.A)]

    def check(self, st: int) -> None:
        if st != Status.OK:
            raise ConsensusRevert(Status(st))
