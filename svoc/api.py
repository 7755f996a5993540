"""Contract-compatible public API.

:class:`ConsensusService` = B independent contracts on one device (engine + governance + addresses).
:class:`OracleConsensus` = one contract with the reference ABI (``IOracleConsensusNDS``,
contract/src/contract.cairo:4-35): felt252 values in and out, ``caller`` arguments instead of
``get_caller_address()``, and :class:`svoc.status.ConsensusRevert` where the contract would revert.
North-star aliases: ``get_consensus()`` and ``get_reliability()``.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch

from .codec import as_wsad, felt_to_i128, i128_to_felt, wsad_tensor_to_felts
from .config import WSAD, ConsensusConfig
from .engine import ConsensusEngine
from .governance import Governance
from .status import ConsensusRevert, Status


class ConsensusService:
    """B contracts sharing one configuration. ``mode='exact'`` is bit-compatible with the contract."""

    def __init__(self, cfg: ConsensusConfig, batch: int, admins, oracles, device="cpu", mode: str = "exact",
                 storage=None):
        self.cfg = cfg
        self.engine = ConsensusEngine(cfg, batch, device=device, mode=mode, storage=storage)
        self.gov = Governance(batch, cfg.n_admins, cfg.n_oracles, device, cfg.enable_oracle_replacement,
                              cfg.required_majority)
        self.gov.set_addresses(admins, oracles)
        self.B = batch

    # ---- writes --------------------------------------------------------------------------------
    def update_predictions(self, items: Sequence[Tuple[int, int, Sequence]]) -> List[Status]:
        """items: (instance, caller_address, prediction).  Predictions are wsad ints (exact mode)
        or floats (fast mode).  Returns one status per item (reverts do not raise)."""
        inst, orc, vals, pre = [], [], [], []
        for k, (b, caller, pred) in enumerate(items):
            if len(pred) != self.cfg.dimension:
                raise ValueError("prediction length != dimension")
            if self.cfg.constrained:  # interval check precedes the caller lookup (contract.cairo:590-596)
                hi = WSAD if self.engine.mode == "exact" else 1.0
                if any(not (0 <= x <= hi) for x in pred):
                    pre.append((k, Status.INTERVAL_INPUT))
                    continue
            o = self.gov.oracle_index(int(b), caller) if 0 <= int(b) < self.B else None
            if o is None:
                pre.append((k, Status.NOT_ORACLE))       # 'not an oracle' (contract.cairo:596)
                continue
            inst.append(int(b)); orc.append(o); vals.append(list(pred))
        out: List[Status] = [Status.OK] * len(items)
        for k, st in pre:
            out[k] = st
        if inst:
            dt = torch.int64 if self.engine.mode == "exact" else torch.float32
            st = self.engine.step(torch.tensor(inst), torch.tensor(orc), torch.tensor(vals, dtype=dt))
            it = iter(st.cpu().tolist())
            for k in range(len(items)):
                if all(k != p for p, _ in pre):
                    out[k] = Status(next(it))
        return out

    def governance(self, actions) -> Tuple[List[Status], List[bool]]:
        """update_proposition / vote_for_a_proposition transactions (contract.cairo:661-738).  ``actions``: a list
        of ("propose", inst, caller, (oracle_idx, new_address) | None) / ("vote", inst, caller, which_admin,
        support) tuples -> (statuses, applied) lists; or a mapping of action tensors (``inst``, ``caller``,
        ``kind``, ``arg0``, ``arg1``, ``addr``: see :meth:`Governance.submit_batch`) -> (status [K], applied [K])
        device tensors, with no host work (one device sort + one launch)."""
        if isinstance(actions, dict):
            return self.governance_batch(**actions)
        st, ap = self.gov.submit(actions)
        return [Status(s) for s in st.cpu().tolist()], [bool(a) for a in ap.cpu().tolist()]

    def governance_batch(self, inst, caller, kind, arg0, arg1, addr) -> Tuple[torch.Tensor, torch.Tensor]:
        """Tensor form of :meth:`governance` (any number of actions per instance, submission order per
        instance): status [K] int32 (svoc.status.Status codes) and applied [K] uint8, on the device."""
        return self.gov.submit_batch(inst, caller, kind, arg0, arg1, addr)

    def handle(self, b: int) -> "OracleConsensus":
        return OracleConsensus._from_service(self, b)


class OracleConsensus:
    """One ``OracleConsensusNDS`` contract (constructor: contract.cairo:235-265)."""

    def __init__(self, admins: Sequence[int], enable_oracle_replacement: bool, required_majority: int,
                 n_failing_oracles: int, constrained: bool, unconstrained_max_spread: int, dimension: int,
                 oracles: Sequence[int], device="cpu", mode: str = "exact", storage=None):
        ms = felt_to_i128(int(unconstrained_max_spread))
        cfg = ConsensusConfig(n_oracles=len(oracles), dimension=dimension, n_failing_oracles=n_failing_oracles,
                              constrained=bool(constrained), unconstrained_max_spread=ms / WSAD,
                              n_admins=len(admins), required_majority=required_majority,
                              enable_oracle_replacement=bool(enable_oracle_replacement),
                              unconstrained_max_spread_wsad=ms)
        self._max_spread_wsad = ms
        self._svc = ConsensusService(cfg, 1, list(admins), list(oracles), device=device, mode=mode, storage=storage)
        self._b = 0

    @classmethod
    def _from_service(cls, svc: ConsensusService, b: int) -> "OracleConsensus":
        obj = cls.__new__(cls)
        obj._svc, obj._b = svc, b
        obj._max_spread_wsad = svc.cfg.max_spread_wsad
        return obj

    @property
    def engine(self) -> ConsensusEngine:
        return self._svc.engine

    def _raise(self, st) -> None:
        if Status(st).is_revert:
            raise ConsensusRevert(Status(st))

    # ---- writes (ABI) ----------------------------------------------------------------------------
    def update_prediction(self, caller: int, prediction: Sequence[int]) -> Status:
        """``update_prediction(FeltVector)`` (contract.cairo:588-603). Returns OK / NOT_ACTIVE."""
        vals = as_wsad(prediction)
        e = self.engine
        pred = vals if e.mode == "exact" else [v / WSAD for v in vals]
        st = self._svc.update_predictions([(self._b, caller, pred)])[0]
        self._raise(st)
        return st

    def update_proposition(self, caller: int, proposition: Optional[Tuple[int, int]]) -> None:
        st, _ = self._svc.governance([("propose", self._b, caller, proposition)])
        self._raise(st[0])

    def vote_for_a_proposition(self, caller: int, which_admin: int, support_his_proposition: bool) -> bool:
        st, ap = self._svc.governance([("vote", self._b, caller, which_admin, support_his_proposition)])
        self._raise(st[0])
        return ap[0]

    # ---- reads (ABI) -----------------------------------------------------------------------------
    def _out(self, t: torch.Tensor) -> List[int]:
        """Engine output row -> felts (fast mode converts floats to wsad by truncation)."""
        if self.engine.mode == "exact":
            return wsad_tensor_to_felts(t)
        return [i128_to_felt(int(x)) for x in torch.trunc(t.double() * WSAD).to(torch.int64).tolist()]

    def consensus_active(self) -> bool:
        return bool(self.engine.consensus_active[self._b])

    def get_consensus_value(self) -> List[int]:
        return self._out(self.engine.consensus[self._b])

    def get_first_pass_consensus_reliability(self) -> int:
        return self._out(self.engine.rel[self._b, :1])[0]

    def get_second_pass_consensus_reliability(self) -> int:
        return self._out(self.engine.rel[self._b, 1:])[0]

    def get_skewness(self) -> List[int]:
        return self._out(self.engine.skew[self._b])

    def get_kurtosis(self) -> List[int]:
        return self._out(self.engine.kurt[self._b])

    def get_admin_list(self) -> List[int]:
        return self._svc.gov.admin_list(self._b)

    def get_oracle_list(self) -> List[int]:
        return self._svc.gov.oracle_list(self._b)

    def get_oracle_value_list(self, caller: int):
        """Admin-only (contract.cairo:771-799): (address, felt vector, enabled, reliable) per oracle."""
        if self._svc.gov.admin_index(self._b, caller) is None:
            raise ConsensusRevert(Status.NOT_ADMIN, "not admin")
        vals, en, rel = self.engine.get_oracle_value_list(self._b)
        rows = [self._out(v) for v in vals]
        return [(a, r, bool(x), bool(y)) for a, r, x, y in
                zip(self.get_oracle_list(), rows, en.tolist(), rel.tolist())]

    def get_predictions_dimension(self) -> int:
        return self.engine.D

    def get_replacement_propositions(self):
        if not self._svc.gov.enable:
            raise ConsensusRevert(Status.REPLACEMENT_DISABLED, "replacement disabled")
        return self._svc.gov.propositions(self._b)

    def get_a_specific_proposition(self, which_admin: int):
        if not self._svc.gov.enable:
            raise ConsensusRevert(Status.REPLACEMENT_DISABLED, "replacement disabled")
        return self._svc.gov.propositions(self._b)[which_admin]

    # ---- north-star aliases ----------------------------------------------------------------------
    def get_consensus(self) -> List[int]:
        return self.get_consensus_value()

    def get_reliability(self) -> Tuple[int, int]:
        return self.get_first_pass_consensus_reliability(), self.get_second_pass_consensus_reliability()


class LegacyOracleConsensus(OracleConsensus):
    """The obsolete contracts' ABI (contract/obsolete/src/): ``contract_nd.cairo`` (``variant=
    "nd_legacy"``, WsadVector = i128 values in and out) and ``contract_1d_constrained.cairo``
    (``variant="1d_legacy"``, one i128 per oracle, constrained, dimension 1).

    Same state machine and governance as the current contract; the round differs as documented in
    :func:`svoc.reference.consensus_round` (``legacy=True``): no ``/D`` in the constrained
    reliability, no skewness / kurtosis (the getters do not exist in those ABIs).
    """

    def __init__(self, admins: Sequence[int], enable_oracle_replacement: bool, required_majority: int,
                 n_failing_oracles: int, constrained: bool, unconstrained_max_spread: int, dimension: int,
                 oracles: Sequence[int], device="cpu", mode: str = "exact", variant: str = "nd_legacy",
                 storage=None):
        if variant not in ("nd_legacy", "1d_legacy"):
            raise ValueError("variant must be 'nd_legacy' or '1d_legacy'")
        ms = int(unconstrained_max_spread)                     # i128 constructor argument
        cfg = ConsensusConfig(n_oracles=len(oracles), dimension=dimension, n_failing_oracles=n_failing_oracles,
                              constrained=bool(constrained), unconstrained_max_spread=ms / WSAD,
                              n_admins=len(admins), required_majority=required_majority,
                              enable_oracle_replacement=bool(enable_oracle_replacement),
                              unconstrained_max_spread_wsad=ms, variant=variant)
        cfg.validate()
        self._max_spread_wsad = ms
        self._svc = ConsensusService(cfg, 1, list(admins), list(oracles), device=device, mode=mode, storage=storage)
        self._b = 0
        self._scalar = variant == "1d_legacy"

    def _out(self, t: torch.Tensor) -> List[int]:
        if self.engine.mode == "exact":
            return [int(x) for x in t.tolist()]
        return [int(x) for x in torch.trunc(t.double() * WSAD).to(torch.int64).tolist()]

    def update_prediction(self, caller: int, prediction) -> Status:
        """``update_prediction(WsadVector)`` (contract_nd.cairo:538) / ``(i128)`` (1-D, :391)."""
        vals = [int(prediction)] if self._scalar else [int(v) for v in prediction]
        pred = vals if self.engine.mode == "exact" else [v / WSAD for v in vals]
        st = self._svc.update_predictions([(self._b, caller, pred)])[0]
        self._raise(st)
        return st

    def get_consensus_value(self):
        v = self._out(self.engine.consensus[self._b])
        return v[0] if self._scalar else v

    def get_oracle_value_list(self, caller: int):
        rows = super().get_oracle_value_list(caller)
        return [(a, (v[0] if self._scalar else v), e, r) for a, v, e, r in rows]

    def get_skewness(self):
        raise AttributeError("the obsolete contracts store no skewness")

    def get_kurtosis(self):
        raise AttributeError("the obsolete contracts store no kurtosis")
