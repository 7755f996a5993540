"""Consensus configuration: the reference constructor calldata (contract.cairo:235-265) as a dataclass.

Field names follow the contract: ``enable_oracle_replacement``, ``required_majority``,
``n_failing_oracles``, ``constrained``, ``unconstrained_max_spread``, ``dimension``.  Real-unit
floats are used by the fast engine; the exact engine converts with the wsad codec (1e6 scale).
"""
from __future__ import annotations

import dataclasses
import json
from typing import Any, Dict, Optional

WSAD = 1_000_000


@dataclasses.dataclass
class ConsensusConfig:
    n_oracles: int = 7
    dimension: int = 6
    n_failing_oracles: int = 2
    constrained: bool = True
    unconstrained_max_spread: float = 1.0     # real units (wsad / 1e6)
    n_admins: int = 3
    required_majority: int = 2
    enable_oracle_replacement: bool = True
    # exact wsad value of the spread when it must round-trip bit for bit (set by the ABI facade)
    unconstrained_max_spread_wsad: Optional[int] = None
    # contract generation: "nds" = contract/src/contract.cairo (default); "nd_legacy" =
    # contract/obsolete/src/contract_nd.cairo; "1d_legacy" = contract_1d_constrained.cairo (D = 1,
    # constrained).  The obsolete ones compute no moments and no /D in the constrained reliability.
    variant: str = "nds"

    def validate(self) -> None:
        if self.n_oracles < 1 or self.dimension < 1:
            raise ValueError("n_oracles and dimension must be >= 1")
        if not (0 <= self.n_admins <= 64):
            raise ValueError("n_admins must be in [0, 64] (bit-packed vote rows)")
        # unconstrained_max_spread == 0 is accepted: like the contract, every round then reverts
        # with a division by zero (contract.cairo:367)
        if self.variant not in ("nds", "nd_legacy", "1d_legacy"):
            raise ValueError(f"unknown contract variant {self.variant!r}")
        if self.variant == "1d_legacy" and (self.dimension != 1 or not self.constrained):
            raise ValueError("the 1-D obsolete contract is constrained with dimension 1")

    @property
    def legacy(self) -> bool:
        """Obsolete-contract semantics (contract_nd.cairo:418,437): no /D, no moments."""
        return self.variant != "nds"

    @property
    def max_spread_wsad(self) -> int:
        if self.unconstrained_max_spread_wsad is not None:
            return int(self.unconstrained_max_spread_wsad)
        return int(round(self.unconstrained_max_spread * WSAD))

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "ConsensusConfig":
        return cls(**{k: v for k, v in d.items() if k in {f.name for f in dataclasses.fields(cls)}})

    def to_json(self) -> str:
        return json.dumps(self.to_dict())

    # deployed demo configuration (contract/README.md:43-61; client/common.py:8-9,31)
    @classmethod
    def deployed_demo(cls) -> "ConsensusConfig":
        return cls(n_oracles=7, dimension=6, n_failing_oracles=2, constrained=True, n_admins=3,
                   required_majority=2, enable_oracle_replacement=True)
