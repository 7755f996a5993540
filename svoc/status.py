"""Per-instance status codes shared by every engine (Python golden, C++ CPU, HIP kernels).

The reference is a Starknet contract: any failed assertion or arithmetic panic reverts the whole
transaction (``contract/src/contract.cairo:588-603``; survey §2.8-5).  A batched engine cannot raise
per instance, so each instance carries a status word instead.  A non-OK status on an update means
"this transaction reverted": the instance state is left exactly as it was before the update.

Keep in sync with ``csrc/include/svoc/status.hpp``.
"""
from __future__ import annotations

import enum


class Status(enum.IntEnum):
    OK = 0                    # round computed and committed
    NOT_ACTIVE = 1            # update stored, not every oracle has committed yet (contract.cairo:447-449)
    INTERVAL_INPUT = 2        # constrained input outside [0, WSAD] ('interval error', math.cairo:298-310)
    NOT_ORACLE = 3            # caller is not an oracle ('not an oracle', contract.cairo:596)
    DIV_BY_ZERO = 4           # I128Div by zero: sqrt(1), zero variance z-score, max_spread = 0, ...
    INDEX_OOB = 5             # array access out of bounds (smooth_median on < 2 values)
    RELIABILITY_INTERVAL = 6  # reliability outside [0, WSAD] (contract.cairo:467,488 / 395,420)
    OVERFLOW = 7              # i128 overflow in an intermediate product or sum
    USIZE_UNDERFLOW = 8       # usize underflow (n_failing > n_oracles, contract.cairo:346)
    FELT_RANGE = 9            # felt252 -> i128 conversion failed (value outside i128)
    # governance (contract.cairo:661-738)
    REPLACEMENT_DISABLED = 16
    NOT_ADMIN = 17
    WRONG_ORACLE_INDEX = 18
    ALREADY_ORACLE = 19
    UNWRAP_NONE = 20          # majority reached on a None proposition (contract.cairo:572)
    WRONG_ADMIN_INDEX = 21    # which_admin >= n_admins (hardening; see governance.py)
    # fast-mode codes (float path); like every non-OK status they revert the round: no output moves
    ZERO_VARIANCE = 32        # a reliable column has sigma == 0 (exact mode reports DIV_BY_ZERO)
    TOO_FEW_RELIABLE = 33     # R < 4: kurtosis denominator (n-2)(n-3) == 0 (exact: DIV_BY_ZERO)
    NON_FINITE = 34           # unconstrained float update holding NaN / inf (no wsad counterpart)

    @property
    def is_revert(self) -> bool:
        return self not in (Status.OK, Status.NOT_ACTIVE)


class ConsensusRevert(Exception):
    """Raised by the golden Python model where Cairo would panic (transaction revert)."""

    def __init__(self, status: Status, msg: str = ""):
        super().__init__(f"{status.name}: {msg}" if msg else status.name)
        self.status = Status(status)
