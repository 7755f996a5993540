"""Exact golden model of the reference consensus contract (pure Python integers).

This is the semantic spec every other engine is tested against.  It reproduces the Cairo contract
bit for bit, including its quirks (survey §2.8):

* wsad fixed point: i128 scaled by 1e6 (``contract/src/signed_decimal.cairo:82-83``), with the
  *truncate-toward-zero* signed division ``I128Div`` (``signed_decimal.cairo:52-63``);
  ``wsad_mul`` adds HALF_WSAD before dividing whatever the sign (``:110-112``), ``wsad_div``
  adds ``b / 2`` (``:114-116``);
* Newton square root with the ``g == g2`` stop and a 50-iteration cap (``math.cairo:271-292``);
* ``smooth_median`` always averages ranks ``len/2 - 1`` and ``len/2`` -- the odd branch is dead
  (``math.cairo:113-126``, bug at ``:120``);
* ``IndexedMergeSort`` takes the right element on ties, i.e. the order is (value asc, index desc)
  (``sort.cairo:96-101``);
* pass-2 reliability is measured against the *pass-1* centre (``contract.cairo:414,484``);
* every Cairo panic (division by zero, i128 overflow, out-of-bounds, interval error) reverts the
  whole transaction -- modelled by :class:`svoc.status.ConsensusRevert` and a state rollback.

Nothing here is fast; it exists to pin semantics.  The batched engines live in C++/HIP.
"""
from __future__ import annotations

import copy
import dataclasses
from typing import Dict, List, Optional, Sequence, Tuple

from .status import ConsensusRevert, Status

WSAD = 1_000_000
HALF_WSAD = 500_000
I128_MIN = -(1 << 127)
I128_MAX = (1 << 127) - 1
MAX_SQRT_ITERATIONS = 50


# ----------------------------------------------------------------------------------------------
# L0: fixed point (signed_decimal.cairo)
# ----------------------------------------------------------------------------------------------

def chk(x: int) -> int:
    """i128 range check: Cairo's i128 arithmetic panics on overflow."""
    if x < I128_MIN or x > I128_MAX:
        raise ConsensusRevert(Status.OVERFLOW, "i128 overflow")
    return x


def idiv(a: int, b: int) -> int:
    """``I128Div`` (signed_decimal.cairo:52-63): |a| // |b| with the sign of a*b, truncating."""
    if b == 0:
        raise ConsensusRevert(Status.DIV_BY_ZERO, "division by zero")
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def wmul(a: int, b: int) -> int:
    """``wsad_mul`` (signed_decimal.cairo:110-112)."""
    return idiv(chk(chk(a * b) + HALF_WSAD), WSAD)


def wdiv(a: int, b: int) -> int:
    """``wsad_div`` (signed_decimal.cairo:114-116)."""
    return idiv(chk(chk(a * WSAD) + idiv(b, 2)), b)


def wsqrt(value: int) -> int:
    """Newton square root in wsad (math.cairo:271-292). ``wsqrt(1)`` divides by zero (g = 0)."""
    if value == 0:
        return 0
    g = idiv(value, 2)
    g2 = chk(g + WSAD)
    i = 0
    while True:
        if g == g2 or i == MAX_SQRT_ITERATIONS:
            return g
        n = wdiv(value, g)
        g2 = g
        g = idiv(chk(g + n), 2)
        i += 1


# ----------------------------------------------------------------------------------------------
# L1: statistics kernels (math.cairo, sort.cairo)
# ----------------------------------------------------------------------------------------------

def smooth_median(col: Sequence[int]) -> int:
    """math.cairo:113-126 -- mean of sorted[mid-1], sorted[mid] for every length."""
    n = len(col)
    if n == 0:
        raise ConsensusRevert(Status.USIZE_UNDERFLOW, "smooth_median on empty")
    if n == 1:
        raise ConsensusRevert(Status.INDEX_OOB, "smooth_median on one value")
    s = sorted(col)
    mid = n // 2
    return idiv(chk(s[mid - 1] + s[mid]), 2)


def find_index(value: int, col: Sequence[int]) -> int:
    """math.cairo:87-100: the first index holding ``value`` (linear scan; 'value not found' panics)."""
    for i, v in enumerate(col):
        if v == value:
            return i
    raise ConsensusRevert(Status.INDEX_OOB, "value not found")


def median_index(col: Sequence[int]) -> int:
    """math.cairo:102-106: sort a copy, take ``sorted[len / 2]``, then locate it in the ORIGINAL array
    by value -- with duplicates this is the first occurrence, not necessarily the element the sort
    moved there."""
    if not col:
        raise ConsensusRevert(Status.INDEX_OOB, "median on empty")
    return find_index(sorted(col)[len(col) // 2], col)


def median(col: Sequence[int]) -> int:
    """math.cairo:108-110: ``values[median_index(values)]`` (= sorted[len/2])."""
    return col[median_index(col)]


def average(col: Sequence[int]) -> int:
    """math.cairo:240-254: truncating Σ / len."""
    acc = 0
    for v in col:
        acc = chk(acc + v)
    return idiv(acc, len(col))


def quadratic_deviation(a: int, b: int) -> int:
    x = chk(a - b)
    return wmul(x, x)


def nd_quadratic_risk(rows: Sequence[Sequence[int]], center: Sequence[int]) -> List[int]:
    """math.cairo:225-238: one Σ_d wmul(x-c, x-c) per row."""
    out = []
    for row in rows:
        acc = 0
        for x, c in zip(row, center):
            acc = chk(acc + quadratic_deviation(x, c))
        out.append(acc)
    return out


def columns(rows: Sequence[Sequence[int]]) -> List[List[int]]:
    """``nd_array_split`` transpose (math.cairo:55-85)."""
    return [list(c) for c in zip(*rows)]


def indexed_sort(values: Sequence[int]) -> List[Tuple[int, int]]:
    """``IndexedMergeSort::sort`` (sort.cairo:9-103): ascending, ties -> higher index first."""
    order = sorted(range(len(values)), key=lambda i: (values[i], -i))
    return [(i, values[i]) for i in order]


def variance(col: Sequence[int], mean: int) -> int:
    """``nd_component_wise_variance`` for one column (math.cairo:208-222)."""
    return average([quadratic_deviation(x, mean) for x in col])


def skewness(col: Sequence[int], mean: int, var: int) -> int:
    """math.cairo:320-338."""
    n = len(col)
    sd = wsqrt(var)
    acc = 0
    for x in col:
        z = wdiv(chk(x - mean), sd)
        acc = chk(acc + wmul(wmul(z, z), z))
    return idiv(chk(acc * n), chk((n - 1) * (n - 2)))


def kurtosis(col: Sequence[int], mean: int, var: int) -> int:
    """math.cairo:340-363 (sample-adjusted excess kurtosis)."""
    n = len(col)
    sd = wsqrt(var)
    acc = 0
    for x in col:
        z = wdiv(chk(x - mean), sd)
        z2 = wmul(z, z)
        acc = chk(acc + wmul(z2, z2))
    term1 = idiv(chk(chk(acc * n) * (n + 1)), n - 1)
    term2 = chk(chk(chk(3 * WSAD * (n - 1)) * (n - 1)))
    return idiv(chk(term1 - term2), chk((n - 2) * (n - 3)))


def interval_check(v: int, status: Status = Status.RELIABILITY_INTERVAL) -> None:
    if not (0 <= v <= WSAD):
        raise ConsensusRevert(status, "interval error")


# ----------------------------------------------------------------------------------------------
# L2: one consensus round (contract.cairo:365-503)
# ----------------------------------------------------------------------------------------------

@dataclasses.dataclass
class RoundResult:
    c1: List[int]             # pass-1 smooth median (essence_first_pass)
    qr: List[int]             # pass-1 quadratic risk per oracle
    order: List[int]          # oracle indices sorted by (qr asc, idx desc)
    reliable: List[bool]
    consensus: List[int]
    rel1: int
    rel2: int
    skewness: List[int]
    kurtosis: List[int]


def constrained_reliability(mean_qr: int, dim: int) -> int:
    """contract.cairo:436-439: W - 2*sqrt(mean_qr / D)."""
    return chk(WSAD - chk(wsqrt(idiv(mean_qr, dim)) * 2))


def unconstrained_reliability(sd: int, max_spread: int) -> int:
    """contract.cairo:365-368: W - wdiv(min(ms, sd), ms)."""
    return chk(WSAD - wdiv(min(max_spread, sd), max_spread))


def consensus_round(values: Sequence[Sequence[int]], n_failing: int, constrained: bool,
                    max_spread: int = 0, legacy: bool = False) -> RoundResult:
    """Both passes of the reference algorithm on a full [N][D] table of wsad integers.

    Raises :class:`ConsensusRevert` wherever the contract would panic.  ``legacy`` selects the
    obsolete contracts (contract/obsolete/src/contract_nd.cairo:395-443, contract_1d_constrained.cairo:
    250-295): constrained reliability ``W - 2 sqrt(mean qr)`` without the ``/D``
    (contract_nd.cairo:418,437) and no skewness / kurtosis (returned as zeros, never reverting).
    """
    n = len(values)
    dim = 1 if legacy else len(values[0])
    # ---- pass 1 (contract.cairo:451-473 / 379-402)
    cols = columns(values)
    c1 = [smooth_median(c) for c in cols]
    qr = nd_quadratic_risk(values, c1)
    if constrained:
        rel1 = constrained_reliability(average(qr), dim)
    else:
        rel1 = unconstrained_reliability(wsqrt(average(qr)), max_spread)
    interval_check(rel1)
    ordered = indexed_sort(qr)
    if n_failing > n:
        raise ConsensusRevert(Status.USIZE_UNDERFLOW, "n_oracles - n_failing_oracles")
    threshold = n - n_failing
    reliable = [False] * n
    for rank, (idx, _) in enumerate(ordered):
        reliable[idx] = rank < threshold
    # ---- pass 2 (contract.cairo:474-502 / 404-433)
    rel_rows = [values[i] for i in range(n) if reliable[i]]
    rcols = columns(rel_rows) if rel_rows else [[] for _ in range(dim)]
    if constrained:
        consensus = [smooth_median(c) for c in rcols]
    else:
        consensus = [average(c) for c in rcols]
    qr2 = nd_quadratic_risk(rel_rows, c1)
    if constrained:
        rel2 = constrained_reliability(average(qr2), dim)
    else:
        rel2 = unconstrained_reliability(wsqrt(average(qr2)), max_spread)
    interval_check(rel2)
    if legacy:
        zeros = [0] * len(rcols)
        return RoundResult(c1, qr, [i for i, _ in ordered], reliable, consensus, rel1, rel2, zeros, list(zeros))
    means = [average(c) for c in rcols]
    variances = [variance(c, m) for c, m in zip(rcols, means)]
    skew = [skewness(c, m, v) for c, m, v in zip(rcols, means, variances)]
    kurt = [kurtosis(c, m, v) for c, m, v in zip(rcols, means, variances)]
    return RoundResult(c1, qr, [i for i, _ in ordered], reliable, consensus, rel1, rel2, skew, kurt)


# ----------------------------------------------------------------------------------------------
# L3/L4: the whole contract as a state machine, ABI names kept (contract.cairo:4-35, 586-831)
# ----------------------------------------------------------------------------------------------

@dataclasses.dataclass
class OracleInfo:
    address: int
    enabled: bool = False
    reliable: bool = True


class ReferenceContract:
    """Single-instance exact model of ``OracleConsensusNDS`` with transaction-revert semantics.

    ``caller`` arguments play the role of ``get_caller_address()``.  Every public mutator either
    commits fully or raises :class:`ConsensusRevert` leaving the state untouched.
    """

    def __init__(self, admins: Sequence[int], enable_oracle_replacement: bool,
                 required_majority: int, n_failing_oracles: int, constrained: bool,
                 unconstrained_max_spread: int, dimension: int, oracles: Sequence[int],
                 legacy: bool = False):
        # constructor, contract.cairo:235-265 (legacy: contract/obsolete/src/contract_nd.cairo)
        self.legacy = bool(legacy)
        self.dimension = dimension
        self.admins = list(admins)
        self.oracles = [OracleInfo(a) for a in oracles]
        self.values = [[0] * dimension for _ in oracles]
        self.n_active_oracles = 0
        self.enable_oracle_replacement = bool(enable_oracle_replacement)
        self.required_majority = required_majority
        self.n_failing_oracles = n_failing_oracles
        self.constrained = bool(constrained)
        self.unconstrained_max_spread = unconstrained_max_spread
        self.consensus_active_flag = False
        na = len(admins)
        self.vote_matrix = [[False] * na for _ in range(na)]
        self.propositions: List[Optional[Tuple[int, int]]] = [None] * na
        self.consensus_value = [0] * dimension
        self.rel1 = 0
        self.rel2 = 0
        self.skewness = [0] * dimension
        self.kurtosis = [0] * dimension
        self.last_round: Optional[RoundResult] = None

    # -- transactions -----------------------------------------------------------------------
    def _transaction(self, fn, *args):
        snapshot = copy.deepcopy(self.__dict__)
        try:
            return fn(*args)
        except ConsensusRevert:
            self.__dict__.clear()
            self.__dict__.update(snapshot)
            raise

    def update_prediction(self, caller: int, prediction: Sequence[int]) -> Status:
        """contract.cairo:588-603. Returns OK or NOT_ACTIVE; raises on revert."""
        return self._transaction(self._update_prediction, caller, list(prediction))

    def _update_prediction(self, caller, prediction):
        for v in prediction:
            chk(v)
        if len(prediction) != self.dimension:
            raise ValueError("prediction length != dimension")
        if self.constrained:
            for v in prediction:
                interval_check(v, Status.INTERVAL_INPUT)
        idx = self._find_oracle(caller)
        if idx is None:
            raise ConsensusRevert(Status.NOT_ORACLE, "not an oracle")
        info = self.oracles[idx]
        if not info.enabled:
            self.n_active_oracles += 1
        info.enabled = True
        self.values[idx] = list(prediction)
        if self.n_active_oracles != len(self.oracles):
            return Status.NOT_ACTIVE
        r = consensus_round(self.values, self.n_failing_oracles, self.constrained,
                            self.unconstrained_max_spread, self.legacy)
        for i, o in enumerate(self.oracles):
            o.reliable = r.reliable[i]
        self.consensus_value = r.consensus
        self.rel1, self.rel2 = r.rel1, r.rel2
        self.skewness, self.kurtosis = r.skewness, r.kurtosis
        self.consensus_active_flag = True
        self.last_round = r
        return Status.OK

    def update_proposition(self, caller: int, proposition: Optional[Tuple[int, int]]) -> None:
        """contract.cairo:661-717."""
        return self._transaction(self._update_proposition, caller, proposition)

    def _update_proposition(self, caller, proposition):
        if not self.enable_oracle_replacement:
            raise ConsensusRevert(Status.REPLACEMENT_DISABLED, "replacement disabled")
        a = self._find_admin(caller)
        if a is None:
            raise ConsensusRevert(Status.NOT_ADMIN, "not an admin")
        if proposition is None:
            self.propositions[a] = None          # votes are NOT cleared (survey §2.8-7)
            return
        old_idx, new_addr = proposition
        if not (0 <= old_idx < len(self.oracles)):
            raise ConsensusRevert(Status.WRONG_ORACLE_INDEX, "wrong old oracle index")
        if self._find_oracle(new_addr) is not None:
            raise ConsensusRevert(Status.ALREADY_ORACLE, "the oracle is already in the team")
        for i in range(len(self.admins)):
            self.vote_matrix[i][a] = False
        self.vote_matrix[a][a] = True
        self.propositions[a] = (old_idx, new_addr)

    def vote_for_a_proposition(self, caller: int, which_admin: int, support: bool) -> bool:
        """contract.cairo:721-738 (+ check_for_replacement :547-580). Returns True if applied."""
        return self._transaction(self._vote, caller, which_admin, support)

    def _vote(self, caller, which_admin, support):
        if not self.enable_oracle_replacement:
            raise ConsensusRevert(Status.REPLACEMENT_DISABLED, "replacement disabled")
        v = self._find_admin(caller)
        if v is None:
            raise ConsensusRevert(Status.NOT_ADMIN, "not an admin")
        if not (0 <= which_admin < len(self.admins)):
            # the contract writes an unchecked LegacyMap key (survey §2.8-8); we reject instead
            raise ConsensusRevert(Status.WRONG_ADMIN_INDEX, "which_admin out of range")
        self.vote_matrix[v][which_admin] = bool(support)
        n_votes = sum(1 for i in range(len(self.admins)) if self.vote_matrix[i][which_admin])
        if self.required_majority > n_votes:
            return False
        prop = self.propositions[which_admin]
        if prop is None:
            raise ConsensusRevert(Status.UNWRAP_NONE, "unwrap on None proposition")
        oracle_idx, new_addr = prop
        self.oracles[oracle_idx].address = new_addr   # value/enabled/reliable kept (§2.8-6)
        na = len(self.admins)
        self.propositions = [None] * na
        self.vote_matrix = [[False] * na for _ in range(na)]
        return True

    # -- lookups / getters (contract.cairo:505-540, 605-659, 740-830) -----------------------
    def _find_oracle(self, addr) -> Optional[int]:
        for i, o in enumerate(self.oracles):
            if o.address == addr:
                return i
        return None

    def _find_admin(self, addr) -> Optional[int]:
        for i, a in enumerate(self.admins):
            if a == addr:
                return i
        return None

    def consensus_active(self) -> bool:
        return self.consensus_active_flag

    def get_consensus_value(self) -> List[int]:
        return list(self.consensus_value)

    def get_first_pass_consensus_reliability(self) -> int:
        return self.rel1

    def get_second_pass_consensus_reliability(self) -> int:
        return self.rel2

    def get_skewness(self) -> List[int]:
        return list(self.skewness)

    def get_kurtosis(self) -> List[int]:
        return list(self.kurtosis)

    def get_admin_list(self) -> List[int]:
        return list(self.admins)

    def get_oracle_list(self) -> List[int]:
        return [o.address for o in self.oracles]

    def get_oracle_value_list(self, caller: int):
        if self._find_admin(caller) is None:
            raise ConsensusRevert(Status.NOT_ADMIN, "not admin")
        return [(o.address, list(v), o.enabled, o.reliable) for o, v in zip(self.oracles, self.values)]

    def get_predictions_dimension(self) -> int:
        return self.dimension

    def get_replacement_propositions(self):
        if not self.enable_oracle_replacement:
            raise ConsensusRevert(Status.REPLACEMENT_DISABLED, "replacement disabled")
        return list(self.propositions)

    def get_a_specific_proposition(self, which_admin: int):
        if not self.enable_oracle_replacement:
            raise ConsensusRevert(Status.REPLACEMENT_DISABLED, "replacement disabled")
        return self.propositions[which_admin]


def round_status(values, n_failing, constrained, max_spread=0, legacy=False) -> Tuple[Status, Optional[RoundResult]]:
    """Functional wrapper: (status, result-or-None) instead of raising."""
    try:
        return Status.OK, consensus_round(values, n_failing, constrained, max_spread, legacy)
    except ConsensusRevert as e:
        return e.status, None
