"""Golden-model tests: the exact Python model reproduces the reference contract bit for bit."""
import pytest

from fixtures import GOLDEN, N_FAILING, ADMINS, ORACLES, NEW_ORACLE
from svoc import reference as ref
from svoc.status import ConsensusRevert, Status


@pytest.mark.parametrize("name", list(GOLDEN))
def test_round_goldens(name):
    values, constrained, ms, g = GOLDEN[name]
    r = ref.consensus_round(values, N_FAILING, constrained, ms)
    for k, v in g.items():
        assert getattr(r, k) == v, k


def test_indexed_merge_sort():
    # test_math.cairo:10-19
    got = ref.indexed_sort([20, 30, 29, 1, 300, 100])
    assert got == [(3, 1), (0, 20), (2, 29), (1, 30), (5, 100), (4, 300)]


def test_indexed_merge_sort_tie_rule():
    # ties: higher index first (sort.cairo:96-101)
    assert [i for i, _ in ref.indexed_sort([5, 5, 1, 5])] == [2, 3, 1, 0]


def test_sqrt():
    assert ref.wsqrt(9 * ref.WSAD) == 3 * ref.WSAD        # test_math.cairo:36
    assert ref.wsqrt(16 * ref.WSAD) == 4 * ref.WSAD
    assert ref.wsqrt(305 * ref.WSAD) == 17464249
    assert ref.wsqrt(0) == 0
    with pytest.raises(ConsensusRevert) as e:
        ref.wsqrt(1)
    assert e.value.status == Status.DIV_BY_ZERO


def test_fixed_point_quirks():
    assert ref.wmul(-1_300_000, 1_000_000) == -1_299_999     # survey §2.8-4
    assert ref.idiv(-7, 2) == -3 and ref.idiv(7, -2) == -3
    assert ref.smooth_median([3, 1, 2]) == 1                 # odd branch dead: (1+2)/2


def test_contract_flow_unconstrained():
    values, constrained, ms, g = GOLDEN["unconstrained_2d"]
    c = ref.ReferenceContract(ADMINS, True, 2, N_FAILING, constrained, ms, 2, ORACLES)
    assert not c.consensus_active()
    assert c.get_consensus_value() == [0, 0]
    for o, v in zip(ORACLES[:-1], values[:-1]):
        assert c.update_prediction(o, v) == Status.NOT_ACTIVE
    assert c.update_prediction(ORACLES[-1], values[-1]) == Status.OK
    assert c.get_consensus_value() == g["consensus"]
    assert c.get_first_pass_consensus_reliability() == g["rel1"]
    assert c.get_second_pass_consensus_reliability() == g["rel2"]
    # test_contract.cairo:285-288 comment-only expectations, as hard asserts
    assert round(c.get_consensus_value()[0] / 1e6, 3) == 20.715
    assert round(c.get_consensus_value()[1] / 1e6, 1) == 10.4
    assert int(c.rel1 / 1e3) == 533 and int(c.rel2 / 1e3) == 647


def test_replacement_flow():
    # test_contract.cairo:192-213
    values, constrained, ms, _ = GOLDEN["constrained_2d"]
    c = ref.ReferenceContract(ADMINS, True, 2, N_FAILING, constrained, ms, 2, ORACLES)
    for o, v in zip(ORACLES, values):
        c.update_prediction(o, v)
    c.update_proposition(ADMINS[0], (6, NEW_ORACLE))
    assert c.get_oracle_list()[6] == ORACLES[6]
    assert not c.vote_for_a_proposition(ADMINS[0], 0, True)     # self vote already counted: 1 < 2
    assert c.get_oracle_list()[6] == ORACLES[6]
    assert c.vote_for_a_proposition(ADMINS[1], 0, True)
    assert c.get_oracle_list()[6] == NEW_ORACLE
    assert c.get_replacement_propositions() == [None, None, None]
    # value / enabled / reliable survive replacement (survey §2.8-6)
    addr, vals, enabled, reliable = c.get_oracle_value_list(ADMINS[0])[6]
    assert vals == values[6] and enabled


def test_reverts_roll_back():
    values, constrained, ms, _ = GOLDEN["constrained_2d"]
    c = ref.ReferenceContract(ADMINS, True, 2, N_FAILING, constrained, ms, 2, ORACLES)
    with pytest.raises(ConsensusRevert) as e:
        c.update_prediction(ORACLES[0], [1_000_001, 0])
    assert e.value.status == Status.INTERVAL_INPUT
    with pytest.raises(ConsensusRevert) as e:
        c.update_prediction(12345, [1, 2])
    assert e.value.status == Status.NOT_ORACLE
    assert c.n_active_oracles == 0
    # zero variance column -> sqrt(0) = 0 -> wdiv by zero -> whole tx reverts
    for o in ORACLES[:-1]:
        c.update_prediction(o, [500_000, 100_000])
    with pytest.raises(ConsensusRevert) as e:
        c.update_prediction(ORACLES[-1], [500_000, 100_000])
    assert e.value.status == Status.DIV_BY_ZERO
    assert c.n_active_oracles == 6 and not c.consensus_active()
    # None proposition + majority -> unwrap panic
    c.update_proposition(ADMINS[0], (1, NEW_ORACLE))
    c.update_proposition(ADMINS[0], None)
    with pytest.raises(ConsensusRevert) as e:
        c.vote_for_a_proposition(ADMINS[1], 0, True)
    assert e.value.status == Status.UNWRAP_NONE


def test_coalescing_property():
    """Survey §2.8-13: final state depends only on the last value per oracle."""
    import random
    rng = random.Random(0)
    for _ in range(30):
        c = ref.ReferenceContract(ADMINS, True, 2, N_FAILING, True, 0, 3, ORACLES)
        last = {}
        for o in ORACLES:
            v = [rng.randint(0, 1_000_000) for _ in range(3)]
            c.update_prediction(o, v)
            last[o] = v
        for _ in range(20):
            o = rng.choice(ORACLES)
            v = [rng.randint(0, 1_000_000) for _ in range(3)]
            try:
                c.update_prediction(o, v)
                last[o] = v
            except ConsensusRevert:
                pass
        st, r = ref.round_status([last[o] for o in ORACLES], N_FAILING, True)
        assert st == Status.OK
        assert r.consensus == c.get_consensus_value() and r.rel2 == c.rel2


def test_median_index_first_occurrence():
    """math.cairo:87-110: median_index sorts a copy, takes sorted[len/2] and finds its FIRST index in the
    original array by value (find_index), so duplicates resolve to the earliest position."""
    from svoc import reference as r
    assert r.median_index([20, 30, 29, 1, 300, 100]) == 1          # sorted[3] = 30 at index 1
    assert r.median([20, 30, 29, 1, 300, 100]) == 30
    assert r.median_index([5, 7, 7, 1, 7]) == 1                     # sorted[2] = 7: first 7 is index 1
    assert r.median_index([3]) == 0
    with pytest.raises(Exception):
        r.median_index([])
    with pytest.raises(Exception):
        r.find_index(4, [1, 2, 3])                                  # 'value not found'
