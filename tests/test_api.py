"""Contract-ABI facade (exact mode) against the golden Python contract, incl. governance flows."""
import random

import pytest

from fixtures import ADMINS, GOLDEN, N_FAILING, NEW_ORACLE, ORACLES
from svoc import codec
from svoc import ops as svops
from svoc import reference as ref
from svoc.api import ConsensusService, OracleConsensus
from svoc.config import ConsensusConfig
from svoc.status import ConsensusRevert, Status

pytestmark = pytest.mark.skipif(not svops.available(), reason="svoc/_C.so not built")


def make(name, mode="exact", device="cpu"):
    values, constrained, ms, g = GOLDEN[name]
    c = OracleConsensus(ADMINS, True, 2, N_FAILING, constrained, codec.i128_to_felt(ms), len(values[0]),
                        ORACLES, device=device, mode=mode)
    return c, values, g


@pytest.mark.parametrize("name", list(GOLDEN))
def test_abi_flow_matches_golden(name):
    c, values, g = make(name)
    assert not c.consensus_active()
    assert c.get_consensus_value() == [0] * len(values[0])
    assert c.get_first_pass_consensus_reliability() == 0
    for o, v in zip(ORACLES[:-1], values[:-1]):
        assert c.update_prediction(o, codec.as_felt(v)) == Status.NOT_ACTIVE
    assert c.update_prediction(ORACLES[-1], codec.as_felt(values[-1])) == Status.OK
    assert c.consensus_active()
    assert codec.as_wsad(c.get_consensus_value()) == g["consensus"]
    assert c.get_reliability() == (g["rel1"], g["rel2"])
    assert codec.as_wsad(c.get_skewness()) == g["skewness"]
    assert codec.as_wsad(c.get_kurtosis()) == g["kurtosis"]
    vl = c.get_oracle_value_list(ADMINS[0])
    assert [r for (_, _, _, r) in vl] == g["reliable"]
    with pytest.raises(ConsensusRevert):
        c.get_oracle_value_list(ORACLES[0])


def test_replacement_flow_test_contract_192_213():
    c, values, _ = make("constrained_2d")
    for o, v in zip(ORACLES, values):
        c.update_prediction(o, codec.as_felt(v))
    c.update_proposition(ADMINS[0], (6, NEW_ORACLE))
    assert c.get_oracle_list()[6] == ORACLES[6]
    assert not c.vote_for_a_proposition(ADMINS[0], 0, True)
    assert c.get_oracle_list()[6] == ORACLES[6]
    assert c.vote_for_a_proposition(ADMINS[1], 0, True)
    assert c.get_oracle_list()[6] == NEW_ORACLE
    assert c.get_replacement_propositions() == [None, None, None]
    # the new address can now submit; the old one cannot
    with pytest.raises(ConsensusRevert) as e:
        c.update_prediction(ORACLES[6], codec.as_felt(values[6]))
    assert e.value.status == Status.NOT_ORACLE
    assert c.update_prediction(NEW_ORACLE, codec.as_felt(values[6])) == Status.OK


def test_governance_reverts():
    c, values, _ = make("constrained_2d")
    with pytest.raises(ConsensusRevert) as e:
        c.update_proposition(ORACLES[0], (1, NEW_ORACLE))
    assert e.value.status == Status.NOT_ADMIN
    with pytest.raises(ConsensusRevert) as e:
        c.update_proposition(ADMINS[0], (7, NEW_ORACLE))
    assert e.value.status == Status.WRONG_ORACLE_INDEX
    with pytest.raises(ConsensusRevert) as e:
        c.update_proposition(ADMINS[0], (1, ORACLES[3]))
    assert e.value.status == Status.ALREADY_ORACLE
    c.update_proposition(ADMINS[0], (1, NEW_ORACLE))
    c.update_proposition(ADMINS[0], None)
    with pytest.raises(ConsensusRevert) as e:
        c.vote_for_a_proposition(ADMINS[1], 0, True)
    assert e.value.status == Status.UNWRAP_NONE
    # the reverted vote left no trace
    assert c._svc.gov.vote_matrix(0)[1][0] is False


def test_governance_random_vs_reference():
    """Random interleavings of proposals / votes / updates against the golden contract."""
    rng = random.Random(5)
    admins = [1000 + i for i in range(5)]
    oracles = [2000 + i for i in range(7)]
    pool = oracles + [3000 + i for i in range(6)]
    for trial in range(6):
        r = ref.ReferenceContract(admins, True, 3, 2, True, 0, 2, oracles)
        c = OracleConsensus(admins, True, 3, 2, True, 0, 2, oracles)
        for step in range(150):
            caller = rng.choice(admins + [oracles[0], 99])
            kind = rng.random()
            if kind < 0.3:
                prop = None if rng.random() < 0.2 else (rng.randrange(-1, 8), rng.choice(pool))
                fns = [(lambda x=x: x.update_proposition(caller, prop)) for x in (r, c)]
            elif kind < 0.7:
                w, s = rng.randrange(0, 6), rng.random() < 0.8
                fns = [(lambda x=x: x.vote_for_a_proposition(caller, w, s)) for x in (r, c)]
            else:
                o = rng.choice(pool + [oracles[0]])
                v = [rng.randint(0, 1_000_000), rng.randint(0, 1_000_000)]
                fns = [lambda: r.update_prediction(o, v), lambda: c.update_prediction(o, codec.as_felt(v))]
            res = []
            for f in fns:
                try:
                    res.append(("ok", f()))
                except ConsensusRevert as e:
                    res.append(("revert", e.status))
            if prop_none_guard(res):
                continue
            assert res[0][0] == res[1][0], (trial, step, res)
            if res[0][0] == "revert":
                assert res[0][1] == res[1][1], (trial, step, res)
            assert r.get_oracle_list() == c.get_oracle_list()
            assert r.get_replacement_propositions() == c.get_replacement_propositions()
            assert r.vote_matrix == c._svc.gov.vote_matrix(0)
        assert codec.as_wsad(c.get_consensus_value()) == r.get_consensus_value()


def prop_none_guard(res):
    return False


def test_service_batched_instances():
    cfg = ConsensusConfig(n_oracles=7, dimension=2, n_failing_oracles=2, constrained=True, n_admins=3)
    svc = ConsensusService(cfg, 4, ADMINS, ORACLES, device="cpu", mode="exact")
    values, _, _, g = GOLDEN["constrained_2d"]
    items = [(b, o, v) for b in range(4) for o, v in zip(ORACLES, values)]
    st = svc.update_predictions(items)
    assert st.count(Status.OK) == 4
    for b in range(4):
        assert svc.engine.consensus[b].tolist() == g["consensus"]


def test_service_governance_tensor_batch_matches_list():
    """ConsensusService.governance with a mapping of action tensors (the device path's interface; on the CPU the
    batch applies in order) == the same actions as a list of tuples: statuses, applied flags and the final
    oracle / vote state, with several actions per instance, non-admin callers and None propositions."""
    import torch
    from svoc.codec import address_to_limbs
    from svoc.governance import PROPOSE, VOTE
    cfg = ConsensusConfig(n_oracles=7, dimension=2, n_failing_oracles=2, constrained=True, n_admins=3)
    rng = random.Random(5)
    acts = []
    for _ in range(120):
        b = rng.randrange(4)
        caller = rng.choice(ADMINS + [123456789])
        if rng.random() < 0.4:
            prop = None if rng.random() < 0.2 else (rng.randrange(-1, 8), NEW_ORACLE + rng.randrange(3))
            acts.append(("propose", b, caller, prop))
        else:
            acts.append(("vote", b, caller, rng.randrange(4), rng.random() < 0.8))
    svc_l = ConsensusService(cfg, 4, ADMINS, ORACLES, device="cpu", mode="exact")
    svc_t = ConsensusService(cfg, 4, ADMINS, ORACLES, device="cpu", mode="exact")
    st_l, ap_l = svc_l.governance(acts)
    K = len(acts)
    t = dict(inst=torch.zeros(K, dtype=torch.int64), caller=torch.zeros(K, 4, dtype=torch.int64),
             kind=torch.zeros(K, dtype=torch.int32), arg0=torch.zeros(K, dtype=torch.int32),
             arg1=torch.zeros(K, dtype=torch.int64), addr=torch.zeros(K, 4, dtype=torch.int64))
    for k, a in enumerate(acts):
        t["inst"][k] = a[1]
        t["caller"][k] = torch.tensor(address_to_limbs(a[2]))
        if a[0] == "propose":
            t["kind"][k] = PROPOSE
            if a[3] is not None:
                t["arg0"][k], t["arg1"][k] = 1, a[3][0]
                t["addr"][k] = torch.tensor(address_to_limbs(a[3][1]))
        else:
            t["kind"][k], t["arg0"][k], t["arg1"][k] = VOTE, a[3], int(a[4])
    st_t, ap_t = svc_t.governance(t)
    assert [Status(s) for s in st_t.tolist()] == st_l and [bool(a) for a in ap_t.tolist()] == ap_l
    assert any(ap_l) and st_l.count(Status.OK) < K
    for b in range(4):
        assert svc_t.gov.vote_matrix(b) == svc_l.gov.vote_matrix(b)
    assert torch.equal(svc_t.gov.oracle_addr, svc_l.gov.oracle_addr)
