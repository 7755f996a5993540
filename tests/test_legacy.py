"""Obsolete contract generations (contract/obsolete/src/contract_nd.cairo, contract_1d_constrained.cairo).

Differences from the current contract: constrained reliability is
``W - 2 sqrt(mean qr)`` without ``/D`` (contract_nd.cairo:418,437) and no moments are computed (so
no zero-variance / too-few-reliable reverts).  Checked layer by layer: golden Python model, C++
exact engine, ABI facades, fast engine vs the fp32 PyTorch reference; GPU twins in
test_legacy_gpu below (marked gpu).
"""
import random

import pytest
import torch

from fixtures import GOLDEN, N_FAILING
from helpers import run_exact, run_fast
from svoc import reference as ref
from svoc.api import LegacyOracleConsensus
from svoc.ops import torch_ref
from svoc.status import ConsensusRevert, Status

W = 1_000_000


@pytest.mark.parametrize("name", list(GOLDEN))
def test_legacy_golden_model_vs_current(name):
    values, constrained, ms, g = GOLDEN[name]
    cur = ref.consensus_round(values, N_FAILING, constrained, ms)
    st, old = ref.round_status(values, N_FAILING, constrained, ms, legacy=True)
    if st != Status.OK:
        # without /D the 6-D fixture's RMS deviation exceeds 0.5: the obsolete contract reverts
        # (which is why the current one divides by D, contract.cairo:436-439)
        assert name == "constrained_6d" and st == Status.RELIABILITY_INTERVAL
        o = run_exact(torch.tensor([values]), N_FAILING, constrained, ms, legacy=True)
        assert int(o["status"][0]) == Status.RELIABILITY_INTERVAL
        return
    # pass 1 / ranking / consensus are shared
    assert old.c1 == cur.c1 and old.qr == cur.qr and old.reliable == cur.reliable
    assert old.consensus == cur.consensus
    assert old.skewness == [0] * len(values[0]) and old.kurtosis == [0] * len(values[0])
    D = len(values[0])
    if constrained:
        # W - 2 sqrt(mean) vs W - 2 sqrt(mean / D): equal for D = 1, lower for D > 1
        mean1 = ref.idiv(sum(cur.qr), len(cur.qr))
        assert old.rel1 == W - 2 * ref.wsqrt(mean1)
        assert (old.rel1 <= cur.rel1) and (D > 1 or old.rel1 == cur.rel1)
    else:
        assert (old.rel1, old.rel2) == (cur.rel1, cur.rel2)


@pytest.mark.parametrize("constrained", [True, False])
def test_legacy_cpu_engine_matches_model(constrained):
    rng = random.Random(5)
    for N, D, f in [(7, 2, 2), (7, 1, 2), (9, 3, 1), (4, 2, 1), (3, 1, 1), (20, 4, 15)]:
        for _ in range(6):
            hi = W if constrained else 40 * W
            vals = [[rng.randint(W // 3, W // 2) if constrained else rng.randint(-hi, hi) for _ in range(D)]
                    for _ in range(N)]
            ms = 0 if constrained else 30 * W
            st, r = ref.round_status(vals, f, constrained, ms, legacy=True)
            o = run_exact(torch.tensor([vals], dtype=torch.int64), f, constrained, ms, legacy=True)
            assert int(o["status"][0]) == int(st)
            if st == Status.OK:
                assert o["consensus"][0].tolist() == r.consensus
                assert o["rel"][0].tolist() == [r.rel1, r.rel2]
                assert o["qr"][0].tolist() == r.qr
                assert o["skew"][0].tolist() == [0] * D and o["kurt"][0].tolist() == [0] * D


def test_legacy_accepts_three_reliable_oracles():
    """R = 3: the current contract reverts in kurtosis ((n-2)(n-3) = 0); the obsolete one has no moments."""
    vals = [[400000, 500000], [410000, 520000], [390000, 480000], [900000, 100000]]
    st_cur, _ = ref.round_status(vals, 1, True)
    st_old, r = ref.round_status(vals, 1, True, legacy=True)
    assert st_cur.is_revert and st_old == Status.OK
    o = run_exact(torch.tensor([vals]), 1, True, legacy=True)
    assert int(o["status"][0]) == 0 and o["rel"][0].tolist() == [r.rel1, r.rel2]
    of = run_fast(torch.tensor([vals], dtype=torch.float32) / W, 2, 1, True, legacy=True)
    assert int(of["status"][0]) == 0


@pytest.mark.parametrize("constrained", [True, False])
def test_legacy_fast_cpu_vs_torch(constrained):
    from helpers import beta_oracles
    x, _ = beta_oracles(6, 20, 5, 3, seed=11, dtype=torch.float32)
    if not constrained:
        x = x * 8 - 4
    o = run_fast(x, 5, 3, constrained, 10.0, legacy=True)
    r = torch_ref.fast_round(x[:, :, :5], 3, constrained, 10.0, legacy=True)
    ok = o["status"] == 0
    assert ok.all()
    assert torch.equal(o["reliable"].bool(), r["reliable"])
    torch.testing.assert_close(o["rel"], r["rel"], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(o["consensus"], r["consensus"], rtol=0, atol=1e-6)
    assert not o["skew"].any() and not o["kurt"].any()


def _abi_flow(variant, D):
    admins = [0xA1, 0xA2, 0xA3]
    oracles = [0x100 + i for i in range(7)]
    c = LegacyOracleConsensus(admins, True, 2, 2, True, 0, D, oracles, variant=variant)
    m = ref.ReferenceContract(admins, True, 2, 2, True, 0, D, oracles, legacy=True)
    rng = random.Random(3)
    for step in range(20):
        o = oracles[step % 7]
        if D == 1:
            v = rng.randint(300000, 700000)
            pv, mv = v, [v]
        else:
            pv = mv = [rng.randint(300000, 700000) for _ in range(D)]
        try:
            m.update_prediction(o, mv)
            exp = None
        except ConsensusRevert as e:
            exp = e.status
        if exp is None:
            c.update_prediction(o, pv)
        else:
            with pytest.raises(ConsensusRevert):
                c.update_prediction(o, pv)
        cons = c.get_consensus_value()
        assert (cons if D > 1 else [cons]) == m.consensus_value
        assert c.get_first_pass_consensus_reliability() == m.rel1
        assert c.get_second_pass_consensus_reliability() == m.rel2
    with pytest.raises(AttributeError):
        c.get_skewness()


def test_legacy_abi_1d():
    _abi_flow("1d_legacy", 1)


def test_legacy_abi_nd():
    _abi_flow("nd_legacy", 3)


def test_legacy_1d_config_validation():
    with pytest.raises(ValueError):
        LegacyOracleConsensus([1], True, 1, 0, True, 0, 2, [5, 6], variant="1d_legacy")


@pytest.mark.gpu
@pytest.mark.parametrize("constrained", [True, False])
def test_legacy_gpu_exact_and_fast(constrained):
    rng = random.Random(8)
    vals = [[[rng.randint(W // 3, W // 2) for _ in range(3)] for _ in range(9)] for _ in range(16)]
    x = torch.tensor(vals, dtype=torch.int64)
    ms = 0 if constrained else 2 * W
    oc = run_exact(x, 2, constrained, ms, legacy=True)
    og = run_exact(x.cuda(), 2, constrained, ms, legacy=True)
    for k in ("status", "consensus", "rel", "qr", "skew", "kurt", "reliable"):
        assert torch.equal(oc[k], og[k].cpu()), k
    from helpers import beta_oracles
    # without /D a constrained round only passes the interval check for small D (RMS over all
    # dims <= 0.5): D = 3 constrained, D = 300 unconstrained
    D = 3 if constrained else 300
    xb, _ = beta_oracles(12, 64, D, 8, seed=2)
    for hint in (0, -7):
        o = run_fast(xb.cuda(), D, 8, constrained, 30.0, wave_hint=hint, legacy=True)
        r = torch_ref.fast_round(xb.cuda()[:, :, :D], 8, constrained, 30.0, legacy=True)
        oc = run_fast(xb, D, 8, constrained, 30.0, legacy=True)
        assert torch.equal(o["status"].cpu(), oc["status"])
        ok = o["status"] == 0
        assert ok.all()
        torch.testing.assert_close(o["rel"], r["rel"], rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(o["consensus"], r["consensus"], rtol=0, atol=2e-6)
        assert not o["skew"].any()
