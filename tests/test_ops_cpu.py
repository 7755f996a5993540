"""Native CPU engines (csrc/engine/reference_cpu.cpp) vs the golden Python model and the torch ref."""
import random

import pytest
import torch

from fixtures import GOLDEN, N_FAILING
from helpers import beta_oracles, run_exact, run_fast
from svoc import ops as svops
from svoc import reference as ref
from svoc.ops import torch_ref
from svoc.status import Status

pytestmark = pytest.mark.skipif(not svops.available(), reason="svoc/_C.so not built")


@pytest.mark.parametrize("name", list(GOLDEN))
def test_exact_cpu_goldens(name):
    values, constrained, ms, g = GOLDEN[name]
    o = run_exact(torch.tensor([values], dtype=torch.int64), N_FAILING, constrained, ms)
    assert o["status"].tolist() == [0]
    assert o["c1"][0].tolist() == g["c1"]
    assert o["qr"][0].tolist() == g["qr"]
    assert o["reliable"][0].bool().tolist() == g["reliable"]
    assert o["consensus"][0].tolist() == g["consensus"]
    assert o["rel"][0].tolist() == [g["rel1"], g["rel2"]]
    assert o["skew"][0].tolist() == g["skewness"]
    assert o["kurt"][0].tolist() == g["kurtosis"]


def _random_instance(rng, N, D, constrained, spread):
    if constrained:
        c = [rng.randint(0, 1_000_000) for _ in range(D)]
        return [[min(1_000_000, max(0, c[d] + rng.randint(-spread, spread))) for d in range(D)] for _ in range(N)]
    c = [rng.randint(-50_000_000, 50_000_000) for _ in range(D)]
    return [[c[d] + rng.randint(-spread, spread) for d in range(D)] for _ in range(N)]


@pytest.mark.parametrize("constrained", [True, False])
def test_exact_cpu_matches_python_random(constrained):
    """Bit-exact agreement incl. status codes on random instances (many of them revert)."""
    rng = random.Random(1234 + constrained)
    cases = []
    for _ in range(60):
        N = rng.choice([2, 3, 4, 5, 7, 9, 16])
        D = rng.choice([1, 2, 3, 6])
        f = rng.choice([0, 1, 2, 3])
        spread = rng.choice([0, 3, 50, 5000, 400_000])
        cases.append((N, D, f, _random_instance(rng, N, D, constrained, spread)))
    ms = 3_000_000
    for N, D, f, vals in cases:
        st_ref, r = ref.round_status(vals, f, constrained, ms)
        o = run_exact(torch.tensor([vals], dtype=torch.int64), f, constrained, ms)
        assert o["status"].item() == int(st_ref), (N, D, f, vals)
        if st_ref == Status.OK:
            assert o["consensus"][0].tolist() == r.consensus
            assert o["rel"][0].tolist() == [r.rel1, r.rel2]
            assert o["skew"][0].tolist() == r.skewness
            assert o["kurt"][0].tolist() == r.kurtosis
            assert o["reliable"][0].bool().tolist() == r.reliable


def test_exact_cpu_revert_leaves_outputs():
    vals = [[500_000, 100_000]] * 7      # zero variance -> DIV_BY_ZERO
    o = run_exact(torch.tensor([vals], dtype=torch.int64), 2, True)
    assert o["status"].item() == Status.DIV_BY_ZERO
    assert o["consensus"].abs().sum().item() == 0


@pytest.mark.parametrize("N,D,f,constrained", [(7, 6, 2, True), (64, 40, 8, True), (33, 17, 5, False),
                                                (256, 24, 32, True), (20, 3, 15, True)])
def test_fast_cpu_vs_torch_ref(N, D, f, constrained):
    x, _ = beta_oracles(6, N, D, f, seed=N + D)
    ms = 1.0
    o = run_fast(x, D, f, constrained, ms)
    r = torch_ref.fast_round(x[:, :, :D], f, constrained, ms)
    ok = o["status"] == 0
    assert ok.any()
    assert torch.equal(o["reliable"][ok].bool(), r["reliable"][ok])
    torch.testing.assert_close(o["c1"][ok], r["c1"][ok], rtol=0, atol=1e-6)
    torch.testing.assert_close(o["consensus"][ok], r["consensus"][ok], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(o["qr"][ok], r["qr"][ok], rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(o["rel"][ok], r["rel"][ok], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(o["skew"][ok], r["skew"][ok], rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(o["kurt"][ok], r["kurt"][ok], rtol=1e-3, atol=1e-3)


def test_fast_cpu_tracks_exact_on_fixtures():
    """Fast mode on the reference fixtures stays within wsad rounding of the exact engine (A.3)."""
    for name, (values, constrained, ms, g) in GOLDEN.items():
        x = torch.tensor([values], dtype=torch.float64) / 1e6
        o = run_fast(x.float(), x.shape[2], N_FAILING, constrained, ms / 1e6 if ms else 1.0)
        assert o["status"].item() == 0
        assert o["reliable"][0].bool().tolist() == g["reliable"]
        assert torch.allclose(o["consensus"][0].double(), torch.tensor(g["consensus"], dtype=torch.float64) / 1e6, atol=2e-6)
        assert torch.allclose(o["rel"][0].double(), torch.tensor([g["rel1"], g["rel2"]], dtype=torch.float64) / 1e6, atol=2e-5)


def test_unconstrained_updates_reject_non_finite():
    """Fast-mode unconstrained updates holding NaN / inf are rejected (NON_FINITE), others applied."""
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    from svoc.status import Status
    e = ConsensusEngine(ConsensusConfig(n_oracles=4, dimension=3, n_failing_oracles=0, constrained=False,
                                        unconstrained_max_spread=10.0), 2, device="cpu", mode="fast",
                        storage="fp32")
    vals = torch.tensor([[1.0, 2.0, 3.0], [float("nan"), 0.0, 0.0], [0.0, float("inf"), 0.0], [5.0, -5.0, 1e30]])
    st = e.apply_updates(torch.tensor([0, 0, 1, 1]), torch.tensor([0, 1, 2, 3]), vals)
    assert st.tolist() == [Status.OK, Status.NON_FINITE, Status.NON_FINITE, Status.OK]
    assert e.values[0, 0, :3].tolist() == [1.0, 2.0, 3.0] and int(e.enabled[0, 1]) == 0


def test_exact_int32_storage_matches_int64_cpu():
    """int32 wsad storage (constrained) gives the identical exact round as int64 storage."""
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    cfg = ConsensusConfig(n_oracles=16, dimension=20, n_failing_oracles=3, constrained=True)
    e32 = ConsensusEngine(cfg, 6, device="cpu", mode="exact", storage="int32")
    e64 = ConsensusEngine(cfg, 6, device="cpu", mode="exact")
    assert e32.values.dtype == torch.int32
    for e in (e32, e64):
        e.randomize(seed=2)
        e.run_round()
    for k in ("consensus", "skew", "kurt", "rel", "qr", "reliable", "c1", "status"):
        assert torch.equal(getattr(e32, k), getattr(e64, k)), k
    # an update beyond int32 is rejected (not wrapped into range)
    st = e32.step(torch.tensor([0]), torch.tensor([1]), torch.tensor([[2 ** 32 + 5] * 20]))
    assert int(st[0]) != 0
    with pytest.raises(ValueError):
        ConsensusEngine(ConsensusConfig(n_oracles=8, dimension=2, n_failing_oracles=1, constrained=False), 1,
                        device="cpu", mode="exact", storage="int32")
