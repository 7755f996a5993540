"""Exact-mode transactional streaming (ConsensusEngine.step -> _exact_transactions) against the golden
contract replayed one instance at a time: every update is its own transaction (store + full round; a
failing round reverts the whole transaction, contract.cairo:588-603), with injected reverts --
zero-variance columns (DIV_BY_ZERO), out-of-range values (INTERVAL_INPUT), unknown oracles
(NOT_ORACLE).  Both wave groupings: the general device-side one (interleaved batches, uneven counts)
and the strided ``updates_per_instance`` layout."""
import random

import pytest
import torch

from svoc import ops as svops
from svoc import reference as ref
from svoc.config import ConsensusConfig
from svoc.status import ConsensusRevert, Status

pytestmark = pytest.mark.skipif(not svops.available(), reason="svoc/_C.so not built")

N, D, F = 7, 3, 2
ADMINS = [1000, 1001, 1002]
ORACLES = [2000 + i for i in range(N)]


def _update(rng, flat):
    """A random constrained prediction: often with a pinned column 0 (zero-variance bait), sometimes out
    of range, otherwise uniform."""
    r = rng.random()
    if r < 0.08:
        return [1_000_001 if rng.random() < 0.5 else -3] + [rng.randint(0, 1_000_000) for _ in range(D - 1)]
    if r < 0.7:   # column 0 pinned to the instance's value: enough of them zero that column's variance
        return [flat[0]] + [rng.randint(0, 1_000_000) for _ in range(D - 1)]
    return [rng.randint(0, 1_000_000) for _ in range(D)]


def _stream(seed, B, per_inst):
    rng = random.Random(seed)
    flats = [[rng.randint(0, 1_000_000) for _ in range(D)] for _ in range(B)]
    ups = []
    for b in range(B):
        seq = [(o, _update(rng, flats[b])) for o in range(N)]       # bootstrap: every oracle once
        for _ in range(per_inst - N):
            o = rng.randrange(N + 1)                                 # N = an unknown oracle
            seq.append((o, _update(rng, flats[b])))
        ups.append(seq)
    return ups


def _replay_reference(ups):
    out = []
    contracts = []
    for seq in ups:
        c = ref.ReferenceContract(ADMINS, True, 2, F, True, 0, D, ORACLES)
        st = []
        for o, v in seq:
            try:
                st.append(c.update_prediction(ORACLES[o] if o < N else 99, v))
            except ConsensusRevert as e:
                st.append(e.status)
        out.append(st)
        contracts.append(c)
    return out, contracts


def _engine(B, device):
    from svoc.engine import ConsensusEngine
    cfg = ConsensusConfig(n_oracles=N, dimension=D, n_failing_oracles=F, constrained=True)
    return ConsensusEngine(cfg, batch=B, device=device, mode="exact")


def _check(e, contracts, st_eng, st_ref):
    assert st_eng == st_ref
    for b, c in enumerate(contracts):
        assert e.values[b, :, :D].tolist() == c.values, b
        assert int(e.n_active[b]) == c.n_active_oracles, b
        assert bool(e.consensus_active[b]) == c.consensus_active(), b
        if c.consensus_active():
            assert e.consensus[b].tolist() == c.get_consensus_value(), b
            assert [int(x) for x in e.rel[b]] == [c.rel1, c.rel2], b
            assert e.skew[b].tolist() == c.skewness and e.kurt[b].tolist() == c.kurtosis, b


def _run_general(device, seed=3, B=5, per_inst=14, n_batches=3):
    ups = _stream(seed, B, per_inst)
    st_ref, contracts = _replay_reference(ups)
    # interleave the instances' updates at random (order kept per instance), cut into batches
    rng = random.Random(seed + 1)
    cursor = [0] * B
    order = []
    while len(order) < B * per_inst:
        b = rng.choice([i for i in range(B) if cursor[i] < per_inst])
        order.append((b, cursor[b]))
        cursor[b] += 1
    e = _engine(B, device)
    st_eng = [[None] * per_inst for _ in range(B)]
    cuts = sorted(rng.sample(range(1, len(order)), n_batches - 1))
    for lo, hi in zip([0] + cuts, cuts + [len(order)]):
        part = order[lo:hi]
        inst = torch.tensor([b for b, _ in part])
        orc = torch.tensor([ups[b][k][0] for b, k in part])
        vals = torch.tensor([ups[b][k][1] for b, k in part], dtype=torch.int64)
        st = e.step(inst, orc, vals).cpu().tolist()
        for (b, k), s in zip(part, st):
            st_eng[b][k] = Status(s)
    _check(e, contracts, st_eng, st_ref)
    return st_ref


def _run_strided(device, seed=12, B=6, per_inst=7 + 9):
    ups = _stream(seed, B, per_inst)
    st_ref, contracts = _replay_reference(ups)
    e = _engine(B, device)
    st_eng = [[] for _ in range(B)]
    # bootstrap batch (7 per instance), then K = 3 per instance per batch, laid out b * K + k
    for lo, hi in [(0, N)] + [(k, k + 3) for k in range(N, per_inst, 3)]:
        K = hi - lo
        inst = torch.tensor([b for b in range(B) for _ in range(K)])
        orc = torch.tensor([ups[b][k][0] for b in range(B) for k in range(lo, hi)])
        vals = torch.tensor([ups[b][k][1] for b in range(B) for k in range(lo, hi)], dtype=torch.int64)
        st = e.step(inst, orc, vals, updates_per_instance=K).cpu().tolist()
        for b in range(B):
            st_eng[b] += [Status(s) for s in st[b * K:(b + 1) * K]]
    _check(e, contracts, st_eng, st_ref)
    return st_ref


def _covers_reverts(*st_lists):
    seen = {s for st in st_lists for seq in st for s in seq}
    assert {Status.OK, Status.NOT_ACTIVE, Status.DIV_BY_ZERO, Status.INTERVAL_INPUT, Status.NOT_ORACLE} <= seen, seen


def test_exact_stream_general_waves_cpu():
    _covers_reverts(_run_general("cpu"), _run_general("cpu", seed=8, B=4, per_inst=20, n_batches=2))


def test_exact_stream_strided_waves_cpu():
    _covers_reverts(_run_strided("cpu"))


def test_strided_layout_must_divide():
    e = _engine(2, "cpu")
    with pytest.raises(ValueError):
        e.step(torch.tensor([0, 1, 1]), torch.tensor([0, 0, 1]), torch.zeros(3, D, dtype=torch.int64),
               updates_per_instance=2)


@pytest.mark.gpu
def test_exact_stream_gpu():
    _covers_reverts(_run_general("cuda"), _run_strided("cuda"))


def test_synthetic_stream_keeps_engine_failing_set():
    """bench.py's update stream draws its U(0,1) rows for the engine's own failing oracles
    (ConsensusEngine.failing_mask): an honest oracle never receives a uniform row, so no instance ends
    up with more than f noisy oracles (which the exact column kernel hands to the i128 kernel)."""
    from svoc.engine import ConsensusEngine
    from svoc.stream import SyntheticUpdateStream
    B, n, d, f, U = 3, 16, 40, 3, 8
    cfg = ConsensusConfig(n_oracles=n, dimension=d, n_failing_oracles=f, constrained=True)
    eng = ConsensusEngine(cfg, batch=B, device="cpu", mode="exact")
    eng.randomize(seed=4)
    m = eng.failing_mask
    assert m.shape == (B, n) and (m.sum(1) == f).all()
    s = SyntheticUpdateStream(B, n, d, U, f, pool=2, device="cpu", seed=1, dtype=torch.int64, failing=m)
    assert torch.equal(s.failing, m)
    for k in range(2):
        inst, orc, vals = s.batch(k)
        # honest rows are Beta(20, 20): none is near 0 or 1 in every column, uniform rows spread out
        spread = (vals.double() / 1e6).std(dim=1)
        fail = m[inst, orc]
        assert (spread[~fail] < 0.15).all() and (spread[fail] > 0.15).all()
    eng.step(*s.batch(0), updates_per_instance=U)
    assert (eng.status == int(Status.OK)).all()
