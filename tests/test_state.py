"""Checkpoint / resume: .svoc round trip and restart equivalence (survey §5.4)."""
import os
import random

import pytest
import torch

from fixtures import ADMINS, ORACLES, NEW_ORACLE
from svoc import ops as svops
from svoc import state
from svoc.api import ConsensusService
from svoc.config import ConsensusConfig

pytestmark = pytest.mark.skipif(not svops.available(), reason="svoc/_C.so not built")


def _drive(svc, rng, steps):
    for _ in range(steps):
        b = rng.randrange(svc.B)
        if rng.random() < 0.85:
            svc.update_predictions([(b, rng.choice(ORACLES), [rng.randint(0, 1_000_000) for _ in range(3)])])
        else:
            svc.governance([("propose", b, ADMINS[0], (rng.randrange(7), NEW_ORACLE + rng.randrange(3))),
                            ("vote", b, ADMINS[1], 0, True)])


def _snapshot(svc):
    e, g = svc.engine, svc.gov
    return [x.clone() for x in (e.values, e.enabled, e.reliable, e.n_active, e.consensus_active, e.consensus,
                                e.rel, e.skew, e.kurt, g.oracle_addr, g.votes, g.prop_tag, g.prop_idx)]


def test_restart_equivalence(tmp_path):
    cfg = ConsensusConfig(n_oracles=7, dimension=3, n_failing_oracles=2, constrained=True, n_admins=3)
    a = ConsensusService(cfg, 3, ADMINS, ORACLES, device="cpu", mode="exact")
    rng = random.Random(7)
    _drive(a, rng, 60)
    p = os.path.join(tmp_path, "s.svoc")
    state.save(a, p)
    b = state.load(p)
    for x, y in zip(_snapshot(a), _snapshot(b)):
        assert torch.equal(x, y)
    r1, r2 = random.Random(9), random.Random(9)
    _drive(a, r1, 80)
    _drive(b, r2, 80)
    for x, y in zip(_snapshot(a), _snapshot(b)):
        assert torch.equal(x, y)


def test_corruption_detected(tmp_path):
    cfg = ConsensusConfig(n_oracles=7, dimension=3, n_failing_oracles=2, n_admins=3)
    a = ConsensusService(cfg, 2, ADMINS, ORACLES, device="cpu", mode="exact")
    p = os.path.join(tmp_path, "s.svoc")
    state.save(a, p)
    raw = bytearray(open(p, "rb").read())
    raw[-3] ^= 0xFF
    open(p, "wb").write(bytes(raw))
    with pytest.raises(Exception, match="CRC"):
        state.load(p)


def test_corrupt_header_rejected_without_allocation(tmp_path):
    """A section header claiming a huge shape (overflowing numel, or more bytes than the file holds)
    fails cleanly instead of allocating: the load checks sizes against the bytes left in the file."""
    import struct
    cfg = ConsensusConfig(n_oracles=7, dimension=3, n_failing_oracles=2, n_admins=3)
    a = ConsensusService(cfg, 2, ADMINS, ORACLES, device="cpu", mode="exact")
    p = os.path.join(tmp_path, "s.svoc")
    state.save(a, p)
    raw = bytearray(open(p, "rb").read())
    ml = struct.unpack_from("<I", raw, 12)[0]
    o = 16 + ml                                  # first section header
    nl = struct.unpack_from("<I", raw, o)[0]
    o += 4 + nl + 1                              # name, dtype
    nd = raw[o]
    assert nd >= 1
    for huge, msg in ((1 << 62, "overflow|size mismatch|truncated"), (1 << 40, "size mismatch|truncated")):
        bad = bytearray(raw)
        struct.pack_into("<Q", bad, o + 1, huge)
        open(p, "wb").write(bytes(bad))
        with pytest.raises(Exception, match=msg):
            state.load(p)
    # a consistent header (shape and nbytes agree) that promises more bytes than the file holds
    bad = bytearray(raw)
    es_nb_off = o + 1 + 8 * nd
    old_nb = struct.unpack_from("<Q", bad, es_nb_off)[0]
    old_d0 = struct.unpack_from("<Q", bad, o + 1)[0]
    struct.pack_into("<Q", bad, o + 1, old_d0 * 10**9)
    struct.pack_into("<Q", bad, es_nb_off, old_nb * 10**9)
    open(p, "wb").write(bytes(bad))
    with pytest.raises(Exception, match="truncated"):
        state.load(p)


@pytest.mark.parametrize("storage", ["bf16", "fp32"])
def test_fast_mode_roundtrip(tmp_path, storage):
    cfg = ConsensusConfig(n_oracles=16, dimension=20, n_failing_oracles=2, n_admins=2)
    a = ConsensusService(cfg, 4, ADMINS[:2], [100 + i for i in range(16)], device="cpu", mode="fast",
                         storage=storage)
    a.engine.randomize(0)
    a.engine.run_round()
    p = os.path.join(tmp_path, "f.svoc")
    state.save(a, p)
    b = state.load(p)
    assert b.engine.storage == storage and b.engine.values.dtype == a.engine.values.dtype
    assert torch.equal(a.engine.values, b.engine.values)
    assert torch.equal(a.engine.consensus, b.engine.consensus)


def test_old_checkpoint_without_storage_key(tmp_path, monkeypatch):
    """A checkpoint from before the 'storage' meta key (only value_dtype) restores at its own dtype: an
    fp32 fast checkpoint is not silently narrowed to bf16."""
    import json
    assert state.storage_of({"value_dtype": "float32"}) == "fp32"
    assert state.storage_of({"value_dtype": "int32", "storage": "int32"}) == "int32"
    cfg = ConsensusConfig(n_oracles=16, dimension=20, n_failing_oracles=2, n_admins=2)
    a = ConsensusService(cfg, 4, ADMINS[:2], [100 + i for i in range(16)], device="cpu", mode="fast", storage="fp32")
    a.engine.randomize(0)
    a.engine.run_round()
    dumps = json.dumps
    monkeypatch.setattr(json, "dumps", lambda m, **k: dumps({x: y for x, y in m.items() if x != "storage"}, **k))
    p = os.path.join(tmp_path, "old.svoc")
    state.save(a, p)
    monkeypatch.setattr(json, "dumps", dumps)
    b = state.load(p)
    assert b.engine.storage == "fp32"
    assert torch.equal(a.engine.values, b.engine.values)


def _pending_engine_pair():
    cfg = ConsensusConfig(n_oracles=16, dimension=20, n_failing_oracles=2, n_admins=2)
    svc = ConsensusService(cfg, 4, ADMINS[:2], [100 + i for i in range(16)], device="cpu", mode="fast",
                           storage="fp32")
    svc.engine.randomize(0)
    svc.engine.run_round()
    return svc


def test_checkpoint_with_pending_batch_reverts_the_same(tmp_path):
    """apply_updates, checkpoint, reload, run_round: the reverted instance goes back to its pre-batch rows
    in the reloaded engine exactly as in the one that wrote the checkpoint (the rollback info
    used to live only in Python and was lost by a checkpoint)."""
    a = _pending_engine_pair()
    e = a.engine
    N, D = e.N, e.D
    before = e.values.clone()
    e.apply_updates(torch.full((N,), 1), torch.arange(N), torch.full((N, D), 0.5))   # instance 1: zero variance
    e.apply_updates(torch.tensor([0, 0]), torch.tensor([3, 4]), torch.rand(2, D, generator=torch.Generator().manual_seed(4)))
    p = os.path.join(tmp_path, "pending.svoc")
    state.save(a, p)
    b = state.load(p)
    for eng in (a.engine, b.engine):
        eng.run_round()
        assert eng.status[1].item() != 0 and eng.status[0].item() == 0
    assert torch.equal(a.engine.values, b.engine.values)
    assert torch.equal(a.engine.values[1], before[1])                 # reverted: pre-batch rows
    assert not torch.equal(a.engine.values[0], before[0])             # kept its update
    for k in ("enabled", "n_active", "consensus", "rel"):
        assert torch.equal(getattr(a.engine, k), getattr(b.engine, k)), k


def test_many_pending_batches_fold_into_one_preimage():
    """More than FOLD_AT batches before one round: the saved rows fold into one dense pre-image (bounded
    memory) and the revert still restores the state from before the FIRST batch, statuses included."""
    from svoc.engine import _PendingBatches
    a = _pending_engine_pair()
    e = a.engine
    N, D = e.N, e.D
    before = {k: getattr(e, k).clone() for k in ("values", "enabled", "n_active")}
    sts = []
    g = torch.Generator().manual_seed(5)
    for k in range(_PendingBatches.FOLD_AT + 3):
        # instance 2 collapses to one point over the batches (reverts); instance 3 gets ordinary rows
        sts.append(e.apply_updates(torch.tensor([2, 2, 3]), torch.tensor([k % N, (k + 5) % N, k % N]),
                                   torch.cat([torch.full((2, D), 0.5), torch.rand(1, D, generator=g)])))
    assert e._pending.dense is not None and len(e._pending.entries) < _PendingBatches.FOLD_AT
    e.values[2, :, :D] = 0.5                                           # (a direct write: every row of 2 at 0.5)
    e.touched[2] = 1
    e.run_round()
    assert e.status[2].item() != 0 and e.status[3].item() == 0
    # the batches' rows of instance 2 are back at the pre-image; the direct write to its other rows stands
    # (the unfolded path restores the same rows: ADVICE r5)
    hit = sorted({k % N for k in range(_PendingBatches.FOLD_AT + 3)} | {(k + 5) % N for k in range(_PendingBatches.FOLD_AT + 3)})
    rest = [i for i in range(N) if i not in hit]
    assert torch.equal(e.values[2, hit], before["values"][2, hit]) and torch.equal(e.enabled, before["enabled"])
    assert bool((e.values[2, rest, :D] == 0.5).all())
    assert torch.equal(e.n_active, before["n_active"])
    for st in sts:
        assert st[:2].tolist() == [e.status[2].item()] * 2 and st[2].item() == 0
    assert not e._pending
