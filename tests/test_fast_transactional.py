"""Transactional fast streaming: a coalesced batch whose round reverts leaves no trace.

The reference's update_prediction is one transaction -- store the prediction, then the consensus round;
any failed assert of the round reverts the store too (contract.cairo:588-603 -> :442-503, :331-343).
The fast engine coalesces a batch per instance, so a reverting round restores that instance's stored
rows, ``enabled`` flags and ``n_active`` to their pre-batch state (the update kernels saved the rows
they overwrote), and every update of the batch reports the round's code.  Instances whose round
succeeds keep their updates.
"""
import pytest
import torch

from svoc.config import ConsensusConfig
from svoc.engine import ConsensusEngine
from svoc.status import Status

DEVS = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _engine(dev, storage="fp32", N=64, D=256, f=8, B=4):
    cfg = ConsensusConfig(n_oracles=N, dimension=D, n_failing_oracles=f, constrained=True)
    return ConsensusEngine(cfg, batch=B, device=dev, mode="fast", storage=storage)


def _snap(e):
    e.pipeline_join()
    return {k: getattr(e, k).clone() for k in ("values", "enabled", "n_active", "consensus", "rel", "skew", "kurt",
                                               "reliable", "c1")}


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("storage", ["fp32", "bf16"])
def test_reverted_batch_restores_rows(dev, storage):
    e = _engine(dev, storage)
    e.randomize(seed=5)
    e.run_round()
    before = _snap(e)
    N, D = e.N, e.D
    # instance 2: every oracle -> one point (zero variance: the round reverts); instance 0: 3 fresh rows
    inst = torch.tensor([2] * N + [0, 0, 0], device=dev)
    orc = torch.cat([torch.arange(N), torch.tensor([5, 9, 11])]).to(dev)
    vals = torch.full((N + 3, D), 0.5, device=dev)
    vals[N:] = torch.rand(3, D, generator=torch.Generator().manual_seed(1)).to(dev)
    st = e.step(inst, orc, vals)
    e.pipeline_join()
    if dev == "cuda":
        torch.cuda.synchronize()
    assert e.status[2].item() == int(Status.ZERO_VARIANCE) and e.status[0].item() == 0
    assert st[:N].cpu().tolist() == [int(Status.ZERO_VARIANCE)] * N     # the tx status is the round's
    assert st[N:].cpu().tolist() == [0, 0, 0]
    after = _snap(e)
    for k in ("values", "consensus", "rel", "skew", "kurt", "reliable", "c1"):
        assert torch.equal(after[k][2], before[k][2]), k                # instance 2: no trace
    assert torch.equal(after["enabled"], before["enabled"]) and torch.equal(after["n_active"], before["n_active"])
    # instance 0 kept its updates; the untouched instances kept everything
    assert torch.equal(after["values"][0, [5, 9, 11], :D], vals[N:].to(after["values"].dtype))
    assert torch.equal(after["values"][1], before["values"][1]) and torch.equal(after["values"][3], before["values"][3])


@pytest.mark.parametrize("dev", DEVS)
def test_reverted_activation_restores_enabled_and_n_active(dev):
    """The batch that activates an instance (first commit of every oracle) reverts: enabled / n_active
    go back to zero, the rows to their constructor zeros (contract.cairo:106-120, 331-343)."""
    e = _engine(dev, B=2)
    N, D = e.N, e.D
    inst = torch.zeros(N, dtype=torch.long, device=dev)
    vals = torch.full((N, D), 0.25, device=dev)
    st = e.step(inst, torch.arange(N, device=dev), vals)
    e.pipeline_join()
    assert e.status[0].item() == int(Status.ZERO_VARIANCE)
    assert (st.cpu() == int(Status.ZERO_VARIANCE)).all()
    assert e.n_active.cpu().tolist() == [0, 0] and int(e.enabled.sum()) == 0
    assert int(e.values.abs().sum()) == 0
    # an instance that does not become fully active keeps its stored rows (no round, no revert)
    st2 = e.step(torch.ones(3, dtype=torch.long, device=dev), torch.tensor([0, 1, 2], device=dev),
                 torch.full((3, D), 0.25, device=dev))
    e.pipeline_join()
    assert st2.cpu().tolist() == [0, 0, 0] and e.n_active.cpu().tolist() == [0, 3]


@pytest.mark.parametrize("dev", DEVS)
def test_two_batches_before_one_round(dev):
    """Two apply_updates calls, one round: the revert restores the state from before the FIRST batch,
    the same slot overwritten by both batches included."""
    e = _engine(dev)
    e.randomize(seed=9)
    e.run_round()
    before = _snap(e)
    N, D = e.N, e.D
    e.apply_updates(torch.full((N,), 1, device=dev), torch.arange(N, device=dev), torch.full((N, D), 0.75, device=dev))
    e.apply_updates(torch.tensor([1, 1], device=dev), torch.tensor([3, 4], device=dev),
                    torch.full((2, D), 0.75, device=dev))
    e.run_round()
    e.pipeline_join()
    assert e.status[1].item() == int(Status.ZERO_VARIANCE)
    after = _snap(e)
    for k in before:
        assert torch.equal(after[k], before[k]), k


def test_non_transactional_keeps_rows():
    """transactional=False: the round-3 behaviour (coalesced rows stay, outputs untouched)."""
    e = _engine("cpu")
    e.transactional = False
    e.randomize(seed=5)
    e.run_round()
    N, D = e.N, e.D
    e.step(torch.full((N,), 2), torch.arange(N), torch.full((N, D), 0.5))
    assert e.status[2].item() == int(Status.ZERO_VARIANCE)
    assert bool((e.values[2, :, :D] == 0.5).all())


@pytest.mark.gpu
@pytest.mark.parametrize("overlap", [False, True])
@pytest.mark.parametrize("storage,D", [("fp32", 512), ("fp32", 1000), ("bf16", 512)])
def test_pipelined_step_restores_reverted_instances(overlap, storage, D):
    """step_pipelined (per-range update + round + rollback on side streams: the fused fp32 path, the bf16
    window kernel's in-kernel rollback) == step() (update kernel, round, restore kernel) on a batch where
    some instances revert (eager and overlapped across steps; D = 1000: fp32 rows of 250 16-B chunks, not a
    multiple of the commit kernel's 64 lanes)."""
    N, B = 64, 8
    U = N                            # every oracle of every instance publishes
    ref, pipe = _engine("cuda", storage, N=N, D=D, B=B), _engine("cuda", storage, N=N, D=D, B=B)
    if storage == "bf16":
        assert pipe._kernel_rollback_ok(U)
    for e in (ref, pipe):
        e.randomize(seed=3)
        e.run_round()
    g = torch.Generator(device="cuda").manual_seed(0)
    inst = torch.arange(B, device="cuda").repeat_interleave(U)
    orc = torch.stack([torch.randperm(N, device="cuda", generator=g) for _ in range(B)]).reshape(-1)
    vals = torch.rand(B * U, D, device="cuda", generator=g)
    vals[3 * U:4 * U] = 0.5          # instance 3: one point -> zero variance, the round reverts
    ref.step(inst, orc, vals)
    pipe.step_pipelined(inst, orc, vals, U, chunks=2, overlap=overlap)
    pipe.pipeline_join()
    torch.cuda.synchronize()
    assert torch.equal(pipe.status, ref.status)
    assert pipe.status[3].item() == int(Status.ZERO_VARIANCE) and int((pipe.status == 0).sum()) == B - 1
    for k in ("values", "enabled", "n_active", "consensus", "rel", "c1"):
        assert torch.equal(getattr(pipe, k), getattr(ref, k)), k


@pytest.mark.gpu
@pytest.mark.parametrize("storage,N,D,f,U", [("fp32", 256, 1024, 32, 64), ("fp32", 64, 700, 8, 16),
                                             ("fp32", 200, 300, 20, 50)])
def test_fused_streaming_matches_generic_path(storage, N, D, f, U):
    """The fused transactional step (window kernel reading the updated rows from the batch + commit kernel)
    equals the generic transactional path (update kernel with saved rows + round + restore) bit for bit:
    state, outputs, update statuses -- with a reverting instance (zero variance) and an instance whose
    batch holds an invalid row (interval error: that update alone reverts, the round runs without it)."""
    B = 6
    cfg = ConsensusConfig(n_oracles=N, dimension=D, n_failing_oracles=f, constrained=True)
    fz = ConsensusEngine(cfg, batch=B, device="cuda", mode="fast", storage=storage)
    gen = ConsensusEngine(cfg, batch=B, device="cuda", mode="fast", storage=storage)
    for e in (fz, gen):
        e.randomize(seed=N + D)
        e.run_round()
    g = torch.Generator(device="cuda").manual_seed(3)
    inst = torch.arange(B, device="cuda").repeat_interleave(U)
    orc = torch.stack([torch.randperm(N, device="cuda", generator=g)[:U] for _ in range(B)]).reshape(-1)
    vals = torch.rand(B * U, D, device="cuda", generator=g).to(fz.vdtype)
    assert fz._fused_ok(inst, orc, vals, U)
    # instance 1: an update row with 1.5 in one column (rejected alone); instance 4: all its updated rows at
    # one value and the rest of the column too -> zero variance in column 3 if U == N, else a plain round
    vals[1 * U + 2, D // 2] = 1.5
    # instance 2: two updates name no oracle (one of them with an out-of-interval row as well): the first
    # reports NOT_ORACLE, the second INTERVAL_INPUT (the contract checks the interval first), neither is stored
    orc[2 * U + 1] = N + 5
    orc[2 * U + 3] = -1
    vals[2 * U + 3, 0] = 2.0
    # instance 3: a negative value (rejected) and a -0.0 (inside the interval: accepted) in two update rows
    # (the N = 256 kernel takes the rows' interval extremes from its sorted keys)
    vals[3 * U + 1, 5] = -0.25
    vals[3 * U + 4, 7] = -0.0
    fz.values[4, :, 3] = 0.625
    gen.values[4, :, 3] = 0.625
    vals[4 * U:5 * U, 3] = 0.625
    fz.step_pipelined(inst, orc, vals, U, chunks=2, overlap=False)
    st_f = fz._status_buffer(B * U).clone()
    gen._all_active = False      # force the generic path (update kernel + saved rows + restore)
    gen._fused_ok = lambda *a: False
    gen.step_pipelined(inst, orc, vals, U, chunks=2, overlap=False)
    st_g = gen._save_bufs[("pipe",)][2][:B * U].clone()
    torch.cuda.synchronize()
    assert torch.equal(st_f, st_g), (st_f.view(B, U), st_g.view(B, U))
    assert st_f[1 * U + 2].item() == int(Status.INTERVAL_INPUT)
    assert st_f[2 * U + 1].item() == int(Status.NOT_ORACLE) and st_f[2 * U + 3].item() == int(Status.INTERVAL_INPUT)
    assert st_f[3 * U + 1].item() == int(Status.INTERVAL_INPUT) and st_f[3 * U + 4].item() == int(Status.OK)
    assert fz.status[4].item() == int(Status.ZERO_VARIANCE)
    for k in ("status", "values", "enabled", "n_active", "consensus", "rel", "c1", "reliable", "skew", "kurt", "qr"):
        a, b_ = getattr(fz, k), getattr(gen, k)
        if not torch.equal(a, b_):
            bad = (a != b_).reshape(B, -1)
            rows = bad.any(1).nonzero().flatten().tolist()
            cols = bad.nonzero()[:8].tolist()
            raise AssertionError(f"{k}: instances {rows}, first (inst, col) {cols}, "
                                 f"{a.reshape(B, -1)[bad][:4].tolist()} vs {b_.reshape(B, -1)[bad][:4].tolist()}")


@pytest.mark.gpu
@pytest.mark.parametrize("N,D,f,U", [(256, 1024, 32, 64), (64, 700, 8, 16), (200, 300, 20, 50)])
def test_bf16_kernel_rollback_matches_restore_kernel(N, D, f, U):
    """bf16 pipelined step: the window kernel's in-kernel rollback (FastParams.rst_saved) equals the restore
    kernel after the round bit for bit -- state, enabled / n_active, outputs, update statuses -- with
    reverting instances (zero variance) among succeeding ones."""
    B = 6
    cfg = ConsensusConfig(n_oracles=N, dimension=D, n_failing_oracles=f, constrained=True)
    kr = ConsensusEngine(cfg, batch=B, device="cuda", mode="fast", storage="bf16")
    rk = ConsensusEngine(cfg, batch=B, device="cuda", mode="fast", storage="bf16")
    for e in (kr, rk):
        e.randomize(seed=N + D)
        e.run_round()
    rk._kernel_rollback_ok = lambda U: False
    g = torch.Generator(device="cuda").manual_seed(5)
    inst = torch.arange(B, device="cuda").repeat_interleave(U)
    orc = torch.stack([torch.randperm(N, device="cuda", generator=g)[:U] for _ in range(B)]).reshape(-1)
    vals = torch.rand(B * U, D, device="cuda", generator=g)
    for e in (kr, rk):                 # instances 1 and 4: one column constant -> zero variance (revert)
        e.values[1, :, 3] = 0.625
        e.values[4, :, 7] = 0.25
    vals[1 * U:2 * U, 3] = 0.625
    vals[4 * U:5 * U, 7] = 0.25
    for e in (kr, rk):
        e.step_pipelined(inst, orc, vals, U, chunks=2, overlap=False)
    torch.cuda.synchronize()
    st_k = kr._save_bufs[("pipe",)][2][:B * U]
    st_r = rk._save_bufs[("pipe",)][2][:B * U]
    assert torch.equal(st_k, st_r)
    assert kr.status[1].item() == int(Status.ZERO_VARIANCE) and kr.status[4].item() == int(Status.ZERO_VARIANCE)
    assert (st_k.view(B, U)[1] == int(Status.ZERO_VARIANCE)).all()
    for k in ("status", "values", "enabled", "n_active", "consensus", "rel", "c1", "reliable", "skew", "kurt", "qr"):
        assert torch.equal(getattr(kr, k), getattr(rk, k)), k


@pytest.mark.gpu
@pytest.mark.parametrize("storage", ["fp32", "bf16"])
def test_pipelined_step_takes_host_batches(storage):
    """step_pipelined with the batch on the host (int32 indices, float64 rows): converted to the state's
    device and dtypes before any kernel reads it -- the same result as the device batch."""
    N, D, B, U = 64, 256, 4, 16
    dev_e, host_e = _engine("cuda", storage, N=N, D=D, B=B), _engine("cuda", storage, N=N, D=D, B=B)
    for e in (dev_e, host_e):
        e.randomize(seed=11)
        e.run_round()
    g = torch.Generator().manual_seed(2)
    inst = torch.arange(B).repeat_interleave(U)
    orc = torch.stack([torch.randperm(N, generator=g)[:U] for _ in range(B)]).reshape(-1)
    vals = torch.rand(B * U, D, generator=g, dtype=torch.float64)
    dev_e.step_pipelined(inst.cuda(), orc.cuda(), vals.cuda().to(dev_e.vdtype), U, chunks=2)
    host_e.step_pipelined(inst.int(), orc.int(), vals, U, chunks=2)
    dev_e.pipeline_join()
    host_e.pipeline_join()
    torch.cuda.synchronize()
    for k in ("status", "values", "enabled", "n_active", "consensus", "rel", "c1"):
        assert torch.equal(getattr(dev_e, k), getattr(host_e, k)), k


@pytest.mark.gpu
def test_kernels_reject_host_index_tensors():
    """The update / restore / commit bindings refuse index tensors that are not on the state's device
    (a host pointer handed to a GPU kernel)."""
    from svoc import ops as svops
    e = _engine("cuda", "fp32", N=16, D=64, B=2)
    e.randomize(seed=1)
    o = svops.ops()
    rows = torch.rand(2, 64, device="cuda")
    st = torch.zeros(2, dtype=torch.int32, device="cuda")
    with pytest.raises(RuntimeError, match="must be on|device"):
        o.commit_updates(rows, torch.tensor([0, 1]), st, e.values, 1)
    with pytest.raises(RuntimeError, match="must be on|device"):
        o.apply_updates(e.values, e.enabled, e.n_active, e.touched, e._winner, torch.tensor([0, 1]),
                        torch.tensor([0, 1], device="cuda"), rows, True, st, True, None, None)


def test_restore_kernel_inactive_status_cpu_twin():
    """restore_updates (the CPU twin of updates.hip upd_restore_kernel): reverted instances get their rows, enabled
    flag and n_active back and the round's code; with inactive_status >= 0 the updates of an instance whose round
    did not run keep their row and report that status (the exact engine's NOT_ACTIVE); -1 keeps OK."""
    from svoc import ops as svops
    B, N, D = 3, 4, 2
    vals = torch.arange(B * N * D, dtype=torch.int32).reshape(B, N, D).clone()
    enabled = torch.ones(B, N, dtype=torch.uint8)
    enabled[2, 1] = 0
    n_active = enabled.sum(1).to(torch.int32)
    inst = torch.tensor([0, 1, 2], dtype=torch.int64)
    oracle = torch.tensor([1, 2, 3], dtype=torch.int64)
    saved = torch.full((3, D), -7, dtype=torch.int32)
    saved_en = torch.tensor([1, 0, 1], dtype=torch.uint8)
    status = torch.tensor([int(Status.OK), int(Status.DIV_BY_ZERO), int(Status.OK)], dtype=torch.int32)
    active = torch.tensor([1, 1, 0], dtype=torch.uint8)   # instance 2: not fully active, no round
    for inactive, want2 in ((-1, int(Status.OK)), (int(Status.NOT_ACTIVE), int(Status.NOT_ACTIVE))):
        v, en, na = vals.clone(), enabled.clone(), n_active.clone()
        st = torch.zeros(3, dtype=torch.int32)
        svops.ops().restore_updates(v, en, na, inst, oracle, st, saved, saved_en, status, active, inactive)
        assert st.tolist() == [int(Status.OK), int(Status.DIV_BY_ZERO), want2]
        assert v[1, 2].tolist() == [-7, -7] and int(en[1, 2]) == 0 and int(na[1]) == n_active[1] - 1
        assert torch.equal(v[0], vals[0]) and torch.equal(v[2], vals[2])
