"""fp32-storage fast kernel (csrc/kernels/consensus_fast_f32.hip): reference-resolution fast mode.

Checked against (1) the plain-PyTorch fp64/fp32 reference of the same round (svoc/ops/torch_ref.py),
(2) its CPU twin (reference_cpu.cpp fast_round_one over fp32 storage), (3) the EXACT wsad engine on
the same wsad data (reliable masks equal, consensus within one wsad ulp: SURVEY A.3), and (4) revert
atomicity: a reverted round leaves every committed output bitwise unchanged (contract.cairo:588-603).
"""
import pytest
import torch

from helpers import alloc_fast_out, beta_oracles, fast_work, run_exact, run_fast
from svoc import ops as svops
from svoc.ops import torch_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _f32(B, N, D, f, seed, a=20.0):
    x, _ = beta_oracles(B, N, D, f, a=a, seed=seed, dtype=torch.float32)
    return x


SHAPES = [(4, 3, 0), (7, 6, 2), (16, 33, 3), (50, 300, 5), (64, 1024, 8), (65, 129, 9), (100, 260, 10),
          (128, 512, 16), (200, 136, 20), (256, 600, 32), (33, 1, 4), (300, 70, 30), (512, 130, 64),
          (1000, 40, 100), (1024, 256, 128)]


@pytest.mark.parametrize("N,D,f", SHAPES)
@pytest.mark.parametrize("constrained", [True, False])
def test_f32_kernel_vs_torch(N, D, f, constrained):
    torch.manual_seed(N * 31 + D)
    B = 12
    x = _f32(B, N, D, f, seed=N + D)
    if not constrained:
        x = x * 4.0 - 1.5          # unconstrained: any finite values
    o = run_fast(x.to(DEV), D, f, constrained, 3.0)
    torch.cuda.synchronize()
    ref = torch_ref.fast_round(x[:, :, :D].to(DEV), f, constrained, 3.0)
    ok = o["status"] == 0
    assert ok.all(), o["status"]
    assert torch.equal(o["c1"], ref["c1"].float())        # medians of fp32 values: exact
    torch.testing.assert_close(o["qr"], ref["qr"].float(), rtol=2e-5, atol=1e-6)
    assert torch.equal(o["reliable"].bool(), ref["reliable"])
    if constrained:
        assert torch.equal(o["consensus"], ref["consensus"])
    else:
        torch.testing.assert_close(o["consensus"], ref["consensus"], rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(o["rel"], ref["rel"], rtol=1e-5, atol=1e-6)
    # fp32 shifted power sums, fp64 combination: ~1e-4 absolute on the moments (measured max 1.4e-4)
    torch.testing.assert_close(o["skew"], ref["skew"], rtol=1e-3, atol=5e-4)
    torch.testing.assert_close(o["kurt"], ref["kurt"], rtol=1e-3, atol=5e-4)


@pytest.mark.parametrize("N,D,f", [(7, 6, 2), (64, 257, 8), (256, 100, 32)])
def test_f32_kernel_vs_cpu_twin(N, D, f):
    B = 10
    x = _f32(B, N, D, f, seed=7 * N + D)
    g = run_fast(x.to(DEV), D, f, True)
    c = run_fast(x, D, f, True)
    torch.cuda.synchronize()
    for k in ("status", "c1", "consensus", "reliable"):
        assert torch.equal(g[k].cpu(), c[k]), k
    for k in ("qr", "rel"):
        torch.testing.assert_close(g[k].cpu(), c[k], rtol=1e-4, atol=1e-5)
    for k in ("skew", "kurt"):
        torch.testing.assert_close(g[k].cpu(), c[k], rtol=1e-3, atol=5e-4)


@pytest.mark.parametrize("N,D,f", [(64, 1024, 8), (256, 512, 32), (100, 77, 10), (512, 96, 64)])
def test_f32_agrees_with_exact_at_reference_resolution(N, D, f):
    """Same wsad data (1e-6 grid) through fast-fp32 and the exact engine: identical reliable masks,
    consensus within one wsad ulp, rel1 / rel2 within a few ulps (the contract truncates each product),
    moments within the fast-mode tolerance of SURVEY A.3.  Instances whose exact quadratic risks tie
    across the rank cut would be decided by values the modes round differently: none here (checked)."""
    B = 24
    x, _ = beta_oracles(B, N, D, f, seed=N * 3 + D, dtype=torch.float64)
    w = (x[:, :, :D] * 1e6).to(torch.int64).contiguous()
    xf = torch.zeros(B, N, (D + 7) // 8 * 8, dtype=torch.float32)
    xf[:, :, :D] = (w.double() / 1e6).float()
    fa = run_fast(xf.to(DEV), D, f, True)
    ex = run_exact(w.to(DEV, torch.int32), f, True)
    torch.cuda.synchronize()
    fa = {k: v.cpu() for k, v in fa.items()}
    ex = {k: v.cpu() for k, v in ex.items()}
    assert (ex["status"] == 0).all() and (fa["status"] == 0).all()
    srt = torch.sort(ex["qr"], dim=1).values
    assert (srt[:, N - f - 1] != srt[:, N - f]).all()
    assert torch.equal(fa["reliable"].bool(), ex["reliable"].bool())
    assert (fa["c1"].double() * 1e6 - ex["c1"].double()).abs().max().item() <= 1.0 + 1e-6
    cons = (fa["consensus"].double() * 1e6 - ex["consensus"].double()).abs()
    assert cons.max().item() <= 1.0 + 1e-6, cons.max()
    rel = (fa["rel"].double() * 1e6 - ex["rel"].double()).abs()
    assert rel.max().item() <= 32.0, rel.max()
    # moments: the contract truncates z to 1e-6 before cubing it (math.cairo:320-363), fast mode does not
    sk = (fa["skew"].double() - ex["skew"].double() / 1e6).abs()
    ku = (fa["kurt"].double() - ex["kurt"].double() / 1e6).abs()
    assert sk.max().item() < 2e-3 and ku.max().item() < 5e-3, (sk.max(), ku.max())


def test_f32_reverts_leave_outputs_untouched():
    """ZERO_VARIANCE, RELIABILITY_INTERVAL and TOO_FEW_RELIABLE on instances with committed outputs:
    every output tensor stays bitwise unchanged, statuses equal the CPU twin's."""
    B, N, D, f = 6, 64, 200, 8
    x = _f32(B, N, D, f, seed=3)
    xg = x.to(DEV)
    o = run_fast(xg, D, f, True)
    torch.cuda.synchronize()
    assert (o["status"] == 0).all()
    before = {k: v.clone() for k, v in o.items() if k != "status"}
    y = x.clone()
    y[1, :, 17] = 0.25                          # zero variance
    y[2, : N // 2 + 1, :D] = 0.0                # rel1 < 0
    y[2, N // 2 + 1:, :D] = 1.0
    yg = y.to(DEV)
    op = svops.ops().fast_round
    op(yg, None, D, f, True, 1.0, o["c1"], o["consensus"], o["skew"], o["kurt"], o["rel"], o["qr"], o["reliable"],
       o["status"], 0, 0, 0, False, fast_work(B, D, DEV))
    cpu = run_fast(y, D, f, True)
    torch.cuda.synchronize()
    assert torch.equal(o["status"].cpu(), cpu["status"])
    st = o["status"].cpu()
    assert st[1].item() != 0 and st[2].item() != 0 and (st[[0, 3, 4, 5]] == 0).all()
    bad = st != 0
    for k, v in before.items():
        assert torch.equal(o[k].cpu()[bad], v.cpu()[bad]), k
    # too few reliable: f = N - 3
    o2 = run_fast(xg, D, N - 3, True)
    torch.cuda.synchronize()
    assert (o2["status"].cpu() == run_fast(x, D, N - 3, True)["status"]).all()
    assert (o2["status"] != 0).all() and (o2["consensus"] == 0).all()


def test_f32_split_modes_match_whole_round():
    """Mode 1 (c1 + qr partials) / mode 2 (from the summed qr) on two column slices == the whole round
    (the two-network kernel, wave_hint -7: mode 2 reads nothing from mode 1 but c1 and the qr)."""
    B, N, D, f = 8, 100, 300, 10
    x = _f32(B, N, D, f, seed=11)[:, :, :D].contiguous()
    whole = run_fast(x.to(DEV), D, f, True)
    cut = 152
    parts = [x[:, :, :cut].contiguous().to(DEV), x[:, :, cut:].contiguous().to(DEV)]
    outs = [alloc_fast_out(B, N, p.shape[2], DEV) for p in parts]
    op = svops.ops().fast_round
    for p, o in zip(parts, outs):
        op(p, None, p.shape[2], f, True, 1.0, o["c1"], o["consensus"], o["skew"], o["kurt"], o["rel"], o["qr"],
           o["reliable"], o["status"], -7, 1, D, False, None)
    qr = outs[0]["qr"] + outs[1]["qr"]
    for p, o in zip(parts, outs):
        o["qr"].copy_(qr)
        op(p, None, p.shape[2], f, True, 1.0, o["c1"], o["consensus"], o["skew"], o["kurt"], o["rel"], o["qr"],
           o["reliable"], o["status"], -7, 2, D, False, fast_work(B, p.shape[2], DEV))
    torch.cuda.synchronize()
    for o in outs:
        assert (o["status"] == 0).all()
        assert torch.equal(o["reliable"], whole["reliable"])
        torch.testing.assert_close(o["rel"], whole["rel"], rtol=1e-5, atol=1e-6)
    for k in ("c1", "consensus"):
        assert torch.equal(torch.cat([outs[0][k], outs[1][k]], 1), whole[k]), k


def test_engine_fp32_storage_gpu():
    """ConsensusEngine(storage="fp32") on the GPU: updates, rounds, getters; agrees with the CPU engine."""
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    cfg = ConsensusConfig(n_oracles=32, dimension=100, n_failing_oracles=4, constrained=True)
    eg = ConsensusEngine(cfg, 16, device=DEV, mode="fast", storage="fp32")
    ec = ConsensusEngine(cfg, 16, device="cpu", mode="fast", storage="fp32")
    torch.manual_seed(0)
    vals = torch.rand(16 * 32, 100)
    inst = torch.arange(16).repeat_interleave(32)
    orc = torch.arange(32).repeat(16)
    for e in (eg, ec):
        st = e.step(inst, orc, vals)
        assert (st.cpu() == 0).all()
    torch.cuda.synchronize()
    assert eg.values.dtype == torch.float32 and bool(eg.consensus_active.all())
    for k in ("status", "reliable", "consensus", "c1"):
        assert torch.equal(getattr(eg, k).cpu(), getattr(ec, k)), k
    torch.testing.assert_close(eg.rel.cpu(), ec.rel, rtol=1e-5, atol=1e-6)


# ----------------------------------------------------------------------------------------------------
# One-network window kernel (consensus_fast_winf.hip): the default for N <= 256, f <= 32.  Cross-checked
# against the two-network fp32 kernel (wave_hint -7) and the PyTorch reference.

WIN_SHAPES = [(256, 4096, 32), (256, 300, 32), (64, 1024, 8), (64, 100, 8), (200, 136, 20), (128, 512, 16),
              (100, 260, 10), (33, 70, 4), (7, 6, 2), (256, 1000, 5), (250, 129, 31), (65, 129, 9)]


@pytest.mark.parametrize("N,D,f", WIN_SHAPES)
@pytest.mark.parametrize("constrained", [True, False])
def test_f32_window_matches_two_network_kernel(N, D, f, constrained):
    B = 6 if D >= 1000 else 12
    x = _f32(B, N, D, f, seed=N * 7 + D + f)
    if not constrained:
        x = x * 4.0 - 1.5
    xg = x.to(DEV)
    w = run_fast(xg, D, f, constrained, 3.0)
    t = run_fast(xg, D, f, constrained, 3.0, wave_hint=-7)
    ref = torch_ref.fast_round(x[:, :, :D].to(DEV), f, constrained, 3.0)
    torch.cuda.synchronize()
    assert (w["status"] == 0).all() and (t["status"] == 0).all(), (w["status"], t["status"])
    for k in ("c1", "reliable"):
        assert torch.equal(w[k], t[k]), k
    assert torch.equal(w["c1"], ref["c1"].float())
    assert torch.equal(w["reliable"].bool(), ref["reliable"])
    if constrained:
        assert torch.equal(w["consensus"], t["consensus"])
        assert torch.equal(w["consensus"], ref["consensus"])
    else:
        torch.testing.assert_close(w["consensus"], ref["consensus"], rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(w["qr"], t["qr"], rtol=2e-5, atol=1e-6)
    torch.testing.assert_close(w["rel"], ref["rel"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(w["skew"], ref["skew"], rtol=1e-3, atol=5e-4)
    torch.testing.assert_close(w["kurt"], ref["kurt"], rtol=1e-3, atol=5e-4)


@pytest.mark.parametrize("cancel", ["0.5", "1e30"])
def test_f32_window_cleanup_path(cancel, monkeypatch):
    """SVOC_WIN_CANCEL=0.5 sends every column through the exact two-pass recomputation, 1e30 none: both
    agree with the PyTorch reference (the cleanup is the cancellation guard of the all-minus-removed
    power sums)."""
    monkeypatch.setenv("SVOC_WIN_CANCEL", cancel)
    B, N, D, f = 8, 256, 700, 32
    x = _f32(B, N, D, f, seed=5)
    o = run_fast(x.to(DEV), D, f, True)
    ref = torch_ref.fast_round(x[:, :, :D].to(DEV), f, True)
    torch.cuda.synchronize()
    assert (o["status"] == 0).all()
    assert torch.equal(o["consensus"], ref["consensus"])
    torch.testing.assert_close(o["skew"], ref["skew"], rtol=1e-3, atol=5e-4)
    torch.testing.assert_close(o["kurt"], ref["kurt"], rtol=1e-3, atol=5e-4)


def test_f32_window_zero_variance_and_mixed_signed_zero():
    """A constant reliable column (also one mixing +0.0 and -0.0: equal values) reverts the window round
    with ZERO_VARIANCE, as the two-network kernel does; outputs stay untouched."""
    B, N, D, f = 4, 256, 300, 32
    x = _f32(B, N, D, f, seed=9)
    x[1, :, 40] = 0.375
    x[2, :, 7] = 0.0
    x[2, ::2, 7] = -0.0
    xg = x.to(DEV)
    w = run_fast(xg, D, f, True)
    t = run_fast(xg, D, f, True, wave_hint=-7)
    torch.cuda.synchronize()
    assert torch.equal(w["status"], t["status"])
    st = w["status"].cpu()
    assert st[1].item() != 0 and st[2].item() != 0 and st[0].item() == 0 and st[3].item() == 0


def test_f32_window_split_modes_match_whole_round():
    """D-sharded halves (mode 1 / mode 2 with a persistent workspace) through the window kernel."""
    B, N, D, f = 6, 256, 520, 32
    x = _f32(B, N, D, f, seed=13)[:, :, :D].contiguous()
    whole = run_fast(x.to(DEV), D, f, True)
    cut = 264
    parts = [x[:, :, :cut].contiguous().to(DEV), x[:, :, cut:].contiguous().to(DEV)]
    outs = [alloc_fast_out(B, N, p.shape[2], DEV) for p in parts]
    works = [fast_work(B, p.shape[2], DEV) for p in parts]
    op = svops.ops().fast_round
    for p, o, w in zip(parts, outs, works):
        op(p, None, p.shape[2], f, True, 1.0, o["c1"], o["consensus"], o["skew"], o["kurt"], o["rel"], o["qr"],
           o["reliable"], o["status"], 0, 1, D, False, w)
    qr = outs[0]["qr"] + outs[1]["qr"]
    for p, o, w in zip(parts, outs, works):
        o["qr"].copy_(qr)
        op(p, None, p.shape[2], f, True, 1.0, o["c1"], o["consensus"], o["skew"], o["kurt"], o["rel"], o["qr"],
           o["reliable"], o["status"], 0, 2, D, False, w)
    torch.cuda.synchronize()
    for o in outs:
        assert (o["status"] == 0).all()
        assert torch.equal(o["reliable"], whole["reliable"])
    for k in ("c1", "consensus"):
        assert torch.equal(torch.cat([outs[0][k], outs[1][k]], 1), whole[k]), k


# ----------------------------------------------------------------------------------------------------
# N = 256: the pruned window network (middle 32 keys per lane, exact check, full-network fallback per
# wave: sortnet.hpp window_group_pruned).  Adversarial columns force the fallback; results stay exact.

def _pruned_round(x, D, f):
    B, N = x.shape[:2]
    o = alloc_fast_out(B, N, D, DEV)
    stats = torch.zeros(1, dtype=torch.int32, device=DEV)
    svops.ops().fast_round(x, None, D, f, True, 1.0, o["c1"], o["consensus"], o["skew"], o["kurt"], o["rel"],
                           o["qr"], o["reliable"], o["status"], 0, 0, 0, False, None, stats)
    return o, stats


@pytest.mark.parametrize("pattern", ["random", "sorted_rows", "one_lane_low", "ties", "signed_zero", "two_values"])
def test_f32_pruned_window_exact(pattern):
    B, N, D, f = 6, 256, 1024, 32
    x = _f32(B, N, D, f, seed=77)[:, :, :D].contiguous()
    if pattern == "sorted_rows":        # each column ascending in the row index: lane 0 holds the lowest 64
        x = torch.sort(x, dim=1).values
    elif pattern == "one_lane_low":     # rows 0..63 (segment 0) pushed below everything in half the columns
        x[:, :64, ::2] *= 0.01
    elif pattern == "ties":             # 9 distinct values per column: the window is full of ties
        x = torch.round(x * 8) / 8
    elif pattern == "signed_zero":      # many +0.0 / -0.0 around a low median
        x = torch.where(x < 0.55, torch.zeros_like(x), x)
        x[:, ::3] = -x[:, ::3]
        x = torch.where(x < 0, torch.zeros_like(x), x)        # (-0.0 from the negation of +0.0 stays)
        x[:, 1::3, 5] = -0.0
    elif pattern == "two_values":
        x = torch.where(x < 0.5, torch.full_like(x, 0.25), torch.full_like(x, 0.75))
    xg = x.to(DEV)
    o, stats = _pruned_round(xg, D, f)
    ref = torch_ref.fast_round(xg, f, True, 1.0)
    full = run_fast(xg, D, f, True, wave_hint=-7)          # the two-network kernel (no pruning)
    torch.cuda.synchronize()
    st = o["status"]
    assert torch.equal(st, full["status"]), (st, full["status"])
    ok = st == 0
    if pattern != "two_values":
        assert ok.all(), st
    assert torch.equal(o["c1"][ok], ref["c1"].float()[ok])
    assert torch.equal(o["reliable"][ok].bool(), ref["reliable"][ok])
    assert torch.equal(o["consensus"][ok], ref["consensus"][ok])
    assert torch.equal(o["consensus"][ok], full["consensus"][ok])
    fb = int(stats.item())
    slabs = B * (D // 64) * 4                                    # (instances x slab steps x waves)
    if pattern == "random":
        assert fb <= slabs // 20, (fb, slabs)                    # exchangeable rows: a few percent at most
    if pattern in ("sorted_rows", "one_lane_low"):
        assert fb > 0, fb                                        # the check must have caught these


def test_f32_pruned_window_engine_counter():
    """The engine passes its counter; c3-like random data falls back on < 5 % of the slab networks."""
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    cfg = ConsensusConfig(n_oracles=256, dimension=2048, n_failing_oracles=32, constrained=True)
    e = ConsensusEngine(cfg, batch=16, device=DEV, mode="fast", storage="fp32")
    e.randomize(seed=2)
    e.run_round()
    torch.cuda.synchronize()
    assert (e.status == 0).all()
    st = e.net_stats()
    assert st["slab_networks"] == 16 * (2048 // 64) * 4
    assert st["fallbacks"] <= 0.05 * st["slab_networks"], st
