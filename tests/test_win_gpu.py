"""One-network window kernel (csrc/kernels/consensus_fast_win.hip) on a real MI355X.

The pass-2 smooth median comes from the pass-1 order-statistic window and the sorted removed keys, the
reliable moments from all-row minus removed-row power sums.  Checked against the two-network register
kernel (wave_hint -7: same order statistics -> bit-identical consensus, qr, rel, mask) and the plain
PyTorch fp32 reference (svoc/ops/torch_ref.py)."""
import pytest
import torch

from helpers import alloc_fast_out, beta_oracles, fast_work, run_fast
from svoc import ops as svops
from svoc.ops import torch_ref
from test_ops_gpu import _cmp_fast

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _both(x, D, f, cons, ms=1.0, legacy=False):
    win = run_fast(x, D, f, cons, ms, legacy=legacy)          # default: window kernel (temp workspace)
    reg = run_fast(x, D, f, cons, ms, wave_hint=-7, legacy=legacy)
    torch.cuda.synchronize()
    return win, reg


def _same(win, reg, constrained=True):
    """Same order statistics -> identical c1 / mask / constrained consensus; qr, rel, the moments and the
    unconstrained mean differ in rounding only (shift c1 here, first reliable row there)."""
    assert torch.equal(win["status"], reg["status"])
    ok = win["status"] == 0
    for k in ("c1", "reliable") + (("consensus",) if constrained else ()):
        assert torch.equal(win[k][ok], reg[k][ok]), k
    # qr: same terms, last-bit freedom in the compiler's FMA contraction of (x - c)^2 sums
    torch.testing.assert_close(win["qr"][ok], reg["qr"][ok], rtol=2e-6, atol=0)
    torch.testing.assert_close(win["rel"][ok], reg["rel"][ok], rtol=1e-6, atol=1e-7)
    if not constrained:
        torch.testing.assert_close(win["consensus"][ok], reg["consensus"][ok], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(win["skew"][ok], reg["skew"][ok], rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(win["kurt"][ok], reg["kurt"][ok], rtol=1e-3, atol=2e-3)
    return ok


_SHAPES = [(17, 40, 2), (33, 130, 4), (50, 300, 5), (64, 1024, 8), (64, 1000, 0), (63, 7, 1), (65, 96, 8),
           (100, 260, 10), (128, 512, 16), (129, 33, 32), (200, 136, 20), (255, 300, 31), (256, 4096, 32),
           (256, 600, 17), (256, 1, 3), (24, 8, 15)]


@pytest.mark.parametrize("N,D,f", _SHAPES)
@pytest.mark.parametrize("constrained", [True, False])
def test_win_vs_reg_and_torch(N, D, f, constrained):
    B = 10
    x, _ = beta_oracles(B, N, D, f, seed=3 * N + D + f)
    xg = x.to(DEV)
    win, reg = _both(xg, D, f, constrained)
    ok = _same(win, reg, constrained)
    assert ok.any(), win["status"]
    r = torch_ref.fast_round(xg[:, :, :D], f, constrained, 1.0)
    _cmp_fast(win, r, ok)


@pytest.mark.parametrize("N,f,levels", [(64, 8, 3), (256, 32, 5), (100, 13, 2), (200, 32, 9), (40, 6, 1)])
def test_win_ties(N, f, levels):
    """Heavily tied columns (few distinct values): the window/removed-key ranking is exact under ties."""
    B, D = 16, 200
    g = torch.Generator().manual_seed(N + levels)
    x = torch.zeros(B, N, 200, dtype=torch.bfloat16)
    x[:, :, :D] = (torch.randint(0, levels + 1, (B, N, D), generator=g).float() / max(levels, 1) * 0.5 + 0.25)
    xg = x.to(DEV)
    win, reg = _both(xg, D, f, True)
    assert torch.equal(win["status"], reg["status"])
    ok = win["status"] == 0
    for k in ("consensus", "reliable"):
        assert torch.equal(win[k][ok], reg[k][ok]), k
    r = torch_ref.fast_round(xg[:, :, :D], f, True, 1.0)
    ok = ok & (r["status"] == 0) if "status" in r else ok
    torch.testing.assert_close(win["consensus"][ok], r["consensus"][ok], rtol=0, atol=2e-6)


def test_win_cancellation_cleanup():
    """Honest rows almost equal, removed rows far away: the all-minus-removed power sums would cancel,
    so those columns are recomputed exactly over the reliable rows by win_cleanup_kernel."""
    B, N, D, f = 8, 256, 300, 32
    g = torch.Generator().manual_seed(5)
    base = 0.5 + 0.01 * torch.rand(B, 1, D, generator=g)
    x = torch.zeros(B, N, 304, dtype=torch.bfloat16)
    vals = base + 0.002 * torch.randn(B, N, D, generator=g)
    vals[:, :f] = torch.where(torch.rand(B, f, D, generator=g) < 0.5, 0.05, 0.95)
    x[:, :, :D] = vals.clamp(0, 1)
    xg = x.to(DEV)
    win, reg = _both(xg, D, f, True)
    ok = _same(win, reg)
    assert ok.any()


def test_win_zero_variance_flag():
    B, N, D, f = 4, 128, 64, 16
    x = torch.full((B, N, 64), 0.5, dtype=torch.bfloat16)
    x[:, :f, :] = 0.25
    x[1, :, 3] = torch.linspace(0.3, 0.7, N).to(torch.bfloat16)   # instance 1: one varying column
    xg = x.to(DEV)
    win, reg = _both(xg, D, f, True)
    assert torch.equal(win["status"], reg["status"])
    assert int(win["status"][0]) == 32      # ZERO_VARIANCE: the round reverts


def test_win_zero_variance_mixed_signed_zero():
    """A reliable column of +0.0 and -0.0 (equal values, different sort keys) is zero variance: the
    window kernel's pre-check compares window bounds as values, so it reverts like the reg kernel."""
    B, N, D, f = 4, 256, 128, 32
    x, _ = beta_oracles(B, N, D, f, seed=21)
    x[2, :, 9] = 0.0
    x[2, ::2, 9] = -0.0
    xg = x.to(DEV)
    win, reg = _both(xg, D, f, True)
    assert torch.equal(win["status"], reg["status"])
    assert int(win["status"][2]) == 32 and int(win["status"][0]) == 0


def test_win_legacy():
    x, _ = beta_oracles(6, 100, 200, 10, seed=1)
    xg = x.to(DEV)
    win, reg = _both(xg, 200, 10, True, legacy=True)
    ok = _same(win, reg)
    assert (win["skew"][ok] == 0).all() and (win["kurt"][ok] == 0).all()


def test_win_unconstrained_wide_range():
    B, N, D, f = 6, 96, 150, 12
    g = torch.Generator().manual_seed(9)
    x = torch.zeros(B, N, 152, dtype=torch.bfloat16)
    v = 300.0 + 20.0 * torch.randn(B, N, D, generator=g)
    v[:, :f] = -1000.0 + 5000.0 * torch.rand(B, f, D, generator=g)
    x[:, :, :D] = v
    xg = x.to(DEV)
    win, reg = _both(xg, D, f, False, ms=1000.0)
    ok = _same(win, reg, False)
    assert ok.any()


@pytest.mark.parametrize("N,D,f,constrained", [(64, 1000, 8, True), (256, 700, 32, True), (100, 260, 10, False)])
def test_win_split_modes_bitwise(N, D, f, constrained):
    """mode 1 + mode 2 through a persistent workspace == the fused window round, bit for bit."""
    B = 6
    x, _ = beta_oracles(B, N, D, f, seed=N + 1)
    xg = x.to(DEV)
    full = run_fast(xg, D, f, constrained, 1.0)
    o = alloc_fast_out(B, N, D, DEV)
    w = fast_work(B, D, DEV)
    args = (xg, None, D, f, constrained, 1.0, o["c1"], o["consensus"], o["skew"], o["kurt"], o["rel"], o["qr"],
            o["reliable"], o["status"], 0)
    svops.ops().fast_round(*args, 1, D, False, w)
    svops.ops().fast_round(*args, 2, D, False, w)
    for k in full:
        assert torch.equal(o[k], full[k]), k


def test_win_active_mask_and_workspace_reuse():
    B, N, D, f = 12, 256, 512, 32
    x, _ = beta_oracles(B, N, D, f, seed=77)
    xg = x.to(DEV)
    w = fast_work(B, D, DEV)
    act = (torch.arange(B) % 3 != 1).to(torch.uint8).to(DEV)
    a = run_fast(xg, D, f, True, active=act, work=w)
    b = run_fast(xg, D, f, True, active=act, work=w)
    reg = run_fast(xg, D, f, True, active=act, wave_hint=-7)
    torch.cuda.synchronize()
    on = act.bool()
    for k in ("consensus", "skew", "kurt", "rel", "status"):
        assert torch.equal(a[k], b[k]), k
    assert (a["status"][~on] == -1).all()   # inactive instances untouched
    assert torch.equal(a["consensus"][on], reg["consensus"][on])
