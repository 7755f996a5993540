"""HIP kernels on a real MI355X vs the plain-PyTorch fp32 reference / the bit-exact CPU engine."""
import random

import pytest
import torch

from fixtures import GOLDEN, N_FAILING
from helpers import beta_oracles, run_exact, run_fast
from svoc import ops as svops
from svoc.ops import torch_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _cmp_fast(o, r, ok):
    assert torch.equal(o["reliable"][ok].bool().cpu(), r["reliable"][ok].cpu())
    torch.testing.assert_close(o["c1"][ok], r["c1"][ok], rtol=0, atol=1e-6)
    torch.testing.assert_close(o["consensus"][ok], r["consensus"][ok], rtol=0, atol=2e-6)
    torch.testing.assert_close(o["qr"][ok], r["qr"][ok], rtol=2e-4, atol=1e-5)
    torch.testing.assert_close(o["rel"][ok], r["rel"][ok], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(o["skew"][ok], r["skew"][ok], rtol=2e-3, atol=2e-3)
    torch.testing.assert_close(o["kurt"][ok], r["kurt"][ok], rtol=2e-3, atol=5e-3)


_SHAPES = [(7, 6, 2, True), (64, 1024, 8, True), (64, 1000, 8, False), (50, 300, 5, True),
           (128, 512, 16, True), (100, 260, 10, False), (256, 4096, 32, True), (256, 600, 32, False),
           (200, 136, 20, True), (20, 8, 15, True),
           # small-instance kernel (N <= 16, D <= 128) under hint 0
           (7, 6, 2, False), (16, 100, 3, True), (9, 1, 2, True), (12, 128, 4, False), (8, 33, 2, True)]


# hint 0: default dispatch (window kernel / small kernel); -7: the two-network register-streaming kernel
@pytest.mark.parametrize("N,D,f,constrained,hint", [s + (h,) for s in _SHAPES for h in (0, -7)])
def test_fast_hip_vs_torch(N, D, f, constrained, hint):
    B = 12
    x, _ = beta_oracles(B, N, D, f, seed=7 * N + D)
    xg = x.to(DEV)
    o = run_fast(xg, D, f, constrained, 1.0, wave_hint=hint)
    torch.cuda.synchronize()
    r = torch_ref.fast_round(xg[:, :, :D], f, constrained, 1.0)
    ok = (o["status"] == 0)
    assert ok.any(), o["status"]
    _cmp_fast(o, r, ok)
    # the CPU engine agrees on status
    oc = run_fast(x, D, f, constrained, 1.0)
    assert torch.equal(oc["status"], o["status"].cpu())


def test_fast_small_kernel_batch_edges():
    """Deployed config 7 x 6: partial last workgroup, inactive instances, reverts, vs the CPU engine."""
    B, N, D = 1000, 7, 6
    x, _ = beta_oracles(B, N, D, 2, seed=21)
    x[5] = 0.0                               # zero variance -> ZERO_VARIANCE (the round reverts)
    x[6, :4, :D] = 0.0                       # rel1 < 0 -> RELIABILITY_INTERVAL
    x[6, 4:, :D] = 1.0
    active = (torch.arange(B) % 7 != 3).to(torch.uint8)
    o = run_fast(x.to(DEV), D, 2, True, 1.0, active=active.to(DEV))
    oc = run_fast(x, D, 2, True, 1.0, active=active)
    assert torch.equal(o["status"].cpu(), oc["status"])
    ok = o["status"].cpu() == 0
    assert ok.sum() > 800
    r = torch_ref.fast_round(x[:, :, :D], 2, True, 1.0)
    _cmp_fast({k: v.cpu() for k, v in o.items()}, r, ok)


def test_fast_hip_active_mask_and_revert():
    B, N, D = 6, 64, 128
    x, _ = beta_oracles(B, N, D, 8, seed=3)
    x[1] = 0.0                          # zero variance everywhere -> ZERO_VARIANCE (the round reverts)
    x[2, :40, :D] = 0.0                 # c1 = 0, 24/64 rows at distance 1: rel1 = 1 - 2*sqrt(.375) < 0
    x[2, 40:, :D] = 1.0
    xg = x.to(DEV)
    active = torch.tensor([1, 1, 1, 0, 1, 1], dtype=torch.uint8, device=DEV)
    o = run_fast(xg, D, 8, True, 1.0, active=active)
    st = o["status"].cpu().tolist()
    assert st[3] == -1                  # inactive: untouched
    assert st[0] == 0 and st[4] == 0
    assert st[1] == 32                  # ZERO_VARIANCE
    assert st[2] == 6                   # RELIABILITY_INTERVAL
    oc = run_fast(x, D, 8, True, 1.0, active=active.cpu())
    assert oc["status"].tolist() == st


@pytest.mark.parametrize("name", list(GOLDEN))
def test_exact_hip_goldens(name):
    values, constrained, ms, g = GOLDEN[name]
    o = run_exact(torch.tensor([values] * 3, dtype=torch.int64, device=DEV), N_FAILING, constrained, ms)
    assert o["status"].tolist() == [0, 0, 0]
    assert o["consensus"][2].tolist() == g["consensus"]
    assert o["rel"][1].tolist() == [g["rel1"], g["rel2"]]
    assert o["skew"][0].tolist() == g["skewness"]
    assert o["kurt"][0].tolist() == g["kurtosis"]
    assert o["qr"][0].tolist() == g["qr"]


def test_exact_hip_wide_instances_workspace():
    """6*D int64 intermediates beyond 64 KiB of LDS: the kernel switches to an HBM workspace."""
    rng = random.Random(4)
    B, N, D = 3, 9, 1500
    vals = torch.tensor([[[rng.randint(400000, 600000) for _ in range(D)] for _ in range(N)] for _ in range(B)])
    oc = run_exact(vals, 2, True)
    og = run_exact(vals.to(DEV), 2, True)
    for k in ("status", "consensus", "rel", "qr", "skew", "kurt", "reliable", "c1"):
        assert torch.equal(oc[k], og[k].cpu()), k


@pytest.mark.parametrize("constrained", [True, False])
def test_exact_hip_matches_cpu_random(constrained):
    rng = random.Random(99)
    for N, D, f in [(7, 6, 2), (9, 3, 1), (70, 5, 9), (130, 4, 20), (5, 2, 1), (4, 2, 0), (3, 1, 1)]:
        B = 16
        if constrained:
            base = torch.randint(0, 1_000_001, (B, 1, D))
            v = (base + torch.randint(-rng.choice([3, 500, 90_000]), 90_001, (B, N, D))).clamp(0, 1_000_000)
        else:
            v = torch.randint(-10**8, 10**8, (B, 1, D)) + torch.randint(-4_000_000, 4_000_000, (B, N, D))
        v[0] = v[0, :1]                 # zero variance instance -> revert
        oc = run_exact(v, f, constrained, 5_000_000)
        og = run_exact(v.to(DEV), f, constrained, 5_000_000)
        for k in oc:
            assert torch.equal(oc[k], og[k].cpu()), (k, N, D, f)


def test_apply_updates_hip_vs_cpu():
    B, N, D, ld = 5, 16, 24, 24
    U = 200
    g = torch.Generator().manual_seed(0)
    inst = torch.randint(0, B, (U,), generator=g)
    orc = torch.randint(0, N, (U,), generator=g)
    orc[7] = N + 3                      # not an oracle
    upd = torch.rand(U, D, generator=g).to(torch.bfloat16)
    upd[11, 3] = 1.5                    # interval error
    res = []
    for dev in ("cpu", DEV):
        vals = torch.zeros(B, N, ld, dtype=torch.bfloat16, device=dev)
        en = torch.zeros(B, N, dtype=torch.uint8, device=dev)
        na = torch.zeros(B, dtype=torch.int32, device=dev)
        tch = torch.zeros(B, dtype=torch.uint8, device=dev)
        win = torch.full((B, N), -1, dtype=torch.int32, device=dev)
        st = torch.empty(U, dtype=torch.int32, device=dev)
        svops.ops().apply_updates(vals, en, na, tch, win, inst.to(dev), orc.to(dev), upd.to(dev), True, st)
        res.append([t.cpu() for t in (vals, en, na, tch, st, win)])
    for a, b in zip(*res):
        assert torch.equal(a, b)
    assert res[1][5].eq(-1).all()


@pytest.mark.parametrize("N,D,f,constrained", [(64, 1000, 8, True), (256, 700, 32, True), (100, 260, 10, False)])
def test_fast_hip_split_modes_match_full(N, D, f, constrained):
    """mode 1 (pass 1: qr partials) + mode 2 (pass 2 from qr) == the fused round (D-sharding path),
    and two column shards with a summed qr reproduce the full instance."""
    B = 6
    x, _ = beta_oracles(B, N, D, f, seed=N)
    xg = x.to(DEV)
    full = run_fast(xg, D, f, constrained, 1.0, wave_hint=-7)   # two-network kernel (split = no workspace)
    from helpers import alloc_fast_out
    o = alloc_fast_out(B, N, D, DEV)
    args = (xg, None, D, f, constrained, 1.0, o["c1"], o["consensus"], o["skew"], o["kurt"], o["rel"], o["qr"],
            o["reliable"], o["status"], 0)
    svops.ops().fast_round(*args, 1, D)
    svops.ops().fast_round(*args, 2, D)
    for k in ("consensus", "rel", "reliable", "status", "skew", "kurt"):
        torch.testing.assert_close(o[k], full[k], rtol=0, atol=0)
    # two shards of the columns
    h = (D // 2 + 7) // 8 * 8
    parts = []
    for lo, hi in ((0, h), (h, D)):
        xs = torch.zeros(B, N, (hi - lo + 7) // 8 * 8, dtype=torch.bfloat16, device=DEV)
        xs[:, :, : hi - lo] = xg[:, :, lo:hi]
        os_ = alloc_fast_out(B, N, hi - lo, DEV)
        parts.append((xs, os_, hi - lo, lo, hi))
        svops.ops().fast_round(xs, None, hi - lo, f, constrained, 1.0, os_["c1"], os_["consensus"], os_["skew"],
                               os_["kurt"], os_["rel"], os_["qr"], os_["reliable"], os_["status"], 0, 1, D)
    qsum = parts[0][1]["qr"] + parts[1][1]["qr"]
    for xs, os_, dd, lo, hi in parts:
        os_["qr"].copy_(qsum)
        svops.ops().fast_round(xs, None, dd, f, constrained, 1.0, os_["c1"], os_["consensus"], os_["skew"],
                               os_["kurt"], os_["rel"], os_["qr"], os_["reliable"], os_["status"], 0, 2, D)
        ok = full["status"] == 0
        assert torch.equal(os_["reliable"][ok], full["reliable"][ok])
        torch.testing.assert_close(os_["consensus"][ok], full["consensus"][ok][:, lo:hi], rtol=0, atol=1e-6)
        torch.testing.assert_close(os_["rel"][ok], full["rel"][ok], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("N,D,hint", [(7, 6, 0), (64, 1024, 0), (256, 700, 0), (64, 1024, -7), (200, 96, -7),
                                      (128, 512, 0)])
def test_fast_kernels_deterministic(N, D, hint):
    """Same inputs -> bitwise identical outputs (no float atomics; fixed reduction orders)."""
    x, _ = beta_oracles(9, N, D, max(1, N // 8), seed=N + D)
    xg = x.to(DEV)
    a = run_fast(xg, D, max(1, N // 8), True, 1.0, wave_hint=hint)
    b = run_fast(xg.clone(), D, max(1, N // 8), True, 1.0, wave_hint=hint)
    for k in a:
        assert torch.equal(a[k], b[k]), k
    r = torch_ref.fast_round(xg[:, :, :D], max(1, N // 8), True, 1.0)
    ok = a["status"] == 0
    assert ok.any()
    _cmp_fast(a, r, ok)


def test_unconstrained_updates_reject_non_finite_gpu():
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    from svoc.status import Status
    for D in (3, 64):   # 1 lane and 8 lanes per update
        e = ConsensusEngine(ConsensusConfig(n_oracles=4, dimension=D, n_failing_oracles=0, constrained=False,
                                            unconstrained_max_spread=10.0), 2, device=DEV, mode="fast")
        vals = torch.zeros(4, D)
        vals[1, D - 1] = float("nan")
        vals[2, 0] = float("-inf")
        st = e.apply_updates(torch.tensor([0, 0, 1, 1], device=DEV), torch.tensor([0, 1, 2, 3], device=DEV),
                             vals.to(DEV))
        assert st.cpu().tolist() == [Status.OK, Status.NON_FINITE, Status.NON_FINITE, Status.OK]


@pytest.mark.parametrize("D,constrained,storage", [(6, True, "bf16"), (4096, True, "bf16"), (100, False, "bf16"),
                                                   (6, True, "fp32"), (2048, True, "fp32"), (4096, True, "fp32"),
                                                   (4096, False, "fp32"), (100, False, "fp32")])
def test_unique_update_path_matches_general(D, constrained, storage):
    """apply_updates(unique=True) (one fused pass) == the last-writer path on distinct pairs."""
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    cfg = ConsensusConfig(n_oracles=16, dimension=D, n_failing_oracles=2, constrained=constrained,
                          unconstrained_max_spread=5.0)
    g = torch.Generator().manual_seed(D)
    B, U = 40, 300
    flat = torch.randperm(B * 16, generator=g)[:U]
    inst, orc = flat // 16, flat % 16
    vals = torch.rand(U, D, generator=g)
    vals[3, 0] = 1.5                 # interval error (constrained) / fine (unconstrained)
    vals[7, D - 1] = float("nan")    # rejected either way
    vals[9, 0] = -0.0                # accepted (0 <= -0.0 <= 1)
    vals[11, 1] = -1e-30             # interval error (constrained)
    outs = []
    for unique in (False, True):
        e = ConsensusEngine(cfg, B, device=DEV, mode="fast", storage=storage)
        st = e.apply_updates(inst.to(DEV), orc.to(DEV), vals.to(DEV), unique=unique)
        outs.append((st.cpu(), e.values.cpu(), e.enabled.cpu(), e.n_active.cpu(), e.touched.cpu()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("constrained", [True, False])
def test_apply_updates_unique_short_rows(constrained):
    """The unique-update kernel's short-row path (7 x 6 bf16 rows, 12 B): distinct (instance, oracle)
    pairs, an out-of-range oracle, an interval / non-finite value; equal to the CPU loop."""
    B, N, D, ld = 40, 7, 6, 8
    g = torch.Generator().manual_seed(5)
    pairs = torch.randperm(B * N, generator=g)[:150]
    inst, orc = pairs // N, pairs % N
    orc[7] = N + 3                      # not an oracle
    upd = torch.rand(150, D, generator=g).to(torch.bfloat16)
    upd[11, 3] = 1.5 if constrained else float("nan")
    res = []
    for dev in ("cpu", DEV):
        vals = torch.zeros(B, N, ld, dtype=torch.bfloat16, device=dev)
        en = torch.zeros(B, N, dtype=torch.uint8, device=dev)
        en[3] = 1                       # some oracles already enabled
        na = en.sum(1, dtype=torch.int32)
        tch = torch.zeros(B, dtype=torch.uint8, device=dev)
        win = torch.full((B, N), -1, dtype=torch.int32, device=dev)
        st = torch.empty(150, dtype=torch.int32, device=dev)
        svops.ops().apply_updates(vals, en, na, tch, win, inst.to(dev), orc.to(dev), upd.to(dev), constrained, st,
                                  True)
        res.append([t.cpu() for t in (vals, en, na, tch, st)])
    for a, b in zip(*res):
        assert torch.equal(a.view(torch.uint8) if a.dtype == torch.bfloat16 else a,
                           b.view(torch.uint8) if b.dtype == torch.bfloat16 else b)
    assert res[1][4][7].item() != 0 and res[1][4][11].item() != 0
