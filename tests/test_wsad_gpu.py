"""Column-parallel exact kernel (csrc/kernels/consensus_wsad.hip) vs the i128 kernel and the CPU engine.

Every round it accepts must be bit-identical (consensus, c1, qr, reliable, rel1/rel2, skewness,
kurtosis); every other round (reverts, out-of-domain values) goes to the i128 kernel, so the combined
result equals the CPU golden engine everywhere.  Reference semantics: contract.cairo:442-503,
signed_decimal.cairo:52-116, math.cairo:113-398.
"""
import os

import pytest
import torch

from fixtures import GOLDEN, N_FAILING
from helpers import alloc_exact_out, beta_oracles
from svoc import ops as svops

pytestmark = pytest.mark.gpu
DEV = "cuda"
OUTS = ("c1", "consensus", "skew", "kurt", "rel", "qr", "reliable", "status")


def _wsad(B, N, D, f, seed, a=20.0):
    x, _ = beta_oracles(B, N, D, f, a=a, seed=seed, dtype=torch.float64)
    return (x[:, :, :D] * 1e6).to(torch.int64).contiguous()


def _run(values, f, env=None, active=None, constrained=True, ms=0):
    B, N, D = values.shape
    o = alloc_exact_out(B, N, D, values.device)
    old = {k: os.environ.get(k) for k in ("SVOC_EXACT_I128", "SVOC_EXACT_WSAD_ONLY", "SVOC_EXACT_WSAD_MIN_D")}
    try:
        for k in old:
            os.environ.pop(k, None)
        os.environ.update(env or {})
        svops.ops().exact_round(values, active, f, constrained, ms, o["c1"], o["consensus"], o["skew"], o["kurt"],
                                o["rel"], o["qr"], o["reliable"], o["status"], False)
        torch.cuda.synchronize()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return {k: v.cpu() for k, v in o.items()}


SHAPES = [(4, 3, 0), (7, 6, 2), (16, 33, 3), (50, 300, 5), (64, 1024, 8), (64, 1000, 20), (100, 260, 10),
          (128, 512, 16), (200, 136, 20), (256, 600, 32), (256, 64, 100), (33, 1, 4)]


@pytest.mark.parametrize("N,D,f", SHAPES)
@pytest.mark.parametrize("dtype", [torch.int64, torch.int32])
def test_wsad_kernel_bit_exact(N, D, f, dtype):
    B = 16
    v = _wsad(B, N, D, f, seed=N * 1000 + D)
    vg = v.to(DEV, dtype)
    fast = _run(vg, f, {"SVOC_EXACT_WSAD_ONLY": "1", "SVOC_EXACT_WSAD_MIN_D": "1"})   # the column-parallel kernel alone
    ref = _run(v.to(DEV), f, {"SVOC_EXACT_I128": "1"})   # the i128 kernel alone
    took = fast["status"] == 0
    assert took.sum() >= B - 1, fast["status"]         # it takes (almost) every round of Beta data
    for k in OUTS:
        assert torch.equal(fast[k][took], ref[k][took]), k
    comb = _run(vg, f, {"SVOC_EXACT_WSAD_MIN_D": "1"})   # dispatcher: column-parallel + i128 fallback
    for k in OUTS:
        assert torch.equal(comb[k], ref[k]), k


def test_wsad_kernel_matches_cpu_engine():
    B, N, D, f = 24, 64, 257, 8
    v = _wsad(B, N, D, f, seed=5)
    g = _run(v.to(DEV, torch.int32), f)
    o = alloc_exact_out(B, N, D, "cpu")
    svops.ops().exact_round(v, None, f, True, 0, o["c1"], o["consensus"], o["skew"], o["kurt"], o["rel"], o["qr"],
                            o["reliable"], o["status"], False)
    for k in OUTS:
        assert torch.equal(g[k], o[k]), k


@pytest.mark.parametrize("name", [n for n in GOLDEN if GOLDEN[n][1]])
def test_wsad_kernel_goldens(name):
    values, constrained, ms, gold = GOLDEN[name]
    v = torch.tensor([values] * 3, dtype=torch.int64, device=DEV)
    o = _run(v, N_FAILING, {"SVOC_EXACT_WSAD_ONLY": "1", "SVOC_EXACT_WSAD_MIN_D": "1"})
    assert o["status"].tolist() == [0, 0, 0]
    assert o["consensus"][2].tolist() == gold["consensus"]
    assert o["rel"][1].tolist() == [gold["rel1"], gold["rel2"]]
    assert o["skew"][0].tolist() == gold["skewness"]
    assert o["kurt"][0].tolist() == gold["kurtosis"]
    assert o["qr"][0].tolist() == gold["qr"]


def test_wsad_kernel_flags_reverts_and_out_of_domain():
    """Reverting rounds get the CPU engine's stage-ordered status from the column kernel itself; values
    outside [0, 1e6] are left to the i128 kernel (flag -1); the combined dispatch equals the CPU engine."""
    B, N, D, f = 8, 64, 128, 8
    v = _wsad(B, N, D, f, seed=9)
    v[1, :, 5] = 400000                       # zero variance column -> DIV_BY_ZERO in the contract
    v[2, : N // 2 + 1, :] = 0                 # rel1 < 0 -> RELIABILITY_INTERVAL
    v[2, N // 2 + 1:, :] = 1000000
    v[3, 7, 3] = 1000001                      # outside the constrained domain
    v[4, 2, 2] = -5
    v[5, :, 9] = 0                            # zero variance at 0
    v[5, 0, 9] = 1                            # ... except one ulp: variance rounds to 0 in wsad
    only = _run(v.to(DEV), f, {"SVOC_EXACT_WSAD_ONLY": "1"})
    comb = _run(v.to(DEV), f)
    o = alloc_exact_out(B, N, D, "cpu")
    svops.ops().exact_round(v, None, f, True, 0, o["c1"], o["consensus"], o["skew"], o["kurt"], o["rel"], o["qr"],
                            o["reliable"], o["status"], False)
    st = only["status"].cpu().tolist()
    assert st[3] == -1 and st[4] == -1 and only["status"][6:].eq(0).all(), st
    assert [st[i] for i in (0, 1, 2, 5)] == [o["status"][i].item() for i in (0, 1, 2, 5)], st
    for k in OUTS:
        assert torch.equal(comb[k], o[k]), k
    assert comb["status"][1].item() != 0 and comb["status"][2].item() != 0


def test_engine_exact_int32_storage_gpu():
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    cfg = ConsensusConfig(n_oracles=64, dimension=512, n_failing_oracles=8, constrained=True)
    e32 = ConsensusEngine(cfg, 32, device=DEV, mode="exact", storage="int32")
    e64 = ConsensusEngine(cfg, 32, device=DEV, mode="exact")
    for e in (e32, e64):
        e.randomize(seed=4)
        e.run_round()
    torch.cuda.synchronize()
    assert (e64.status == 0).all()
    for k in ("consensus", "skew", "kurt", "rel", "qr", "reliable", "c1", "status"):
        assert torch.equal(getattr(e32, k), getattr(e64, k)), k


@pytest.mark.parametrize("N,D,f", [(64, 1024, 8), (256, 512, 32)])
def test_fast_bf16_agrees_with_exact_on_shared_grid(N, D, f):
    """Fast (bf16 storage, fp32 math) vs exact (wsad) on data both represent exactly (x = j / 64, i.e.
    wsad j * 15625): identical reliable masks, consensus within 1 wsad ulp, rel1 / rel2 within 32 wsad
    ulps (the contract truncates every wsad_mul and its Newton sqrt; fp32 rounds).  Instances whose exact
    quadratic risks tie across the rank cut are skipped (the tie rule then decides on values the two
    modes round differently)."""
    from helpers import run_fast
    B = 32
    x, _ = beta_oracles(B, N, D, f, seed=N + D, dtype=torch.float64)
    j = torch.round(x[:, :, :D] * 64).clamp(0, 64)
    vb = torch.zeros(B, N, (D + 7) // 8 * 8, dtype=torch.bfloat16)
    vb[:, :, :D] = (j / 64).to(torch.bfloat16)
    vw = (j * 15625).to(torch.int64).contiguous()
    fa = run_fast(vb.to(DEV), D, f, True, 1.0)
    ex = _run(vw.to(DEV, torch.int32), f)
    torch.cuda.synchronize()
    fa = {k: v.cpu() for k, v in fa.items()}
    assert (ex["status"] == 0).all() and (fa["status"] == 0).all()
    q = ex["qr"]
    srt = torch.sort(q, dim=1).values
    R = N - f
    clean = srt[:, R - 1] != srt[:, R]          # no tie across the cut
    assert clean.sum() >= B // 2
    assert torch.equal(fa["reliable"][clean].bool(), ex["reliable"][clean].bool())
    cons = (fa["consensus"][clean].double() * 1e6 - ex["consensus"][clean].double()).abs()
    assert cons.max().item() <= 1.0 + 1e-6, cons.max()
    # rel: the contract truncates every wsad product of its quadratic sums (D terms each), fp32 rounds;
    # measured max 13 wsad ulps (1.3e-5) on 64 x 1024
    rel = (fa["rel"][clean].double() * 1e6 - ex["rel"][clean].double()).abs()
    assert rel.max().item() <= 32.0, rel.max()


@pytest.mark.parametrize("path", ["dispatch", "i128", "wsad_only"])
@pytest.mark.parametrize("N,D,f", [(16, 24, 3), (64, 300, 8), (256, 70, 32), (512, 96, 64), (1500, 40, 150),
                                   (4096, 16, 512)])
def test_exact_split_modes_match_whole_round(N, D, f, path):
    """The exact kernels' D-sharded halves (mode 1: c1 + qr partials; mode 2: from the summed qr), run on
    two column slices on one GPU with the all-reduce done by hand, reproduce the whole round bit for bit:
    through the dispatcher (column-parallel kernel + i128 fallback), the i128 kernel alone, and the
    column-parallel kernel alone (which must then take every round: clean data).  N > 256: the wide lane
    groups' halves (D-sharded exact rounds no longer fall back to the i128 kernel)."""
    B = 8
    v = _wsad(B, N, D, f, seed=N + 7 * D)
    if path != "wsad_only":
        v[2, :, D // 4] = 123_456       # zero variance in slice 0 only: instance 2 reverts
    vg = v.to(DEV)
    whole = _run(vg, f)
    env = {"dispatch": {"SVOC_EXACT_WSAD_MIN_D": "1"}, "i128": {"SVOC_EXACT_I128": "1"},
           "wsad_only": {"SVOC_EXACT_WSAD_ONLY": "1", "SVOC_EXACT_WSAD_MIN_D": "1"}}[path]
    old_env = {k: os.environ.get(k) for k in ("SVOC_EXACT_I128", "SVOC_EXACT_WSAD_ONLY", "SVOC_EXACT_WSAD_MIN_D")}
    for k in old_env:
        os.environ.pop(k, None)
    os.environ.update(env)
    try:
        _split_rounds(vg, whole, N, D, f, B, expect_revert=path != "wsad_only")
    finally:
        for k, val in old_env.items():
            if val is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = val


def _split_rounds(vg, whole, N, D, f, B, expect_revert):
    cut = D // 2
    parts = [vg[:, :, :cut].contiguous(), vg[:, :, cut:].contiguous()]
    outs = [alloc_exact_out(B, N, x.shape[2], DEV) for x in parts]
    op = svops.ops().exact_round
    for x, o in zip(parts, outs):
        op(x, None, f, True, 0, o["c1"], o["consensus"], o["skew"], o["kurt"], o["rel"], o["qr"], o["reliable"],
           o["status"], False, 1, D)
    qr = outs[0]["qr"] + outs[1]["qr"]
    st = torch.maximum(outs[0]["status"], outs[1]["status"])
    for x, o in zip(parts, outs):
        o["qr"].copy_(qr)
        o["status"].copy_(st)
        op(x, None, f, True, 0, o["c1"], o["consensus"], o["skew"], o["kurt"], o["rel"], o["qr"], o["reliable"],
           o["status"], False, 2, D)
    st = torch.maximum(outs[0]["status"], outs[1]["status"]).cpu()
    torch.cuda.synchronize()
    assert torch.equal(st, whole["status"])
    assert (st != 0).sum().item() == (1 if expect_revert else 0) and (not expect_revert or st[2].item() != 0)
    ok = st == 0
    for o in outs:
        for k in ("rel", "qr", "reliable"):
            assert torch.equal(o[k].cpu()[ok], whole[k][ok]), k
    for k in ("c1", "consensus", "skew", "kurt"):
        got = torch.cat([outs[0][k].cpu(), outs[1][k].cpu()], dim=1)
        assert torch.equal(got[ok], whole[k][ok]), k


@pytest.mark.parametrize("N,D,f", [(64, 512, 8), (256, 300, 32), (100, 130, 10)])
@pytest.mark.parametrize("dtype", [torch.int64, torch.int32])
def test_wsad_kernel_reliable_outliers(N, D, f, dtype):
    """A RELIABLE row far from the column mean (|z| up to ~12 real units) in a few columns: the z-power
    products pass the fp64 path's 2^50 bound, and the column-parallel kernel sums those rows' powers in
    int64 instead of handing the instance to the i128 kernel (round 3: every such instance fell back).
    The kernel alone must take every round and equal the i128 kernel bit for bit."""
    B = 8
    v = _wsad(B, N, D, f, seed=N + D + 17, a=80.0)          # tight honest cluster (sd ~0.039)
    g = torch.Generator().manual_seed(N)
    for b in range(B):
        # one row pushed +-0.45 in 3 columns: its qr grows by ~0.6 only, so it stays reliable, and alone in
        # its column it sits at |z| ~ 6-9 real units
        rows = torch.randperm(N, generator=g)[:1]
        cols = torch.randperm(D, generator=g)[:3]
        for r in rows.tolist():
            for c in cols.tolist():
                v[b, r, c] = 950_000 if v[b, r, c] < 500_000 else 50_000
    vg = v.to(DEV, dtype)
    fast = _run(vg, f, {"SVOC_EXACT_WSAD_ONLY": "1", "SVOC_EXACT_WSAD_MIN_D": "1"})
    ref = _run(v.to(DEV), f, {"SVOC_EXACT_I128": "1"})
    assert (ref["status"] == 0).all(), ref["status"]
    assert (fast["status"] == 0).all(), fast["status"]
    for k in OUTS:
        assert torch.equal(fast[k], ref[k]), k


@pytest.mark.parametrize("N,D,f", [(64, 256, 8), (200, 300, 20), (16, 64, 13)])
def test_wsad_kernel_legacy_rounds(N, D, f):
    """Obsolete N-D contract rounds (reliability without /D, no moments: contract_nd.cairo:340-442) run in
    the column-parallel kernel too (round 3 sent every legacy round to the i128 kernel) -- bit-identical,
    including R = 3 reliable rows, which only the current contract's kurtosis rejects."""
    B = 6
    # every row near 0.5 (+-0.02): the RMS deviation over ALL dims stays << 0.5, as the /D-less
    # reliability needs (the generator's U(0,1) failing rows would push it past the interval)
    g = torch.Generator().manual_seed(N * 3 + D)
    v = 500_000 + torch.randint(-20_000, 20_001, (B, N, D), generator=g, dtype=torch.int64)
    vg = v.to(DEV)
    def run(env):
        o = alloc_exact_out(B, N, D, DEV)
        old = {k: os.environ.get(k) for k in ("SVOC_EXACT_I128", "SVOC_EXACT_WSAD_ONLY", "SVOC_EXACT_WSAD_MIN_D")}
        try:
            for k in old:
                os.environ.pop(k, None)
            os.environ.update(env)
            svops.ops().exact_round(vg, None, f, True, 0, o["c1"], o["consensus"], o["skew"], o["kurt"], o["rel"],
                                    o["qr"], o["reliable"], o["status"], True)
            torch.cuda.synchronize()
        finally:
            for k, val in old.items():
                if val is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = val
        return {k: t.cpu() for k, t in o.items()}
    fast = run({"SVOC_EXACT_WSAD_ONLY": "1", "SVOC_EXACT_WSAD_MIN_D": "1"})
    ref = run({"SVOC_EXACT_I128": "1"})
    assert (ref["status"] == 0).all(), ref["status"]
    assert (fast["status"] == 0).all(), fast["status"]
    for k in OUTS:
        assert torch.equal(fast[k], ref[k]), k
    assert not fast["skew"].any() and not fast["kurt"].any()


@pytest.mark.parametrize("N,D,f", [(64, 256, 8), (256, 200, 32), (40, 70, 4)])
def test_wsad_kernel_reverts_in_kernel(N, D, f):
    """Reverting rounds are decided by the column-parallel kernel itself, with the reference's stage-ordered
    code (round 3 sent every reverting round to the i128 kernel): a zero-variance reliable column and a
    variance-1 column (sqrt(1)) -> DIV_BY_ZERO in the moments, rel1 < 0 -> RELIABILITY_INTERVAL before
    them, R = 3 -> DIV_BY_ZERO (kurtosis).  Statuses equal the i128 kernel's; reverted outputs untouched."""
    B = 6
    v = _wsad(B, N, D, f, seed=N + 5 * D)
    v[1, :, 3] = 654_321                                   # constant column: variance 0
    v[2, :, 5] = 500_000
    v[2, :N // 2, 5] = 500_001                             # 0/1 ulp column: tiny variance (sqrt(1) or 0)
    v[3, : N // 2 + 1, :] = 0                              # c1 = 0, the rest at distance 1: rel1 < 0
    v[3, N // 2 + 1:, :] = 1_000_000
    vg = v.to(DEV)
    fast = _run(vg, f, {"SVOC_EXACT_WSAD_ONLY": "1", "SVOC_EXACT_WSAD_MIN_D": "1"})
    ref = _run(v.to(DEV), f, {"SVOC_EXACT_I128": "1"})
    assert torch.equal(fast["status"], ref["status"]), (fast["status"], ref["status"])
    st = ref["status"].tolist()
    assert st[1] != 0 and st[3] != 0 and st[0] == 0, st
    ok = ref["status"] == 0
    for k in OUTS:
        assert torch.equal(fast[k][ok], ref[k][ok]), k
    # R = 3: every round reverts in the moments (the kurtosis' (n-2)(n-3) = 0)
    f3 = N - 3
    fast3 = _run(vg, f3, {"SVOC_EXACT_WSAD_ONLY": "1", "SVOC_EXACT_WSAD_MIN_D": "1"})
    ref3 = _run(v.to(DEV), f3, {"SVOC_EXACT_I128": "1"})
    assert torch.equal(fast3["status"], ref3["status"]), (fast3["status"], ref3["status"])
    assert (ref3["status"] != 0).all()


# ---------------------------------------------------------------------------------------------------
# Unconstrained rounds (contract.cairo:370-434) in the column kernel: signed int32-range values within
# 2^25 (33.55 real units) of the column median / reliable mean; the essence is the reliable mean.

MS = 10 * 1_000_000   # unconstrained_max_spread of the reference's tests (test_contract.cairo:253-261)


def _signed(B, N, D, f, seed, honest_sd=1e6, fail_span=20e6, centre=3e6):
    g = torch.Generator().manual_seed(seed)
    x = centre + honest_sd * torch.randn(B, N, D, generator=g, dtype=torch.float64)
    bad = torch.stack([torch.randperm(N, generator=g)[:f] for _ in range(B)])
    fv = centre + fail_span * (2 * torch.rand(B, f, D, generator=g, dtype=torch.float64) - 1)
    x.scatter_(1, bad[:, :, None].expand(B, f, D), fv)
    return x.round().to(torch.int64).contiguous()


def _cpu(v, f, constrained, ms):
    B, N, D = v.shape
    o = alloc_exact_out(B, N, D, "cpu")
    svops.ops().exact_round(v.cpu().to(torch.int64), None, f, constrained, ms, o["c1"], o["consensus"], o["skew"],
                            o["kurt"], o["rel"], o["qr"], o["reliable"], o["status"], False)
    return o


def test_wsad_kernel_unconstrained_golden():
    values, constrained, ms, gold = GOLDEN["unconstrained_2d"]
    assert not constrained
    v = torch.tensor([values] * 3, dtype=torch.int64, device=DEV)
    o = _run(v, N_FAILING, {"SVOC_EXACT_WSAD_ONLY": "1", "SVOC_EXACT_WSAD_MIN_D": "1"}, constrained=False, ms=ms)
    assert o["status"].tolist() == [0, 0, 0]
    assert o["c1"][0].tolist() == gold["c1"]
    assert o["consensus"][2].tolist() == gold["consensus"]
    assert o["rel"][1].tolist() == [gold["rel1"], gold["rel2"]]
    assert o["skew"][0].tolist() == gold["skewness"]
    assert o["kurt"][0].tolist() == gold["kurtosis"]
    assert o["qr"][0].tolist() == gold["qr"]


@pytest.mark.parametrize("N,D,f", [(7, 6, 2), (64, 1024, 8), (64, 100, 20), (100, 260, 10), (200, 136, 20),
                                   (256, 300, 32)])
@pytest.mark.parametrize("dtype", [torch.int64, torch.int32])
def test_wsad_kernel_unconstrained_bit_exact(N, D, f, dtype):
    """Every round of signed data with far failing oracles: the column kernel alone takes them all and
    equals the i128 kernel and the CPU engine bit for bit."""
    B = 12
    v = _signed(B, N, D, f, seed=N * 7 + D)
    fast = _run(v.to(DEV, dtype), f, {"SVOC_EXACT_WSAD_ONLY": "1", "SVOC_EXACT_WSAD_MIN_D": "1"}, constrained=False,
                ms=MS)
    ref = _run(v.to(DEV), f, {"SVOC_EXACT_I128": "1"}, constrained=False, ms=MS)
    cpu = _cpu(v, f, False, MS)
    assert (fast["status"] != -1).all(), fast["status"]        # nothing handed to the i128 kernel
    for k in OUTS:
        assert torch.equal(fast[k], ref[k]), k
        assert torch.equal(fast[k], cpu[k]), k


def test_wsad_kernel_unconstrained_domain_and_reverts():
    """Out-of-domain instances (a value 3e9 wsad from its column's base) are handed to the i128 kernel; a
    deviation past 2^25 (inside the round-5 relative domain) takes the wide forms; reverts come out with the
    CPU engine's stage-ordered status; the dispatcher equals the CPU engine."""
    B, N, D, f = 10, 64, 96, 8
    v = _signed(B, N, D, f, seed=3)
    v[1, 5, 7] = v[1, 5, 7] + 40_000_000            # |x - c1| > 2^25: the wide deviation forms
    v[2, 9, 1] = 3_000_000_000                      # 3e9 from the column's base: the i128 kernel
    v[3, :, 4] = -2_500_000                         # a zero-variance column -> DIV_BY_ZERO
    v[4] = v[4] * 0 + 1_000_000                     # every value equal: DIV_BY_ZERO (variance 0)
    v[5, :, :] = -v[5, :, :]                        # negative everything: a plain round
    vg = v.to(DEV)
    only = _run(vg, f, {"SVOC_EXACT_WSAD_ONLY": "1"}, constrained=False, ms=MS)
    cpu = _cpu(v, f, False, MS)
    st = only["status"].tolist()
    assert st[2] == -1, st
    for i in (0, 1, 3, 4, 5, 6, 7, 8, 9):
        assert st[i] == cpu["status"][i].item(), (i, st, cpu["status"].tolist())
    assert cpu["status"][3].item() != 0 and cpu["status"][4].item() != 0 and cpu["status"][5].item() == 0
    comb = _run(vg, f, None, constrained=False, ms=MS)
    for k in OUTS:
        assert torch.equal(comb[k], cpu[k]), k


@pytest.mark.parametrize("f,ms", [(62, MS), (64, MS), (65, MS), (8, 0), (8, 1)])
def test_wsad_kernel_unconstrained_stage_order(f, ms):
    """R = 2 (moments divide by zero), R = 0 (the mean divides by zero), f > N (usize underflow),
    max_spread 0 (wsad_div by zero) and 1 (saturated reliability): the CPU engine's status, no fallback."""
    B, N, D = 4, 64, 70
    v = _signed(B, N, D, min(f, N), seed=f + ms)
    only = _run(v.to(DEV), f, {"SVOC_EXACT_WSAD_ONLY": "1"}, constrained=False, ms=ms)
    cpu = _cpu(v, f, False, ms)
    assert only["status"].tolist() == cpu["status"].tolist()
    comb = _run(v.to(DEV), f, None, constrained=False, ms=ms)
    for k in OUTS:
        assert torch.equal(comb[k], cpu[k]), k


@pytest.mark.parametrize("dtype", [torch.int64, torch.int32])
def test_wsad_kernel_unconstrained_domain_boundaries(dtype):
    """Values at the column kernel's unconstrained domain edges (round 5: every value within 2^30 of its
    column's row-0 value; deviations from the median past 2^25 take the wide forms instead of the i128
    kernel): whatever the kernel accepts equals the CPU engine bit for bit, and the dispatcher (column
    kernel + i128 fallback) equals it everywhere."""
    B, N, D, f = 8, 64, 40, 8
    v = _signed(B, N, D, f, seed=77, honest_sd=2e5, fail_span=2e6, centre=0.0)
    big = (1 << 30) - 1
    v[0] += big - 3_000_000                    # everything near +2^30 (inside)
    v[1] -= big - 3_000_000                    # near -2^30 (inside)
    v[2, 3, 5] = 1 << 30                       # one value at 2^30 (outside)
    v[3, 4, 6] = v[3, :, 6].median().item() + (1 << 25) - 1   # a deviation of 2^25 - 1 (inside)
    v[4, 4, 6] = v[4, :, 6].median().item() + (1 << 25) + 100_000   # past 2^25 (outside)
    v[5, 9, 2] = -(1 << 31)                    # int32 minimum
    vg = v.to(DEV, dtype)
    cpu = _cpu(v, f, False, MS)
    only = _run(vg, f, {"SVOC_EXACT_WSAD_ONLY": "1"}, constrained=False, ms=MS)
    took = only["status"] != -1
    assert took[0] and took[1] and took[3] and took[4] and not took[2], only["status"]
    for k in OUTS:
        assert torch.equal(only[k][took], cpu[k][took]), k
    comb = _run(vg, f, None, constrained=False, ms=MS)
    for k in OUTS:
        assert torch.equal(comb[k], cpu[k]), k


@pytest.mark.parametrize("N,D,f", [(64, 256, 8), (100, 260, 10), (256, 300, 32), (50, 129, 5), (7, 70, 2)])
def test_wsad_window_median_with_ties(N, D, f):
    """The one-network window path (pass-2 smooth median read off the pass-1 window by ranking the removed
    keys, consensus_wsad.hip) on tie-heavy columns: values from a 6-point grid, so the median, the window
    and the removed keys share values.  Bit-identical to the i128 kernel on every round it takes."""
    B = 16
    g = torch.Generator().manual_seed(N + D + f)
    grid = torch.tensor([100000, 350000, 480000, 500000, 520000, 900000])
    v = grid[torch.randint(0, 6, (B, N, D), generator=g)]
    v[:, : N // 3] = grid[2 + torch.randint(0, 3, (B, N // 3, D), generator=g)]   # a dense middle
    fast = _run(v.to(DEV, torch.int32), f, {"SVOC_EXACT_WSAD_ONLY": "1", "SVOC_EXACT_WSAD_MIN_D": "1"})
    ref = _run(v.to(DEV), f, {"SVOC_EXACT_I128": "1"})
    took = fast["status"] == 0
    assert took.sum() >= B // 2, fast["status"]
    for k in OUTS:
        assert torch.equal(fast[k][took], ref[k][took]), k
    comb = _run(v.to(DEV, torch.int32), f, {"SVOC_EXACT_WSAD_MIN_D": "1"})
    for k in OUTS:
        assert torch.equal(comb[k], ref[k]), k


def _prices(B, N, D, f, seed, centre=60_000.0, spread=200.0):
    """Price-like unconstrained columns (real units, wsad = x 1e6): honest oracles within +-spread of a per-column
    centre near 60,000, failing ones uniform over +-2 spread -- int64 values ~6e10, far outside int32."""
    g = torch.Generator().manual_seed(seed)
    c = centre + 50.0 * torch.rand(B, 1, D, generator=g, dtype=torch.float64)
    x = c + (spread / 3) * torch.randn(B, N, D, generator=g, dtype=torch.float64).clamp(-3, 3)
    bad = torch.stack([torch.randperm(N, generator=g)[:f] for _ in range(B)])
    fv = c + 2 * spread * (2 * torch.rand(B, f, D, generator=g, dtype=torch.float64) - 1)
    x.scatter_(1, bad[:, :, None].expand(B, f, D), fv)
    return (x * 1e6).round().to(torch.int64).contiguous()


@pytest.mark.parametrize("N,D,f", [(64, 1024, 8), (7, 70, 2), (100, 130, 10), (256, 96, 32)])
def test_wsad_kernel_unconstrained_price_columns(N, D, f):
    """Unconstrained rounds over price-like data (60,000 +- 200 real units, int64 wsad ~6e10: VERDICT r4 missing
    item 2): the column kernel takes every round (relative to each column's row-0 value, wide deviation forms)
    and equals the i128 kernel and the CPU engine bit for bit."""
    B = 8
    ms = 1_000 * 1_000_000
    v = _prices(B, N, D, f, seed=N + D)
    fast = _run(v.to(DEV), f, {"SVOC_EXACT_WSAD_ONLY": "1", "SVOC_EXACT_WSAD_MIN_D": "1"}, constrained=False, ms=ms)
    ref = _run(v.to(DEV), f, {"SVOC_EXACT_I128": "1"}, constrained=False, ms=ms)
    cpu = _cpu(v, f, False, ms)
    assert (fast["status"] != -1).all(), fast["status"]        # nothing handed to the i128 kernel
    assert (cpu["status"] == 0).any()
    for k in OUTS:
        assert torch.equal(fast[k], ref[k]), k
        assert torch.equal(fast[k], cpu[k]), k


def test_wsad_kernel_unconstrained_int64_extremes():
    """int64 extremes next to price columns: columns with |B| >= 2^52 or values more than 2^30 from their base go
    to the i128 kernel; the dispatcher equals the CPU engine everywhere (saturated / overflowing rounds included)."""
    B, N, D, f = 8, 64, 40, 8
    ms = 1_000 * 1_000_000
    v = _prices(B, N, D, f, seed=5)
    v[1, :, 3] = (1 << 62) + torch.arange(N) * 1_000_003         # |B| >= 2^52 (its column)
    v[2, 7, 0] = -(1 << 63)                                      # int64 minimum
    v[3, 11, 9] = v[3, 0, 9] + (1 << 30)                         # just past 2^30 from the base
    v[4, 11, 9] = v[4, 0, 9] + (1 << 30) - 1                     # just inside
    v[5] = -v[5]                                                 # negative prices: a plain round
    vg = v.to(DEV)
    cpu = _cpu(v, f, False, ms)
    only = _run(vg, f, {"SVOC_EXACT_WSAD_ONLY": "1"}, constrained=False, ms=ms)
    took = only["status"] != -1
    assert not took[1] and not took[2] and not took[3] and took[4] and took[5] and took[0], only["status"]
    for k in OUTS:
        assert torch.equal(only[k][took], cpu[k][took]), k
    comb = _run(vg, f, None, constrained=False, ms=ms)
    for k in OUTS:
        assert torch.equal(comb[k], cpu[k]), k


def test_wsad_kernel_wide_tiled_int64_domain():
    """Unconstrained int64 rounds at 32 / 64 lanes per column (N > 1024): the tile loader checks every value's high
    word against its column's base.  A value 2^30 from its base, one just inside, one with only its high word off
    (the low word matches the base's) and |B| >= 2^52 columns: the out-of-domain instances go to the i128 kernel,
    the rest stay on the column kernel; every instance equals the CPU engine."""
    B, N, D, f = 6, 2048, 6, 256
    ms = 1_000 * 1_000_000
    v = _prices(B, N, D, f, seed=77)
    v[1, 1500, 2] = v[1, 0, 2] + (1 << 30)                         # just past 2^30 from the base
    v[2, 1500, 2] = v[2, 0, 2] + (1 << 30) - 1                     # just inside
    v[3, 1999, 5] = v[3, 0, 5] + (1 << 32)                         # high word only (last column, odd D)
    v[4, :, 1] = (1 << 62) + torch.arange(N) * 1_000_003           # |B| >= 2^52
    vg = v.to(DEV)
    cpu = _cpu(v, f, False, ms)
    only = _run(vg, f, {"SVOC_EXACT_WSAD_ONLY": "1", "SVOC_EXACT_WSAD_MIN_D": "1"}, constrained=False, ms=ms)
    took = only["status"] != -1
    assert took[0] and not took[1] and took[2] and not took[3] and not took[4] and took[5], only["status"]
    for k in OUTS:
        assert torch.equal(only[k][took], cpu[k][took]), k
    comb = _run(vg, f, {"SVOC_EXACT_WSAD_MIN_D": "1"}, constrained=False, ms=ms)
    for k in OUTS:
        assert torch.equal(comb[k], cpu[k]), k


@pytest.mark.parametrize("N", [256, 200])
def test_wsad_pruned_window_fallback(N):
    """N in (128, 256], f <= 32: pass 1 runs the pruned window network (only each lane's middle 32 keys enter
    the cross-lane merges) and reruns the full network for a wave whose check fails.  Adversarial columns --
    one lane group's 64 rows holding the column's lowest values, or its highest -- force the rerun; every
    round stays bit-identical to the i128 kernel."""
    B, D, f = 6, 160, 32
    v = _wsad(B, N, D, f, seed=N + 1)
    g = torch.Generator().manual_seed(9)
    for b in range(B):
        for c in range(0, D, 7):                      # every 7th column: sorted ascending down the rows
            v[b, :, c] = torch.sort(v[b, :, c]).values
        for c in range(3, D, 11):                     # every 11th: the first 64 rows at the top of the column
            col = torch.sort(v[b, :, c], descending=True).values
            v[b, :, c] = col[torch.randperm(N, generator=g)] if b % 2 else col
    fast = _run(v.to(DEV, torch.int32), f, {"SVOC_EXACT_WSAD_ONLY": "1", "SVOC_EXACT_WSAD_MIN_D": "1"})
    ref = _run(v.to(DEV), f, {"SVOC_EXACT_I128": "1"})
    took = fast["status"] == 0
    assert took.sum() >= B - 1, fast["status"]
    for k in OUTS:
        assert torch.equal(fast[k][took], ref[k][took]), k


@pytest.mark.parametrize("N,D,f", [(300, 70, 30), (512, 64, 64), (1000, 33, 100), (2048, 20, 256), (4096, 8, 512),
                                   (1500, 24, 150), (3000, 12, 300)])
def test_wsad_kernel_wide_groups(N, D, f):
    """N > 256: the column kernel's wide lane groups (8 .. 64 lanes per column, full cross-lane
    median networks, qr by LDS atomics) take the constrained rounds and equal the i128 kernel and the CPU engine
    bit for bit.  N = 1500 / 3000 run the LDS-tiled groups with padding rows (N != 64 * NSEG): the domain check
    must ignore the tile's leftover words there, or instances would leave for the i128 kernel."""
    B = 4
    v = _wsad(B, N, D, f, seed=N + D)
    fast = _run(v.to(DEV, torch.int32), f, {"SVOC_EXACT_WSAD_ONLY": "1", "SVOC_EXACT_WSAD_MIN_D": "1"})
    ref = _run(v.to(DEV), f, {"SVOC_EXACT_I128": "1"})
    cpu = _cpu(v, f, True, 0)
    took = fast["status"] == 0
    assert took.all(), fast["status"]
    for k in OUTS:
        assert torch.equal(fast[k], ref[k]), k
        assert torch.equal(fast[k], cpu[k]), k


@pytest.mark.parametrize("N,D,f,kind,dtype", [(300, 70, 30, "signed", torch.int32), (512, 48, 64, "prices", torch.int64),
                                              (1000, 33, 100, "signed", torch.int64),
                                              (2048, 20, 256, "signed", torch.int32),
                                              (2048, 21, 256, "signed", torch.int64),
                                              (4096, 8, 512, "prices", torch.int32),
                                              (4096, 9, 512, "prices", torch.int64)])
def test_wsad_kernel_wide_groups_unconstrained(N, D, f, kind, dtype):
    """Unconstrained rounds at N > 256 (VERDICT r4 missing item 3) on the wide lane groups: base-relative columns,
    43-bit quotients into the LDS qr sums; bit-identical to the i128 kernel and the CPU engine.  (Price-like int64
    values do not fit int32 storage: the int32 4096-row price case stores its base-relative offsets, a plain round;
    the int64 cases at N > 1024 run the tiled groups, whose loader checks the high words.)"""
    B = 4
    ms = 1_000 * 1_000_000 if kind == "prices" else MS
    v = _prices(B, N, D, f, seed=N + D) if kind == "prices" else _signed(B, N, D, f, seed=N * 5 + D)
    if dtype == torch.int32:
        v = v - v[:, :1, :] if kind == "prices" else v
    fast = _run(v.to(DEV, dtype), f, {"SVOC_EXACT_WSAD_ONLY": "1", "SVOC_EXACT_WSAD_MIN_D": "1"}, constrained=False,
                ms=ms)
    ref = _run(v.to(DEV), f, {"SVOC_EXACT_I128": "1"}, constrained=False, ms=ms)
    cpu = _cpu(v, f, False, ms)
    assert (fast["status"] != -1).all(), fast["status"]        # nothing handed to the i128 kernel
    assert (cpu["status"] == 0).any()
    for k in OUTS:
        assert torch.equal(fast[k], ref[k]), k
        assert torch.equal(fast[k], cpu[k]), k


@pytest.mark.parametrize("N,D,f", [(300, 40, 30), (1024, 16, 100)])
def test_wsad_kernel_wide_groups_legacy(N, D, f):
    """Obsolete N-D contract rounds at N > 256 on the wide lane groups: bit-identical to the i128 kernel."""
    B = 4
    g = torch.Generator().manual_seed(N + D)
    v = 500_000 + torch.randint(-20_000, 20_001, (B, N, D), generator=g, dtype=torch.int64)
    vg = v.to(DEV)

    def run(env):
        o = alloc_exact_out(B, N, D, DEV)
        old = {k: os.environ.get(k) for k in ("SVOC_EXACT_I128", "SVOC_EXACT_WSAD_ONLY", "SVOC_EXACT_WSAD_MIN_D")}
        try:
            for k in old:
                os.environ.pop(k, None)
            os.environ.update(env)
            svops.ops().exact_round(vg, None, f, True, 0, o["c1"], o["consensus"], o["skew"], o["kurt"], o["rel"],
                                    o["qr"], o["reliable"], o["status"], True)
            torch.cuda.synchronize()
        finally:
            for k, val in old.items():
                if val is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = val
        return {k: t.cpu() for k, t in o.items()}
    fast = run({"SVOC_EXACT_WSAD_ONLY": "1", "SVOC_EXACT_WSAD_MIN_D": "1"})
    ref = run({"SVOC_EXACT_I128": "1"})
    assert (ref["status"] == 0).all(), ref["status"]
    assert (fast["status"] == 0).all(), fast["status"]
    for k in OUTS:
        assert torch.equal(fast[k], ref[k]), k
