"""N > 256 oracles on the GPU: the register-streaming fast kernels (bf16 and fp32 storage) with 8 .. 64
lanes per column (pair) -- N up to 4096, full cross-lane bitonic sort, sortnet.hpp median_group_wide
-- and the i128 exact kernel with 8 / 16 rows per lane in registers (N <= 1024) and 32 / 64 rows per
lane in private memory (N <= 4096).  The reference has no oracle cap beyond gas
(contract.cairo:310-329)."""
import pytest
import torch

from helpers import beta_oracles, run_exact, run_fast
from svoc.ops import torch_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("N,D,f,constrained,storage", [
    (300, 64, 30, True, "bf16"), (512, 256, 64, True, "bf16"), (512, 100, 40, False, "bf16"),
    (1000, 96, 100, True, "bf16"), (1024, 130, 50, True, "bf16"), (777, 33, 200, True, "bf16"),
    (2048, 70, 200, True, "bf16"), (1500, 33, 100, False, "bf16"), (4096, 20, 300, True, "bf16"),
    (2048, 70, 200, True, "fp32"), (1500, 33, 100, False, "fp32"), (3000, 20, 300, True, "fp32")])
def test_fast_wide_n_vs_torch(N, D, f, constrained, storage):
    B = 6 if N <= 1024 else 3
    x, _ = beta_oracles(B, N, D, f, seed=N + D, dtype=torch.bfloat16 if storage == "bf16" else torch.float32)
    o = run_fast(x.to(DEV), D, f, constrained, 1.0)
    torch.cuda.synchronize()
    r = torch_ref.fast_round(x.to(DEV)[:, :, :D], f, constrained, 1.0)
    ok = o["status"] == 0
    assert ok.all(), o["status"]
    assert torch.equal(o["reliable"].bool(), r["reliable"])
    torch.testing.assert_close(o["c1"], r["c1"], rtol=0, atol=1e-6)
    torch.testing.assert_close(o["consensus"], r["consensus"], rtol=0, atol=2e-6)
    torch.testing.assert_close(o["qr"], r["qr"], rtol=2e-4, atol=1e-5)
    torch.testing.assert_close(o["rel"], r["rel"], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(o["skew"], r["skew"], rtol=2e-3, atol=2e-3)
    torch.testing.assert_close(o["kurt"], r["kurt"], rtol=2e-3, atol=5e-3)
    oc = run_fast(x, D, f, constrained, 1.0)
    assert torch.equal(oc["status"], o["status"].cpu())


@pytest.mark.parametrize("N,D,f,constrained", [
    (512, 8, 50, True), (1024, 4, 100, True), (1500, 5, 100, True), (2048, 4, 200, True),
    (2048, 3, 150, False), (3000, 3, 300, True), (4096, 2, 300, True), (4096, 2, 400, False)])
def test_exact_wide_n_matches_cpu(N, D, f, constrained):
    B = 3
    x, _ = beta_oracles(B, N, D, f, seed=N + D, dtype=torch.float64)
    v = (x[:, :, :D] * 1e6).to(torch.int64).contiguous()
    ms = 0 if constrained else 2_000_000
    g = run_exact(v.to(DEV), f, constrained, ms)
    c = run_exact(v, f, constrained, ms)
    for k in ("consensus", "skew", "kurt", "rel", "qr", "reliable", "status", "c1"):
        assert torch.equal(g[k].cpu(), c[k]), k
    assert (c["status"] == 0).all(), c["status"]


@pytest.mark.parametrize("N,RPL", [(300, 8), (1000, 16), (2000, 32), (4000, 64)])
def test_exact_wide_n_ties_and_signs_match_cpu(N, RPL):
    """The radix-select medians (8+ rows per lane) on tie-heavy columns (21 distinct values), negative
    keys (unconstrained) and one column of int64 extremes, against the CPU engine."""
    B, D = 2, 4
    x, _ = beta_oracles(B, N, D, N // 8, seed=N, dtype=torch.float64)
    v = (((x[:, :, :D] - 0.5) * 20).round() * 100_000).to(torch.int64).contiguous()
    v[0, :, 3] = torch.randint(-(1 << 62), 1 << 62, (N,), generator=torch.Generator().manual_seed(N))
    for constrained, ms in ((False, 3_000_000), (True, 0)):
        g = run_exact(v.to(DEV), N // 8, constrained, ms)
        c = run_exact(v, N // 8, constrained, ms)
        for k in ("consensus", "skew", "kurt", "rel", "qr", "reliable", "status", "c1"):
            assert torch.equal(g[k].cpu(), c[k]), (constrained, k)


@pytest.mark.parametrize("N", [7, 50, 200])
def test_exact_int64_extremes_variance_match_cpu(N):
    """Unconstrained int64 values near +-2^62: the column variance passes 2^63 (the i128 kernel keeps it
    as i128), skewness / kurtosis against the CPU engine."""
    B, D = 2, 3
    g0 = torch.Generator().manual_seed(N)
    v = torch.randint(-(1 << 62), 1 << 62, (B, N, D), generator=g0)
    v[1, :, 0] = torch.randint(-1000, 1000, (N,), generator=g0)
    g = run_exact(v.to(DEV), 1, False, 1 << 62)
    c = run_exact(v, 1, False, 1 << 62)
    for k in ("consensus", "skew", "kurt", "rel", "qr", "reliable", "status", "c1"):
        assert torch.equal(g[k].cpu(), c[k]), k


@pytest.mark.parametrize("N", [2048, 4096])
def test_exact_wide_n_reverts_match_cpu(N):
    """Reverting rounds at N > 1024 (too many failing oracles; a zero-variance column; an interval
    error from a huge max_spread) give the CPU engine's first-error status and no outputs."""
    B, D = 3, 3
    x, _ = beta_oracles(B, N, D, 100, seed=7, dtype=torch.float64)
    v = (x[:, :, :D] * 1e6).to(torch.int64).contiguous()
    v[1, :, 2] = 500_000   # every row equal in one column: zero variance
    for f, constrained, ms in ((N + 1, True, 0), (100, True, 0), (100, False, 1)):
        g = run_exact(v.to(DEV), f, constrained, ms)
        c = run_exact(v, f, constrained, ms)
        for k in ("consensus", "skew", "kurt", "rel", "qr", "reliable", "status", "c1"):
            assert torch.equal(g[k].cpu(), c[k]), (f, constrained, k)


def test_engine_exact_n4096_round():
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    cfg = ConsensusConfig(n_oracles=4096, dimension=4, n_failing_oracles=512, constrained=True)
    e = ConsensusEngine(cfg, batch=2, device=DEV, mode="exact")
    e.randomize(seed=3)
    e.run_round()
    c = ConsensusEngine(cfg, batch=2, device="cpu", mode="exact")
    c.randomize(seed=3)
    c.values.copy_(e.values.cpu())   # (the device generators differ: same values on both engines)
    c.run_round()
    torch.cuda.synchronize()
    assert torch.equal(e.status.cpu(), c.status) and (c.status == 0).all()
    assert torch.equal(e.consensus.cpu(), c.consensus)
    assert int(e.reliable.sum()) == 2 * (4096 - 512)


def test_engine_n1024_streaming_round():
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    cfg = ConsensusConfig(n_oracles=1024, dimension=256, n_failing_oracles=128, constrained=True)
    e = ConsensusEngine(cfg, batch=4, device=DEV, mode="fast")
    e.randomize(seed=1)
    e.run_round()
    torch.cuda.synchronize()
    assert (e.status == 0).all() and e.consensus_active.all()
    assert int(e.reliable.sum()) == 4 * (1024 - 128)
