"""N > 256 oracles on the GPU: the register-streaming fast kernels (bf16 and fp32 storage) with 8 .. 64
lanes per column (pair) -- N up to 4096, full cross-lane bitonic sort, sortnet.hpp median_group_wide
-- and the i128 exact kernel with 8 / 16 rows per lane (N <= 1024).  The reference has no oracle cap
beyond gas (contract.cairo:310-329)."""
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


@pytest.mark.parametrize("N,D,f", [(512, 8, 50), (1024, 4, 100)])
def test_exact_wide_n_matches_cpu(N, D, f):
    B = 3
    x, _ = beta_oracles(B, N, D, f, seed=N, dtype=torch.float64)
    v = (x[:, :, :D] * 1e6).to(torch.int64).contiguous()
    g = run_exact(v.to(DEV), f, True)
    c = run_exact(v, f, True)
    for k in ("consensus", "skew", "kurt", "rel", "qr", "reliable", "status", "c1"):
        assert torch.equal(g[k].cpu(), c[k]), k
    assert (c["status"] == 0).all()


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
