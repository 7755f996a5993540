"""Reverted rounds leave every output untouched on the GPU, exactly like the CPU twin.

The reference reverts the whole transaction on any failed assert (contract.cairo:588-603): a zero
variance column (sqrt(0) -> wsad_div by zero, math.cairo:322,331), a reliability outside [0, 1]
(contract.cairo:467,488) or fewer than 4 reliable oracles (kurtosis (n-2)(n-3) = 0, math.cairo:362).
Every fast HIP kernel (window, register-streaming, small-instance) stages its pass-2
outputs and commits only when the instance's final status is OK; the pass-1 essence c1 is staged by the
op and committed by svoc_commit_rows on the same condition.
"""
import pytest
import torch

from helpers import alloc_fast_out, beta_oracles
from svoc import ops as svops

pytestmark = pytest.mark.gpu
DEV = "cuda"
SENT = {"consensus": 7.25, "skew": -3.5, "kurt": 11.0, "rel": 0.125, "qr": 42.0, "reliable": 9, "c1": 0.8125}
OUTS = ("consensus", "skew", "kurt", "rel", "qr", "reliable", "c1")


def _run(x, D, f, constrained, active, hint):
    B, N = x.shape[:2]
    o = alloc_fast_out(B, N, D, x.device)
    for k, v in SENT.items():
        o[k].fill_(v)
    svops.ops().fast_round(x, active, D, f, constrained, 1.0, o["c1"], o["consensus"], o["skew"], o["kurt"],
                           o["rel"], o["qr"], o["reliable"], o["status"], hint, 0, 0, False, None)
    return o


# (N, D, f, constrained, wave_hint): window kernel (H 5 / 17, NSEG 1 / 2 / 4, unconstrained), the
# register-streaming kernel (forced, f > 32), the small kernel
CASES = [(64, 1024, 8, True, 0), (256, 600, 32, True, 0), (128, 512, 16, True, 0), (100, 260, 10, False, 0),
         (64, 1024, 8, True, -7), (128, 300, 40, True, 0), (64, 1000, 8, False, -7), (64, 256, 8, True, -7),
         (200, 136, 20, False, -7), (7, 6, 2, True, 0), (16, 100, 3, False, 0)]


@pytest.mark.parametrize("N,D,f,constrained,hint", CASES)
def test_revert_leaves_outputs_untouched(N, D, f, constrained, hint):
    B = 6
    x, _ = beta_oracles(B, N, D, f, seed=N + 3 * D)
    x[1, :, min(3, D - 1)] = 0.5                 # one constant column: zero variance over the reliable rows
    if constrained:
        x[2, : N // 2 + 1, :D] = 0.0             # c1 = 0, N/2 - 1 rows at distance 1: rel1 < 0
        x[2, N // 2 + 1:, :D] = 1.0
    active = torch.tensor([1, 1, 1, 0, 1, 1], dtype=torch.uint8)
    o = _run(x.to(DEV), D, f, constrained, active.to(DEV), hint)
    oc = _run(x, D, f, constrained, active, 0)
    torch.cuda.synchronize()
    st = o["status"].cpu()
    assert torch.equal(st, oc["status"]), (st, oc["status"])
    assert st[1] == 32 and st[3] == -1 and st[0] == 0 and st[4] == 0 and st[5] == 0
    if constrained:
        assert st[2] == 6
    for k in OUTS:
        g = o[k].cpu()
        for b in range(B):
            untouched = bool((g[b] == SENT[k]).all())
            assert untouched == (st[b] != 0), (k, b, st[b])
            # the CPU twin writes exactly the same set of instances
            assert bool((oc[k][b] == SENT[k]).all()) == untouched, (k, b)


@pytest.mark.parametrize("N,D,hint", [(64, 512, 0), (34, 512, 0), (64, 512, -7), (8, 6, 0), (40, 200, -7)])
def test_too_few_reliable_reverts(N, D, hint):
    """f = N - 3: three reliable oracles, kurtosis undefined -> every round reverts."""
    B, f = 4, N - 3
    x, _ = beta_oracles(B, N, D, f, seed=5)
    o = _run(x.to(DEV), D, f, True, None, hint)
    torch.cuda.synchronize()
    assert o["status"].cpu().tolist() == [33] * B
    for k in OUTS:
        assert bool((o[k].cpu() == SENT[k]).all()), k


def test_engine_revert_keeps_previous_round():
    """Engine level: a committed round, then a reverting update -- the outputs stay bit for bit."""
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    cfg = ConsensusConfig(n_oracles=64, dimension=1024, n_failing_oracles=8, constrained=True)
    e = ConsensusEngine(cfg, batch=8, device=DEV, mode="fast")
    e.randomize(seed=3)
    e.run_round()
    assert (e.status == 0).all()
    snap = {k: getattr(e, k).clone() for k in ("consensus", "skew", "kurt", "rel", "qr", "reliable", "c1")}
    inst = torch.tensor([2] * 64, device=DEV)
    orc = torch.arange(64, device=DEV)
    vals = torch.full((64, 1024), 0.5, device=DEV)      # every oracle of instance 2 -> one point
    e.apply_updates(inst, orc, vals)
    e.run_round()
    torch.cuda.synchronize()
    assert e.status[2].item() == 32
    for k, v in snap.items():
        assert torch.equal(getattr(e, k), v), k
