"""Window kernel: the exact cleanup path forced for every column (SVOC_WIN_CANCEL=1) and never
(1e30) must agree with the two-network kernel; repeated split-mode calls on one workspace."""
import os

import pytest
import torch

from helpers import alloc_fast_out, beta_oracles, fast_work, run_fast
from svoc import ops as svops
from test_win_gpu import _same

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("cancel", ["1", "1e30"])
@pytest.mark.parametrize("N,D,f,constrained", [(64, 300, 8, True), (256, 520, 32, True), (100, 130, 10, False),
                                               (40, 64, 4, False)])
def test_win_cleanup_forced(cancel, N, D, f, constrained, monkeypatch):
    monkeypatch.setenv("SVOC_WIN_CANCEL", cancel)
    x, _ = beta_oracles(8, N, D, f, seed=N * 7 + D)
    xg = x.to(DEV)
    win = run_fast(xg, D, f, constrained)
    reg = run_fast(xg, D, f, constrained, wave_hint=-7)
    torch.cuda.synchronize()
    ok = _same(win, reg, constrained)
    assert ok.all()


def test_win_repeated_mode2_is_idempotent(monkeypatch):
    monkeypatch.setenv("SVOC_WIN_CANCEL", "1")
    B, N, D, f = 6, 128, 400, 16
    x, _ = beta_oracles(B, N, D, f, seed=3)
    xg = x.to(DEV)
    o = alloc_fast_out(B, N, D, DEV)
    w = fast_work(B, D, DEV)
    args = (xg, None, D, f, True, 1.0, o["c1"], o["consensus"], o["skew"], o["kurt"], o["rel"], o["qr"],
            o["reliable"], o["status"], 0)
    svops.ops().fast_round(*args, 1, D, False, w)
    outs = []
    for _ in range(3):
        svops.ops().fast_round(*args, 2, D, False, w)
        torch.cuda.synchronize()
        outs.append({k: v.clone() for k, v in o.items()})
    for k in o:
        assert torch.equal(outs[0][k], outs[2][k]), k
