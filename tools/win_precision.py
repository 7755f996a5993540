"""Precision of the window kernel's reliable moments (all-row minus removed-row power sums) against
the exact cleanup path, bucketed by the cancellation ratio max(sum_all d^2 / sum_R d^2, same for d^4).
python tools/win_precision.py  ->  max |skew| / |kurt| deviation per ratio bucket (fp32 both)."""
import os
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from helpers import beta_oracles, run_fast  # noqa: E402


def case(name, x, D, f):
    xg = x.cuda()
    os.environ["SVOC_WIN_CANCEL"] = "1e30"
    sub = run_fast(xg, D, f, True)
    os.environ["SVOC_WIN_CANCEL"] = "1"
    ex = run_fast(xg, D, f, True)
    torch.cuda.synchronize()
    ok = (ex["status"] == 0) & (sub["status"] == 0)
    xf = xg[:, :, :D].float()
    d = xf - ex["c1"][:, None, :]
    rel = ex["reliable"].bool()[:, :, None]
    a2, a4 = (d ** 2).sum(1), (d ** 4).sum(1)
    r2, r4 = (d ** 2 * rel).sum(1), (d ** 4 * rel).sum(1)
    ratio = torch.maximum(a2 / r2.clamp_min(1e-30), a4 / r4.clamp_min(1e-30))
    es = (sub["skew"] - ex["skew"]).abs()
    ek = (sub["kurt"] - ex["kurt"]).abs()
    print(f"== {name}: {int(ok.sum())} instances ok")
    for lo, hi in ((0, 16), (16, 32), (32, 64), (64, 128), (128, 256), (256, 1024), (1024, 1e9)):
        m = ok[:, None] & (ratio >= lo) & (ratio < hi)
        if m.any():
            print(f"  ratio [{lo:>5}, {hi:>6}): {int(m.sum()):>8} cols  max|dskew| {es[m].max():.2e}  "
                  f"max|dkurt| {ek[m].max():.2e}  p99|dkurt| {ek[m].float().quantile(0.99) if m.sum() < 1e7 else 0:.2e}")


x, _ = beta_oracles(400, 64, 1024, 8, seed=1)
case("c2-like 64x1024 f=8 Beta(20,20)", x, 1024, 8)
x, _ = beta_oracles(64, 256, 1024, 32, seed=2)
case("c3-like 256x1024 f=32", x, 1024, 32)
x, _ = beta_oracles(200, 64, 1024, 8, a=200.0, seed=3)
case("tight honest Beta(200,200), 64x1024 f=8", x, 1024, 8)
x, _ = beta_oracles(64, 256, 1024, 32, a=1000.0, seed=4)
case("very tight honest Beta(1000,1000), 256x1024 f=32", x, 1024, 32)
