"""Per-phase kernel timing of the fast round on one config: reg (two networks) vs win (one network),
fused and split (mode 1 = pass 1, mode 2 = rank mask + pass 2).  python tools/win_phases.py [N D f B]"""
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from helpers import alloc_fast_out, beta_oracles, fast_work  # noqa: E402
from svoc import ops as svops  # noqa: E402

N, D, f, B = (int(a) for a in (sys.argv[1:5] if len(sys.argv) > 4 else (256, 4096, 32, 1024)))
x, _ = beta_oracles(B, N, D, f, seed=1)
x = x.cuda()
o = alloc_fast_out(B, N, D, "cuda")
w = fast_work(B, D, "cuda")
op = svops.ops().fast_round


def run(hint, mode, work):
    op(x, None, D, f, True, 1.0, o["c1"], o["consensus"], o["skew"], o["kurt"], o["rel"], o["qr"],
       o["reliable"], o["status"], hint, mode, D, False, work)


def t(name, fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    print(f"{name:28s} {a.elapsed_time(b) / reps * 1e3:9.1f} us", flush=True)


t("reg fused (hint -7)", lambda: run(-7, 0, None))
t("reg mode1", lambda: run(0, 1, None))
t("reg mode2", lambda: run(0, 2, None))
t("win fused", lambda: run(0, 0, w))
t("win mode1", lambda: run(0, 1, w))
t("win mode2", lambda: run(0, 2, w))
run(0, 0, w)
torch.cuda.synchronize()
# host view of the reliable sums' conditioning on instance 0
xf = x[0, :, :D].float()
rel = o["reliable"][0].bool()
c1 = o["c1"][0]
d = xf - c1
sa2, sa4 = (d ** 2).sum(0), (d ** 4).sum(0)
sr2, sr4 = (d[rel] ** 2).sum(0), (d[rel] ** 4).sum(0)
r2, r4 = sa2 / sr2, sa4 / sr4
print("instance 0: ratio d^2 median %.2f max %.2f; d^4 median %.2f max %.2f; >32: %d of %d" % (
    r2.median(), r2.max(), r4.median(), r4.max(), int(((r2 > 32) | (r4 > 32)).sum()), D))
import os  # noqa: E402
for wc in ("1e30", "64", "1"):
    os.environ["SVOC_WIN_CANCEL"] = wc
    t(f"win fused cancel={wc}", lambda: run(0, 0, w))
    t(f"win mode2 cancel={wc}", lambda: run(0, 2, w))
