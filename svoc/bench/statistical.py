"""Statistical benchmark of the failing-oracle detector (documentation/README.md:191-341).

Reproduces the reference's only published numbers -- identification success and "true consensus
reliability" -- as a batched Monte Carlo on the device, with many more trials than the notebook's
K = 300 (contract/drafts/beta_kumaraswamy_algorithm_demo copy.ipynb cells 17-21):

* ``notebook`` estimator: 1-D oracles, f failing ~ U(0,1), honest ~ Beta(a, a) (the notebook ignores
  its ``b`` argument, survey §2.8-11), shuffled; median = numpy median (mean of the two middle values
  for even N); failing = the f largest |x - median|; success = exact mask match; distance =
  |median(predicted reliable) - median(true reliable)|; reliability = 100 (1 - 2 mean distance).
* ``contract`` estimator: the same draws quantised to wsad as the client does (int(x * 1e6),
  client/contract.py:48-53) and pushed through one EXACT consensus round each (smooth median, wsad
  squared risk, (qr asc, idx desc) rank mask -- the column-parallel exact kernel on GPU, the C++
  golden engine on CPU), scored with the ``reliable`` flags that round wrote.  Rounds the contract
  would revert (none on these draws in practice) are excluded and counted.

    python -m svoc.bench.statistical --trials 1000000 [--device cuda] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import math
import time
from typing import Dict, List, Tuple

import torch

# published tables (documentation/README.md:248-341): (N, f) -> a -> (success range %, reliability range %)
PUBLISHED: Dict[Tuple[int, int], Dict[int, Tuple[Tuple[float, float], Tuple[float, float]]]] = {
    (7, 2): {10: ((33.00, 40.33), (94.00, 95.92)), 20: ((43.00, 58.33), (97.15, 97.94)),
             30: ((58.33, 63.33), (97.75, 98.53)), 100: ((71.67, 76.33), (99.29, 99.53))},
    (20, 2): {10: ((25.33, 33.33), (98.58, 98.76)), 20: ((42.00, 46.33), (99.27, 99.35)),
              30: ((49.00, 57.33), (99.52, 99.64)), 100: ((69.33, 78.33), (99.81, 99.86))},
    (20, 15): {10: ((0.33, 2.00), (89.04, 90.60)), 20: ((1.33, 2.67), (90.76, 92.74)),
               30: ((1.67, 4.33), (92.89, 93.76)), 100: ((10.67, 13.67), (95.16, 96.53))},
}


def np_median(x: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """numpy.median over the masked entries of each row (mean of the two middle values if even)."""
    k = mask.sum(1)
    s, _ = torch.sort(torch.where(mask, x, torch.full_like(x, float("inf"))), dim=1)
    lo = torch.gather(s, 1, ((k - 1) // 2).clamp(min=0)[:, None]).squeeze(1)
    hi = torch.gather(s, 1, (k // 2).clamp(max=x.shape[1] - 1)[:, None]).squeeze(1)
    return 0.5 * (lo + hi)


def draw(B: int, N: int, f: int, a: float, gen: torch.Generator, device) -> Tuple[torch.Tensor, torch.Tensor]:
    """generate_beta_oracles (notebook cell 3): returns x [B, N] and the true-reliable mask."""
    from ..models.oracle_gen import beta_failing_oracles
    x, failing = beta_failing_oracles(B, N, 1, f, a, gen, device, return_mask=True)
    return x[:, :, 0].double(), ~failing


def notebook_estimator(x: torch.Tensor, f: int) -> torch.Tensor:
    """identify_failing_oracles (documentation/README.md:207-212): reliable mask [B, N]."""
    B, N = x.shape
    med = np_median(x, torch.ones_like(x, dtype=torch.bool))
    dev = (x - med[:, None]).abs()
    order = torch.argsort(dev, dim=1, stable=True)           # ascending deviation
    rank_from_top = torch.empty_like(order)
    rank_from_top.scatter_(1, order, (N - 1 - torch.arange(N, device=x.device)).expand(B, N))
    return rank_from_top >= f


def contract_estimator(x: torch.Tensor, f: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """The contract's own rank mask: (reliable [B, N], round succeeded [B]) of one exact round per trial."""
    from .. import ops as svops
    B, N = x.shape
    vals = (x * 1e6).floor().to(torch.int32).reshape(B, N, 1).contiguous()
    i64 = dict(dtype=torch.int64, device=x.device)
    c1, cons, sk, ku = (torch.zeros(B, 1, **i64) for _ in range(4))
    rel, qr = torch.zeros(B, 2, **i64), torch.zeros(B, N, **i64)
    reliable = torch.zeros(B, N, dtype=torch.uint8, device=x.device)
    st = torch.full((B,), -1, dtype=torch.int32, device=x.device)
    svops.ops().exact_round(vals, None, f, True, 0, c1, cons, sk, ku, rel, qr, reliable, st, False)
    return reliable.bool(), st == 0


def score(x: torch.Tensor, pred: torch.Tensor, truth: torch.Tensor) -> Tuple[float, float]:
    success = (pred == truth).all(1).double().mean().item()
    d = (np_median(x, pred) - np_median(x, truth)).abs().mean().item()
    return 100.0 * success, 100.0 * (1.0 - 2.0 * d)


def run(trials: int, device="cpu", chunk: int = 1 << 18, seed: int = 0, estimators=("notebook", "contract"),
        grid=None) -> List[dict]:
    grid = grid or [(n, f, a) for (n, f), d in PUBLISHED.items() for a in d]
    gen = torch.Generator(device=device).manual_seed(seed)
    out = []
    for N, f, a in grid:
        acc = {e: [0.0, 0.0, 0] for e in estimators}   # success sum, reliability sum, scored trials
        done = 0
        t0 = time.perf_counter()
        while done < trials:
            B = min(chunk, trials - done)
            x, truth = draw(B, N, f, a, gen, device)
            for e in estimators:
                if e == "notebook":
                    pred, ok = notebook_estimator(x, f), None
                else:
                    pred, ok = contract_estimator(x, f)
                xs, ps, ts = (x, pred, truth) if ok is None else (x[ok], pred[ok], truth[ok])
                n = xs.shape[0]
                if n:
                    s, r = score(xs, ps, ts)
                    acc[e][0] += s * n
                    acc[e][1] += r * n
                    acc[e][2] += n
            done += B
        row = dict(N=N, f=f, a=a, trials=trials, seconds=time.perf_counter() - t0)
        for e in estimators:
            n = max(acc[e][2], 1)
            row[f"{e}_success"] = acc[e][0] / n
            row[f"{e}_reliability"] = acc[e][1] / n
            if e == "contract":
                row["contract_reverted"] = trials - acc[e][2]
        pub = PUBLISHED.get((N, f), {}).get(a)
        if pub:
            row["published_success"] = pub[0]
            row["published_reliability"] = pub[1]
            # binomial standard error of the published K=300 estimates, for the agreement check
            p = row.get("notebook_success", 50.0) / 100
            row["published_se_pp"] = 100 * math.sqrt(max(p * (1 - p), 1e-4) / 300)
        out.append(row)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=100_000)
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    rows = run(a.trials, a.device)
    hdr = f"{'N/f':>6} {'a':>4} | {'notebook succ':>13} {'rel':>7} | {'contract succ':>13} {'rel':>7} | published succ / rel"
    print(hdr)
    for r in rows:
        ps, pr = r.get("published_success", ("-", "-")), r.get("published_reliability", ("-", "-"))
        print(f"{r['N']:>3}/{r['f']:<2} {r['a']:>4} | {r['notebook_success']:>12.2f}% {r['notebook_reliability']:>6.2f}% | "
              f"{r['contract_success']:>12.2f}% {r['contract_reliability']:>6.2f}% | {ps} / {pr}")
    if a.json:
        json.dump(rows, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
