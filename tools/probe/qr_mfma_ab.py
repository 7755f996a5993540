"""A/B of the quadratic-risk pass on the VALU vs the matrix cores (tools/probe/qr_probe.hip), on
the c2 and c3 shapes: kernel time (HIP events) and precision against fp64 -- max relative error of
qr and the number of instances whose (qr asc, idx desc) rank mask differs from the fp64 one
(contract.cairo:345-363).

    python tools/qr_mfma_ab.py [--out profiles/r2_qr_mfma_ab.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)

from build import qr_probe  # noqa: E402  (tools/probe/build.py)
from svoc.models.oracle_gen import beta_failing_oracles  # noqa: E402


def rank_mask(qr: torch.Tensor, R: int) -> torch.Tensor:
    B, N = qr.shape
    idx = torch.arange(N, device=qr.device).expand(B, N)
    by_desc = torch.argsort(-idx, dim=1, stable=True)
    order = torch.gather(by_desc, 1, torch.argsort(torch.gather(qr, 1, by_desc), dim=1, stable=True))
    rank = torch.empty_like(order)
    rank.scatter_(1, order, torch.arange(N, device=qr.device).expand(B, N))
    return rank < R


def case(name, B, N, D, f, reps=20):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    ld = (D + 15) // 16 * 16
    x = torch.zeros(B, N, ld, dtype=torch.bfloat16, device=dev)
    for s in range(0, B, 256):
        e = min(B, s + 256)
        x[s:e, :, :D] = beta_failing_oracles(e - s, N, D, f, 20.0, g, dev).to(torch.bfloat16)
    xs = x[:, :, :D].float()
    # the contract's pass-1 centre: smooth median per column (mean of ranks N/2 - 1, N/2)
    srt = torch.sort(xs, dim=1).values
    c1 = (0.5 * (srt[:, N // 2 - 1] + srt[:, N // 2])).contiguous()
    del srt
    out = {"name": name, "B": B, "N": N, "D": D, "f": f}
    ref = torch.empty(B, N, dtype=torch.float64, device=dev)
    for s in range(0, B, 64):
        e = min(B, s + 64)
        ref[s:e] = ((xs[s:e].double() - c1[s:e, None].double()) ** 2).sum(-1)
    ref_mask = rank_mask(ref, N - f)
    for v, vn in ((0, "valu"), (1, "mfma")):
        qr = torch.empty(B, N, dtype=torch.float32, device=dev)
        op = qr_probe
        op(x, c1, qr, v)
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(reps):
            op(x, c1, qr, v)
        t1.record()
        torch.cuda.synchronize()
        us = 1e3 * t0.elapsed_time(t1) / reps
        rel = ((qr.double() - ref).abs() / ref.abs().clamp_min(1e-30)).max().item()
        mism = int((rank_mask(qr.double(), N - f) != ref_mask).any(1).sum())
        out[vn] = {"us": us, "GBps": B * N * D * 2 / us / 1e3, "max_rel_err_vs_fp64": rel,
                   "instances_with_rank_mask_differing_from_fp64": mism}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = [case("c3", 1024, 256, 4096, 32), case("c2", 10000, 64, 1024, 8)]
    for r in rows:
        print(json.dumps(r))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
