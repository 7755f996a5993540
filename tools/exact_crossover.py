"""Exact-mode kernel choice by shape: rounds/s of the column-parallel kernel (forced for every D) vs
the i128 kernel alone, N oracles x D dims, int32 storage -- sets the dispatcher's minimum D.

    python tools/exact_crossover.py [--out profiles/r2_exact_crossover.json]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svoc.config import ConsensusConfig  # noqa: E402
from svoc.engine import ConsensusEngine  # noqa: E402


def rate(N, D, f, B, env):
    for k in ("SVOC_EXACT_I128", "SVOC_EXACT_WSAD_MIN_D"):
        os.environ.pop(k, None)
    os.environ.update(env)
    e = ConsensusEngine(ConsensusConfig(n_oracles=N, dimension=D, n_failing_oracles=f), B, device="cuda", mode="exact")
    e.randomize(seed=1)
    e.touched.fill_(1)
    e.run_round(only_touched=False)
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        e.run_round(only_touched=False)
    torch.cuda.synchronize()
    return B * reps / (time.perf_counter() - t0), int((e.status == 0).sum())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = []
    for N, D, f in [(7, 6, 2), (16, 16, 3), (64, 16, 8), (64, 32, 8), (64, 64, 8), (64, 128, 8), (256, 64, 32)]:
        B = max(1024, min(1 << 20, (1 << 26) // (N * D)))
        col, ok1 = rate(N, D, f, B, {"SVOC_EXACT_WSAD_MIN_D": "1"})
        i128, ok2 = rate(N, D, f, B, {"SVOC_EXACT_I128": "1"})
        rows.append(dict(N=N, D=D, f=f, batch=B, column_parallel=col, i128=i128, ok=[ok1, ok2]))
        print(json.dumps(rows[-1]), flush=True)
    if a.out:
        json.dump(rows, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
