"""The detector reproduces the reference's published statistical benchmark (documentation/README.md)."""
import math

import pytest

from svoc import ops as svops
from svoc.bench import statistical as stat


def _check(rows, trials):
    for r in rows:
        (slo, shi), (rlo, rhi) = r["published_success"], r["published_reliability"]
        p = r["notebook_success"] / 100
        # published values are K=300 Monte Carlo draws: allow 3 sigma of that noise plus ours
        tol = 300 * math.sqrt(max(p * (1 - p), 0.003) / 300) / 100 * 100 + 300 * math.sqrt(max(p * (1 - p), 0.003) / trials)
        assert slo - tol <= r["notebook_success"] <= shi + tol, r
        assert rlo - 1.0 <= r["notebook_reliability"] <= rhi + 1.0, r
        # the contract's own estimator is statistically indistinguishable on this benchmark
        assert abs(r["contract_success"] - r["notebook_success"]) < 4.0, r


@pytest.mark.skipif(not svops.available(), reason="svoc/_C.so not built")
def test_statistical_benchmark_cpu():
    grid = [(7, 2, 10), (7, 2, 100), (20, 2, 30), (20, 15, 100)]
    trials = 6000
    _check(stat.run(trials, "cpu", grid=grid), trials)


@pytest.mark.gpu
def test_statistical_benchmark_gpu_1m():
    trials = 1_000_000
    _check(stat.run(trials, "cuda"), trials)
