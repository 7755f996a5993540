"""The reference's math prototypes (contract/drafts/*.ipynb), batched on the device.

These notebooks are where the consensus algorithm was designed; they hold estimators and generators
that the contract does not (survey C46/C47).  Each function here is a batched ``torch`` version of one
notebook function (B independent draws at once, any device), with the notebook's behaviour kept:

* ``beta_kumaraswamy_algorithm_demo copy.ipynb``: ``beta_mode`` / ``kumaraswamy_mode`` (cell 4),
  ``expected_reliability`` (cell 13), ``kumaraswamy_sample`` (the distribution the notebook is named
  after; inverse-CDF sampling), ``generate_2d_beta_oracles`` (cell 3; the 1-D generator and the
  detector benchmark live in :mod:`svoc.bench.statistical`).
* ``gaussian_algorithm_demo.ipynb``: the arctan normalisation ``normalize`` / ``denormalize`` and its
  generator (cell 4), and the rejected iterative detector ``remove_worst_oracles`` (cell 11) -- mean
  essence, squared-distance scores, one oracle removed per iteration.  The notebook removes the
  ``argmin`` score, i.e. the *closest* oracle (a prototype bug, kept by default; ``worst="max"``
  removes the farthest instead).
* ``gaussian_distribution_for_tests.ipynb``: ``generate_2d_gaussian_oracles`` (cell 3), whose failing
  oracles are ``U(mu, 5 sigma)`` per component -- the generator of the unconstrained test fixture.
"""
from __future__ import annotations

import math
from typing import Tuple

import torch


def beta_mode(a: float, b: float) -> float:
    return (a - 1) / (a + b - 2)


def kumaraswamy_mode(a: float, b: float) -> float:
    return ((a - 1) / (a * b - 1)) ** (1 / a)


def kumaraswamy_sample(shape, a: float, b: float, gen: torch.Generator, device="cpu") -> torch.Tensor:
    """Kumaraswamy(a, b) by inverse CDF: x = (1 - (1 - u)^(1/b))^(1/a)."""
    u = torch.rand(shape, generator=gen, device=device, dtype=torch.float64)
    return (1 - (1 - u) ** (1 / b)) ** (1 / a)


def expected_reliability(x: torch.Tensor) -> torch.Tensor:
    """1 - 2 * mean |x - median(x)| over the last axis (numpy median: mean of the middle pair)."""
    s, _ = torch.sort(x, dim=-1)
    n = x.shape[-1]
    med = 0.5 * (s[..., (n - 1) // 2] + s[..., n // 2])
    return 1 - 2 * (x - med[..., None]).abs().mean(-1)


def normalize(x: torch.Tensor) -> torch.Tensor:
    return torch.atan(x) / math.pi + 0.5


def denormalize(y: torch.Tensor) -> torch.Tensor:
    return torch.tan(math.pi * (y - 0.5))


def _shuffle_failing(B: int, N: int, f: int, gen, device) -> torch.Tensor:
    """[B, N] bool: the f failing slots of each draw after the notebook's shuffle."""
    perm = torch.argsort(torch.rand(B, N, generator=gen, device=device), dim=1)
    return perm < f


def generate_normalized_gaussian_oracles(B: int, N: int, f: int, e: float, sigma: float, gen,
                                         device="cpu") -> Tuple[torch.Tensor, torch.Tensor]:
    """gaussian_algorithm_demo cell 4: honest = normalize(N(denormalize(e), sigma)), failing U(0,1)."""
    honest = normalize(denormalize(torch.tensor(e, dtype=torch.float64)) +
                       sigma * torch.randn(B, N, generator=gen, device=device, dtype=torch.float64))
    fail = torch.rand(B, N, generator=gen, device=device, dtype=torch.float64)
    m = _shuffle_failing(B, N, f, gen, device)
    return torch.where(m, fail, honest), ~m


def generate_2d_beta_oracles(B: int, N: int, f: int, a: Tuple[float, float], b: Tuple[float, float], gen,
                             device="cpu") -> Tuple[torch.Tensor, torch.Tensor]:
    """beta_kumaraswamy demo cell 3: honest component d ~ Beta(a[d], b[d]), failing U(0,1)^2."""
    cols = [torch.distributions.Beta(torch.tensor(float(a[d])), torch.tensor(float(b[d]))).sample((B, N)).double()
            for d in range(2)]
    honest = torch.stack(cols, -1).to(device)
    fail = torch.rand(B, N, 2, generator=gen, device=device, dtype=torch.float64)
    m = _shuffle_failing(B, N, f, gen, device)
    return torch.where(m[..., None], fail, honest), ~m


def generate_2d_gaussian_oracles(B: int, N: int, f: int, mu, sigma, gen, device="cpu") -> Tuple[torch.Tensor, torch.Tensor]:
    """gaussian_distribution_for_tests cell 3: honest ~ N(mu, sigma), failing ~ U(mu, 5 sigma)."""
    mu_t = torch.tensor(mu, dtype=torch.float64, device=device)
    sg_t = torch.tensor(sigma, dtype=torch.float64, device=device)
    honest = mu_t + sg_t * torch.randn(B, N, len(mu), generator=gen, device=device, dtype=torch.float64)
    u = torch.rand(B, N, len(mu), generator=gen, device=device, dtype=torch.float64)
    fail = mu_t + u * (5 * sg_t - mu_t)
    m = _shuffle_failing(B, N, f, gen, device)
    return torch.where(m[..., None], fail, honest), ~m


def remove_worst_oracles(x: torch.Tensor, n_failing: int, worst: str = "min") -> Tuple[torch.Tensor, torch.Tensor]:
    """gaussian_algorithm_demo cell 11, batched: x [B, N] or [B, N, D].

    Repeat ``n_failing`` times: essence = mean of the still-active oracles, score = squared distance
    to it, deactivate the active oracle with the min (notebook) or max score.  Returns
    (active mask [B, N], final scores [B, N] against the final essence, all oracles scored)."""
    xv = x if x.dim() == 3 else x[..., None]
    B, N, _ = xv.shape
    active = torch.ones(B, N, dtype=torch.bool, device=x.device)
    big = torch.finfo(xv.dtype).max
    for _ in range(n_failing):
        w = active.to(xv.dtype)[..., None]
        essence = (xv * w).sum(1) / w.sum(1)
        score = ((xv - essence[:, None]) ** 2).sum(-1)
        if worst == "min":
            pick = torch.where(active, score, torch.full_like(score, big)).argmin(1)
        else:
            pick = torch.where(active, score, torch.full_like(score, -big)).argmax(1)
        active[torch.arange(B, device=x.device), pick] = False
    w = active.to(xv.dtype)[..., None]
    essence = (xv * w).sum(1) / w.sum(1)
    return active, ((xv - essence[:, None]) ** 2).sum(-1)
