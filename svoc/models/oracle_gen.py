"""Synthetic oracle streams (device RNG).

Mirrors the reference's stochastic oracles: honest oracles concentrate around the truth, the first
``f`` are failing and draw ``U(0,1)^D``, then the list is shuffled
(client/oracle_scheduler.py:73-92; notebook ``generate_beta_oracles`` /
``generate_2d_beta_oracles``, contract/drafts/beta_kumaraswamy_algorithm_demo copy.ipynb cell 3).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch


def failing_mask(B: int, N: int, f: int, gen: torch.Generator, device) -> torch.Tensor:
    """Exactly f failing oracles per instance at uniformly random positions (the shuffle)."""
    keys = torch.rand(B, N, generator=gen, device=device)
    rank = keys.argsort(dim=1).argsort(dim=1)
    return rank < f


def beta_failing_oracles(B: int, N: int, D: int, f: int, a: float, gen: torch.Generator, device,
                         b: Optional[float] = None, return_mask: bool = False):
    """[B, N, D] fp32: Beta(a, b or a) honest components, U(0,1) failing rows."""
    b = a if b is None else b
    # Beta via two gammas (torch.distributions.Beta has no generator argument)
    ga = torch._standard_gamma(torch.full((B, N, D), float(a), device=device), generator=gen)
    gb = torch._standard_gamma(torch.full((B, N, D), float(b), device=device), generator=gen)
    honest = ga / (ga + gb)
    fail = torch.rand(B, N, D, generator=gen, device=device)
    m = failing_mask(B, N, f, gen, device)
    x = torch.where(m[:, :, None], fail, honest)
    return (x, m) if return_mask else x


def gaussian_failing_oracles(B: int, N: int, D: int, f: int, mu: torch.Tensor, sigma: torch.Tensor,
                             spread: float, gen: torch.Generator, device) -> Tuple[torch.Tensor, torch.Tensor]:
    """Unconstrained fixture generator (gaussian_distribution_for_tests.ipynb): honest ~ N(mu, sigma),
    failing ~ U(mu - spread, mu + spread)."""
    honest = mu + sigma * torch.randn(B, N, D, generator=gen, device=device)
    fail = mu + spread * (2 * torch.rand(B, N, D, generator=gen, device=device) - 1)
    m = failing_mask(B, N, f, gen, device)
    return torch.where(m[:, :, None], fail, honest), m
