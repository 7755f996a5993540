"""Plain-PyTorch fp32 reference of the fast consensus round (same algorithm, batched).

Used only by the numerics tests: the HIP kernel (csrc/kernels/consensus_fast.hip) and the C++ fast
engine are compared against this.  Semantics follow contract/src/contract.cairo:442-503 in real
units: smooth median = mean of sorted ranks N/2-1 and N/2 (math.cairo:113-126, dead odd branch),
qr vs the pass-1 centre, rank mask by (qr asc, idx desc), pass-2 reliability vs the pass-1 centre,
population variance, sample-adjusted skewness / excess kurtosis (math.cairo:320-363).
"""
from __future__ import annotations

from typing import Dict

import torch


def smooth_median(x: torch.Tensor, count: torch.Tensor | int, dim: int = 1) -> torch.Tensor:
    """x sorted along dim after padding excluded rows with +inf; ranks count//2 - 1, count//2."""
    s, _ = torch.sort(x, dim=dim)
    if isinstance(count, int):
        m = count // 2
        return 0.5 * (s.select(dim, m - 1) + s.select(dim, m))
    m = (count // 2).long()
    idx_hi = m.view(-1, 1, 1).expand(-1, 1, x.shape[2])
    hi = torch.gather(s, dim, idx_hi).squeeze(dim)
    lo = torch.gather(s, dim, idx_hi - 1).squeeze(dim)
    return 0.5 * (lo + hi)


def fast_round(values: torch.Tensor, n_failing: int, constrained: bool, max_spread: float = 1.0,
               legacy: bool = False) -> Dict[str, torch.Tensor]:
    """values: [B, N, D] (any float dtype; computed in fp32). Returns a dict of fp32 outputs.

    legacy: obsolete-contract variant (contract_nd.cairo:418,437): reliability without /D, no moments."""
    x = values.float()
    B, N, D0 = x.shape
    D = 1 if legacy else D0
    c1 = smooth_median(x, N)                                  # [B, D]
    qr = ((x - c1[:, None, :]) ** 2).sum(-1)                  # [B, N]
    mean_qr = qr.double().mean(-1)
    if constrained:
        rel1 = 1 - 2 * torch.sqrt(mean_qr / D)
    else:
        rel1 = 1 - torch.clamp(torch.sqrt(mean_qr), max=max_spread) / max_spread
    # rank by (qr asc, idx desc): stable sort of (qr, -idx)
    idx = torch.arange(N, device=x.device).expand(B, N)
    key_order = torch.argsort(-idx, dim=1, stable=True)      # idx desc
    qr_p = torch.gather(qr, 1, key_order)
    order = torch.gather(key_order, 1, torch.argsort(qr_p, dim=1, stable=True))
    rank = torch.empty_like(order)
    rank.scatter_(1, order, torch.arange(N, device=x.device).expand(B, N))
    R = N - n_failing
    reliable = rank < R
    xr = torch.where(reliable[:, :, None], x, torch.full_like(x, float("inf")))
    if constrained:
        consensus = smooth_median(xr, R)
    else:
        consensus = (torch.where(reliable[:, :, None], x, 0).sum(1) / R)
    mean_qr2 = torch.where(reliable, qr, 0).double().sum(-1) / R
    if constrained:
        rel2 = 1 - 2 * torch.sqrt(mean_qr2 / D)
    else:
        rel2 = 1 - torch.clamp(torch.sqrt(mean_qr2), max=max_spread) / max_spread
    xm = torch.where(reliable[:, :, None], x, 0).double()
    mu = xm.sum(1) / R
    y = torch.where(reliable[:, :, None], x.double() - mu[:, None, :], 0)
    m2 = (y ** 2).sum(1) / R
    m3 = (y ** 3).sum(1) / R
    m4 = (y ** 4).sum(1) / R
    n = float(R)
    safe = m2 > 0
    sd = torch.sqrt(torch.where(safe, m2, 1.0))
    z3 = n * m3 / sd ** 3
    z4 = n * m4 / torch.where(safe, m2, 1.0) ** 2
    skew = torch.where(safe, z3 * n / ((n - 1) * (n - 2)), 0.0)
    kurt = torch.where(safe, ((z4 * n * (n + 1)) / (n - 1) - 3 * (n - 1) ** 2) / ((n - 2) * (n - 3)), 0.0)
    if legacy:
        skew, kurt = torch.zeros_like(skew), torch.zeros_like(kurt)
    return dict(c1=c1, qr=qr, reliable=reliable, consensus=consensus.float(), rel=torch.stack([rel1, rel2], -1).float(),
                skew=skew.float(), kurt=kurt.float())
