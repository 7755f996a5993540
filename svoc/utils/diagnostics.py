"""UI-side outlier preview and pretty printers (client/oracle_scheduler.py:94-153, contract utils).

``rank_array``: rank 0 = most deviant (oracle_scheduler.py:94-104).  ``preview``: per-oracle L2
distance to the component-wise numpy median and the ``[X]`` marks of the reference console
(oracle_scheduler.py:136-153).  ``scatter_components``: the label-pair scatter data the web UI
plotted (predictions_to_eel_values, :106-134).
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch


def rank_array(values: Sequence[float]) -> Tuple[np.ndarray, np.ndarray]:
    s = np.argsort(values)
    rev = np.zeros(len(s), dtype=np.int64)
    for from_idx, to_idx in enumerate(s):
        rev[to_idx] = s.size - from_idx - 1
    return rev / max(1, s.size - 1), rev


def preview(preds: torch.Tensor) -> Dict[str, np.ndarray]:
    p = np.asarray(preds, dtype=np.float64)
    med = np.median(p, axis=0)
    dev = np.linalg.norm(p - med, axis=1)
    norm, ranks = rank_array(dev)
    return dict(mean=p.mean(0), median=med, deviation=dev, ranks=ranks, score=norm)


def show_predictions(preds: torch.Tensor, n_failing: int, labels: Sequence[str]) -> str:
    pv = preview(preds)
    s = "LABELS :\n" + ", ".join(labels) + "\n----------------\n"
    for i, row in enumerate(np.asarray(preds)):
        mark = "[ ]" if pv["ranks"][i] >= n_failing else "[X]"
        s += f"{mark} | oracle {i:2d} : {[float(f'{x:0.2f}') for x in row]} \n"
    return s


def scatter_components(preds: torch.Tensor, labels: Sequence[str]) -> List[dict]:
    p = np.asarray(preds, dtype=np.float64)
    score = preview(preds)["score"]
    comps = []
    for i in range(0, p.shape[1], 2):
        two = i + 1 < p.shape[1]
        comps.append(dict(columnNames=[labels[i], labels[i + 1] if two else "None"],
                          data=[dict(x=float(r[i]), y=float(r[i + 1]) if two else 0.0, score=float(sc))
                                for r, sc in zip(p, score)]))
    return comps


def show_oracle_table(addresses, values, enabled, reliable, fmt=lambda v: f"{v}") -> str:
    """show_nd_felt_oracle_array (contract/src/utils.cairo) equivalent."""
    lines = []
    for a, v, e, r in zip(addresses, values, enabled, reliable):
        lines.append(f"{hex(a):>24} | enabled={bool(e)!s:5} reliable={bool(r)!s:5} | {[fmt(x) for x in v]}")
    return "\n".join(lines)
