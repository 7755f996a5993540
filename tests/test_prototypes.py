"""Notebook prototypes (contract/drafts/*.ipynb) batched on the device: svoc/models/prototypes.py.

numpy loops of the notebook functions serve as the reference (the notebooks themselves are not run:
they need matplotlib/seaborn and unseeded RNG)."""
import math

import numpy as np
import torch

from svoc.models import prototypes as P


def test_modes_and_normalisation():
    assert P.beta_mode(20, 20) == 0.5
    assert abs(P.kumaraswamy_mode(2, 3) - (1 / 5) ** 0.5) < 1e-12
    y = torch.linspace(0.05, 0.95, 19, dtype=torch.float64)
    torch.testing.assert_close(P.normalize(P.denormalize(y)), y)


def test_kumaraswamy_sampler_moments():
    g = torch.Generator().manual_seed(0)
    x = P.kumaraswamy_sample((400_000,), 2.0, 3.0, g)
    # E[X] = b * B(1 + 1/a, b)
    mean = 3.0 * math.gamma(1.5) * math.gamma(3.0) / math.gamma(4.5)
    assert abs(float(x.mean()) - mean) < 3e-3 and float(x.min()) >= 0 and float(x.max()) <= 1


def test_expected_reliability_matches_numpy():
    g = torch.Generator().manual_seed(1)
    x = torch.rand(5, 9, generator=g, dtype=torch.float64)
    ref = [1 - 2 * np.mean(np.abs(r - np.median(r))) for r in x.numpy()]
    torch.testing.assert_close(P.expected_reliability(x), torch.tensor(ref, dtype=torch.float64))


def _np_remove_worst(vals, n_failing):
    """gaussian_algorithm_demo.ipynb cell 11 (argmin quirk included)."""
    res = [(v, True) for v in vals]
    def scores(only_active):
        act = [v for v, a in res if a]
        e = sum(act) / len(act)
        return [np.linalg.norm(v - e) ** 2 if (a or not only_active) else None for v, a in res]
    for _ in range(n_failing):
        sc = scores(True)
        best = min((s, i) for i, s in enumerate(sc) if s is not None)[1]
        res[best] = (res[best][0], False)
    return [a for _, a in res]


def test_remove_worst_oracles_matches_notebook():
    g = torch.Generator().manual_seed(2)
    x, _ = P.generate_normalized_gaussian_oracles(16, 12, 3, 0.9, 5.0, g)
    act, _ = P.remove_worst_oracles(x, 3)
    for b in range(16):
        assert act[b].tolist() == _np_remove_worst(list(x[b].numpy()), 3)
    act_max, _ = P.remove_worst_oracles(x, 3, worst="max")
    assert (act_max.sum(1) == 9).all()


def test_generators_shapes_and_failing_counts():
    g = torch.Generator().manual_seed(3)
    x, ok = P.generate_2d_gaussian_oracles(8, 7, 2, [20.0, 10.0], [3.0, 4.0], g)
    assert x.shape == (8, 7, 2) and (ok.sum(1) == 5).all()
    xb, okb = P.generate_2d_beta_oracles(8, 7, 2, (10, 20), (10, 20), g)
    assert xb.shape == (8, 7, 2) and (okb.sum(1) == 5).all() and float(xb.min()) >= 0 and float(xb.max()) <= 1
