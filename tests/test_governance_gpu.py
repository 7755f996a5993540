"""Batched governance kernel (csrc/kernels/governance.hip) vs the in-order CPU implementation."""
import random

import pytest
import torch

from svoc.governance import Governance

pytestmark = pytest.mark.gpu


def _run(device, actions, B, A, N):
    g = Governance(B, A, N, device, True, 2)
    admins = [[10_000 * (b + 1) + a for a in range(A)] for b in range(B)]
    oracles = [[20_000 * (b + 1) + o for o in range(N)] for b in range(B)]
    g.set_addresses(admins, oracles)
    st, ap = g.submit(actions)
    return ([t.cpu() for t in (g.oracle_addr, g.votes, g.prop_tag, g.prop_idx, g.prop_addr)],
            st.cpu(), ap.cpu())


def test_governance_gpu_matches_cpu():
    rng = random.Random(0)
    B, A, N = 64, 5, 9
    actions = []
    for _ in range(3000):
        b = rng.randrange(B)
        caller = 10_000 * (b + 1) + rng.randrange(A + 1)       # sometimes not an admin
        if rng.random() < 0.35:
            prop = None if rng.random() < 0.15 else (rng.randrange(-1, N + 1), 20_000 * (b + 1) + rng.randrange(N + 6))
            actions.append(("propose", b, caller, prop))
        else:
            actions.append(("vote", b, caller, rng.randrange(A + 1), rng.random() < 0.85))
    cpu = _run("cpu", actions, B, A, N)
    gpu = _run("cuda", actions, B, A, N)
    for x, y in zip(cpu[0], gpu[0]):
        assert torch.equal(x, y)
    assert torch.equal(cpu[1], gpu[1]) and torch.equal(cpu[2], gpu[2])
    assert int(cpu[2].sum()) > 0          # some replacements happened
