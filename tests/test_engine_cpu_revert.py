"""A round that reverts (fast-mode ZERO_VARIANCE, exact-mode DIV_BY_ZERO) commits nothing: the outputs,
consensus_active and the committed-round counter stay as they were (contract.cairo:588-603)."""
import pytest
import torch

from svoc import ops as svops

pytestmark = pytest.mark.skipif(not svops.available(), reason="svoc/_C.so not built")


@pytest.mark.parametrize("mode", ["fast", "exact"])
def test_first_round_revert_leaves_consensus_inactive(mode):
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    cfg = ConsensusConfig(n_oracles=7, dimension=6, n_failing_oracles=2, constrained=True)
    e = ConsensusEngine(cfg, batch=3, device="cpu", mode=mode)
    e.randomize(seed=1)
    scale = 1.0 if mode == "fast" else 1_000_000
    e.values[1, :, :6] = torch.tensor(0.5 * scale).to(e.values.dtype)   # instance 1: every column constant
    e.enabled.fill_(1); e.n_active.fill_(7); e.touched.fill_(1)
    e.run_round()
    st = e.status.tolist()
    assert st[0] == 0 and st[2] == 0 and st[1] != 0
    assert e.consensus_active.tolist() == [True, False, True]
    m = e.metrics().tolist()
    assert m[1] == 2 and m[3] == 1          # committed, reverted
