"""Which c3-shape exact rounds does the column-parallel wsad kernel hand to the i128 kernel?  Rounds on
randomized state with one row replaced (honest Beta row / uniform row / the stream's row), with
SVOC_EXACT_WSAD_ONLY=1 so a flagged instance keeps the sentinel status -99."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svoc.config import ConsensusConfig  # noqa: E402
from svoc.engine import ConsensusEngine  # noqa: E402

B, N, D, f = 16, 256, 4096, 32
cfg = ConsensusConfig(n_oracles=N, dimension=D, n_failing_oracles=f, constrained=True)
eng = ConsensusEngine(cfg, batch=B, device="cuda", mode="exact")
eng.randomize(seed=1)
g = torch.Generator(device="cuda").manual_seed(5)


def flagged(tag):
    os.environ["SVOC_EXACT_WSAD_ONLY"] = "1"
    eng.status.fill_(-99)
    eng.touched.fill_(1)
    eng.run_round()
    torch.cuda.synchronize()
    st = eng.status.cpu()
    os.environ["SVOC_EXACT_WSAD_ONLY"] = "0"
    print(f"{tag:40s} flagged {(st == -99).sum().item():2d}/{B}  statuses {sorted(set(st.tolist()))}", flush=True)


flagged("randomized state")
save = eng.values.clone()
for o in (0, 5, 100, 255):
    eng.values.copy_(save)
    x = torch.distributions.Beta(20.0, 20.0).sample((B, D)).cuda()
    eng.values[:, o, :] = (x.double() * 1e6).to(torch.int32)
    flagged(f"row {o} <- Beta(20,20)")
    eng.values.copy_(save)
    eng.values[:, o, :] = (torch.rand(B, D, device="cuda", generator=g).double() * 1e6).to(torch.int32)
    flagged(f"row {o} <- U(0,1)")
eng.values.copy_(save)
eng.values[:, 7, :] = eng.values[:, 8, :]
flagged("row 7 <- row 8 (duplicate)")
