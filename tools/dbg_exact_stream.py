"""Timing probe of the exact transactional stream at the c3 shape (256 x 4096, int32 wsad): one step of
64 update waves on a small batch, with per-phase timings (eager, no graph)."""
import sys
import time

import torch

import os  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svoc.config import ConsensusConfig  # noqa: E402
from svoc.engine import ConsensusEngine  # noqa: E402
from svoc.stream import SyntheticUpdateStream  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
N, D, f, U = 256, 4096, 32, 64
cfg = ConsensusConfig(n_oracles=N, dimension=D, n_failing_oracles=f, constrained=True)
eng = ConsensusEngine(cfg, batch=B, device="cuda", mode="exact")
eng.randomize(seed=1)
t = time.perf_counter(); eng.run_round(); torch.cuda.synchronize()
print(f"one exact round over {B} instances: {1e3 * (time.perf_counter() - t):.1f} ms", flush=True)
t = time.perf_counter(); eng.run_round(); torch.cuda.synchronize()
print(f"again: {1e3 * (time.perf_counter() - t):.1f} ms; status {eng.status[:4].tolist()}", flush=True)
s = SyntheticUpdateStream(B, N, D, U, f, pool=2, device="cuda", seed=0, dtype=torch.int64)
inst, orc, vals = s.batch(0)
for K in tuple(int(k) for k in (sys.argv[2] if len(sys.argv) > 2 else '1,4,16,64').split(',')):
    sub = lambda x: x.view(B, U, *x.shape[1:])[:, :K].reshape(B * K, *x.shape[1:])
    t = time.perf_counter()
    st = eng._exact_transactions(sub(inst), sub(orc), sub(vals), updates_per_instance=K)
    torch.cuda.synchronize()
    print(f"{K} waves: {1e3 * (time.perf_counter() - t):.1f} ms; status counts {torch.bincount(st.long()).tolist()}", flush=True)
