"""Time the fp32 window round kernel alone (c3 shape, one 512-instance range) -- for the diagnostic
builds of consensus_fast_winf.hip (SVOC_WINF_PROBE): python tools/winf_probe.py [B] [reps]."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svoc.config import ConsensusConfig  # noqa: E402
from svoc.engine import ConsensusEngine  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
cfg = ConsensusConfig(n_oracles=256, dimension=4096, n_failing_oracles=32, constrained=True)
e = ConsensusEngine(cfg, batch=B, device="cuda", mode="fast", storage="fp32")
e.randomize(seed=3)
w = e.work()
args = lambda: (e.values, None, e.D, 32, True, 1.0, e.c1, e.consensus, e.skew, e.kurt, e.rel, e.qr, e.reliable,
                e.status, 0, 0, 0, False, w)
for _ in range(3):
    e._ops.fast_round(*args())
torch.cuda.synchronize()
t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts = []
for _ in range(reps):
    t0.record()
    e._ops.fast_round(*args())
    t1.record()
    t1.synchronize()
    ts.append(t0.elapsed_time(t1))
st = torch.bincount(e.status.long() + 0).tolist()
print(f"probe={os.environ.get('PROBE_TAG', '?')} B={B} min {min(ts) * 1e3:.0f} us  median {sorted(ts)[len(ts) // 2] * 1e3:.0f} us  statuses {st}", flush=True)
if os.environ.get("PROBE_TAG") == "3":   # phase end times (100 MHz ticks) per workgroup in skew[:, 1..5]
    st = e.skew[:, 1:6].double().cpu() * 10.0 / 1e3   # -> us
    names = ["phase A", "+qr/rank/rel", "+pre-check", "+pass 2", "+commit"]
    med = st.median(0).values.tolist()
    print("  median end times (us): " + ", ".join(f"{n} {v:.0f}" for n, v in zip(names, med)))
    print("  max end times (us):    " + ", ".join(f"{n} {v:.0f}" for n, v in zip(names, st.max(0).values.tolist())))
