"""Config 5 as BASELINE.json states it: admin replacement voting + Beta reliability over a 1M-step
stream, with 288 GB HBM state sizing.  Two runs (one MI355X):

  stream  B instances (default 1M) of the deployed 7 x 6 config (contract/README.md:43-61), K steps
          (default 100k).  One step = a fresh prediction for 1/7 of the oracles of every instance
          (update_prediction, contract.cairo:588-603), one consensus round per instance, and governance
          on 1% of the instances alternating a proposition by admin 0 and a supporting vote by admin 1
          (contract.cairo:661-738 -> check_for_replacement :547-580, majority 2 -> replacement).  A HIP
          graph holds one stream period.  A .svoc checkpoint is written every C steps; the one at
          K/2 is reloaded into a fresh service, replayed to K, and the two final states must be equal
          bit for bit (restart equivalence).
  hbm     as many instances as fill >= --target-gb of resident state (engine + governance), S steps
          of the same mix; reports torch.cuda.max_memory_allocated.

    python tools/c5_stream.py stream --steps 100000 --instances 1048576 --ckpt-every 25000 --out rec.json
    python tools/c5_stream.py hbm --target-gb 150 --steps 20 --out rec.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from svoc.api import ConsensusService  # noqa: E402
from svoc.codec import address_to_limbs  # noqa: E402
from svoc.config import ConsensusConfig  # noqa: E402
from svoc.models.oracle_gen import beta_failing_oracles  # noqa: E402
from svoc.stream import SyntheticUpdateStream, governance_stream  # noqa: E402

N, D, F, A = 7, 6, 2, 3


def build(B: int, dev, seed: int = 0) -> ConsensusService:
    """A service of B instances: admins / oracle addresses as device tensors, values from the
    Beta / uniform generator in chunks (bounded temporaries), every oracle active."""
    cfg = ConsensusConfig(n_oracles=N, dimension=D, n_failing_oracles=F, n_admins=A, constrained=True,
                          enable_oracle_replacement=True, required_majority=2)
    svc = ConsensusService.__new__(ConsensusService)
    from svoc.engine import ConsensusEngine
    from svoc.governance import Governance
    svc.cfg, svc.B = cfg, B
    svc.engine = ConsensusEngine(cfg, B, device=dev, mode="fast")
    svc.gov = Governance(B, A, N, dev, True, 2)
    svc.gov.admins.copy_(torch.tensor([address_to_limbs(1000 + a) for a in range(A)], device=dev).expand(B, A, 4))
    svc.gov.oracle_addr.copy_(torch.tensor([address_to_limbs(5000 + o) for o in range(N)], device=dev).expand(B, N, 4))
    e = svc.engine
    g = torch.Generator(device=dev).manual_seed(seed)
    step = 1 << 22
    last = time.perf_counter()
    for s in range(0, B, step):
        t = min(B, s + step)
        e.values[s:t, :, :D] = beta_failing_oracles(t - s, N, D, F, 20.0, g, dev).to(e.vdtype)
        if time.perf_counter() - last > 20:
            torch.cuda.synchronize()
            print(f"[c5] initialised {t}/{B} instances", flush=True)
            last = time.perf_counter()
    e.enabled.fill_(1)
    e.n_active.fill_(N)
    e.touched.fill_(1)
    return svc


class Runner:
    """Steps of the c5 mix; step i uses update batch i % pool and governance batch i % 8 (4
    proposition / supporting-vote pairs on 1% of the instances each: every pair replaces an oracle)."""

    def __init__(self, svc: ConsensusService, pool: int, seed: int = 0):
        self.svc = svc
        e = svc.engine
        self.stream = SyntheticUpdateStream(e.B, N, D, 1, F, pool=pool, device=e.device, seed=seed)
        self.gov = governance_stream(e.B, N, [1000 + a for a in range(A)], e.device, seed)
        import math
        self.period = pool * len(self.gov) // math.gcd(pool, len(self.gov))
        self.graph = None

    def step(self, i: int) -> None:
        e = self.svc.engine
        inst, orc, vals = self.stream.batch(i)
        e.apply_updates(inst, orc, vals, unique=True)
        e.run_round()
        self.svc.gov.submit_tensors(*self.gov[i % len(self.gov)])

    def capture(self) -> None:
        dev = self.svc.engine.device
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for i in range(self.period):
                self.step(i)
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            for i in range(self.period):
                self.step(i)

    def run(self, i0: int, i1: int) -> None:
        """Steps [i0, i1): eager up to a period boundary, graph replays, eager tail (a progress line every
        30 s: long eager replays must not look hung)."""
        i = i0
        last = time.perf_counter()

        def tick():
            nonlocal last
            if time.perf_counter() - last > 30:
                print(f"[c5] step {i}/{i1}", flush=True)
                last = time.perf_counter()
        while i < i1 and i % self.period:
            self.step(i)
            i += 1
        while self.graph is not None and i + self.period <= i1:
            self.graph.replay()
            i += self.period
            if i % (1024 * self.period) == 0:
                tick()
        while i < i1:
            self.step(i)
            i += 1
            if i % 1024 == 0:
                tick()


def state_digest(svc: ConsensusService) -> dict:
    e, g = svc.engine, svc.gov
    out = {}
    for name, t in (("values", e.values), ("consensus", e.consensus), ("skew", e.skew), ("kurt", e.kurt),
                    ("rel", e.rel), ("qr", e.qr), ("reliable", e.reliable), ("status", e.status),
                    ("consensus_active", e.consensus_active), ("oracle_addr", g.oracle_addr), ("votes", g.votes),
                    ("prop_tag", g.prop_tag), ("prop_idx", g.prop_idx), ("prop_addr", g.prop_addr)):
        b = t.contiguous().view(torch.uint8) if t.dtype != torch.bool else t.to(torch.uint8)
        # order-sensitive checksum on the device: sum of (byte * position mix) in int64
        idx = torch.arange(b.numel(), device=b.device, dtype=torch.int64)
        out[name] = int(((b.reshape(-1).to(torch.int64) + 1) * ((idx * 2654435761) % 1000003 + 1)).sum().item())
    return out


def cmd_stream(a) -> dict:
    from svoc import state
    dev = torch.device("cuda")
    svc = build(a.instances, dev)
    run = Runner(svc, a.pool)
    run.step(0)
    torch.cuda.synchronize()
    run.capture()
    tmp = tempfile.mkdtemp(prefix="svoc_c5_")
    half = a.steps // 2
    ckpts, t_ck = [], 0.0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    i = 0
    marks = sorted(set([half] + list(range(a.ckpt_every, a.steps, a.ckpt_every))))
    last_print = time.perf_counter()
    for m in marks + [a.steps]:
        run.run(i, m)
        i = m
        if m < a.steps:
            torch.cuda.synchronize()
            c0 = time.perf_counter()
            path = os.path.join(tmp, f"step{m}.svoc" if m == half else "latest.svoc")
            state.save(svc, path)
            t_ck += time.perf_counter() - c0
            ckpts.append(dict(step=m, seconds=time.perf_counter() - c0, bytes=os.path.getsize(path)))
        if time.perf_counter() - last_print > 30:
            print(f"[c5] step {i}/{a.steps}", flush=True)
            last_print = time.perf_counter()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    final = state_digest(svc)
    e = svc.engine
    metrics = e.metrics().tolist()
    peak = torch.cuda.max_memory_allocated()
    orig = torch.tensor([address_to_limbs(5000 + o) for o in range(N)], device=dev)
    replacements_seen = int((svc.gov.oracle_addr != orig[None]).any(2).any(1).sum())
    del run, svc, e
    torch.cuda.empty_cache()
    # restart equivalence: reload the mid-stream checkpoint and replay its second half
    svc2 = state.load(os.path.join(tmp, f"step{half}.svoc"), device="cuda")
    run2 = Runner(svc2, a.pool)   # eager replay: capturing would run warm-up steps on the restored state
    r0 = time.perf_counter()
    run2.run(half, a.steps)
    torch.cuda.synchronize()
    replay = time.perf_counter() - r0
    final2 = state_digest(svc2)
    equal = final == final2
    steps_timed = a.steps
    compute = wall - t_ck
    return dict(kind="c5_stream", instances=a.instances, steps=a.steps, pool=a.pool,
                wall_seconds=wall, checkpoint_seconds=t_ck, compute_seconds=compute,
                ms_per_step=1e3 * compute / steps_timed, rounds_per_s=a.instances * steps_timed / compute,
                oracle_updates_per_s=a.instances * steps_timed / compute,
                governance_actions_per_s=max(1, int(a.instances * 0.01)) * steps_timed / compute,
                checkpoints=ckpts, restart_from=half, replay_seconds=replay, restart_equivalent=equal,
                digest=final, committed_rounds=metrics[1], processed_rounds=metrics[2], reverted_rounds=metrics[3],
                instances_with_replaced_oracle=replacements_seen, hbm_peak_bytes=peak,
                data="synthetic (Beta(20,20) honest, U(0,1) failing), random-init state", dtype="bf16")


def cmd_hbm(a) -> dict:
    dev = torch.device("cuda")
    free0, total = torch.cuda.mem_get_info()
    # bytes of resident state per instance (engine + governance) from a small probe
    probe = build(1 << 12, dev)
    per = sum(t.numel() * t.element_size() for t in (
        probe.engine.values, probe.engine.enabled, probe.engine.n_active, probe.engine.reliable,
        probe.engine.consensus_active, probe.engine.c1, probe.engine.consensus, probe.engine.skew, probe.engine.kurt,
        probe.engine.rel, probe.engine.qr, probe.engine.status, probe.engine.touched, probe.engine._winner,
        probe.engine._active, probe.gov.admins, probe.gov.oracle_addr, probe.gov.votes, probe.gov.prop_tag,
        probe.gov.prop_idx, probe.gov.prop_addr)) / (1 << 12)
    del probe
    torch.cuda.empty_cache()
    B = a.instances or int(a.target_gb * 1e9 / per) + 1
    t0 = time.perf_counter()
    svc = build(B, dev)
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t0
    state_bytes = int(per * B)
    run = Runner(svc, 2)
    torch.cuda.synchronize()
    for i in range(2):
        run.step(i)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    run.run(2, 2 + a.steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t1
    m = svc.engine.metrics().tolist()
    return dict(kind="c5_hbm", instances=B, state_bytes_per_instance=per, resident_state_bytes=state_bytes,
                resident_state_gb=state_bytes / 1e9, hbm_total_bytes=total, hbm_peak_bytes=torch.cuda.max_memory_allocated(),
                build_seconds=build_s, steps=a.steps, ms_per_step=1e3 * el / a.steps, rounds_per_s=B * a.steps / el,
                governance_actions_per_s=max(1, int(B * 0.01)) * a.steps / el,
                committed_rounds=m[1], processed_rounds=m[2], reverted_rounds=m[3], dtype="bf16",
                data="synthetic (Beta(20,20) honest, U(0,1) failing), random-init state")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run", choices=["stream", "hbm"])
    ap.add_argument("--instances", type=int, default=0)
    ap.add_argument("--steps", type=int, default=100_000)
    ap.add_argument("--pool", type=int, default=8)
    ap.add_argument("--ckpt-every", type=int, default=25_000)
    ap.add_argument("--target-gb", type=float, default=150.0)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if a.run == "stream":
        a.instances = a.instances or (1 << 20)
        rec = cmd_stream(a)
    else:
        rec = cmd_hbm(a)
    print(json.dumps(rec))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
