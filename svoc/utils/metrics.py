"""Structured observability: JSON-lines records, device-event step timers, kernel tables.

The reference has no structured logging -- its metrics are the on-chain outputs (rel1, rel2,
skewness, kurtosis, consensus_active; contract.cairo:605-659) shown as UI bars (survey §5.5).  Here:

* :class:`JsonlLogger` -- one JSON object per line (rank, wall time, fields), append-only, so bench
  and service runs leave machine-readable records (updates/s, GB/s, per-kernel µs, ok fraction).
* :class:`StepTimer` -- HIP-event timing of device work (no host sync inside the timed region);
  falls back to ``time.perf_counter`` on CPU.
* :func:`kernel_table` -- per-kernel device time of a callable via ``torch.profiler`` (roctracer on
  ROCm), the in-process complement of ``rocprofv3 --kernel-trace --stats``.
* :func:`engine_health` -- the contract's domain metrics aggregated over a batch of instances.
"""
from __future__ import annotations

import json
import os
import time
from typing import Any, Callable, Dict, List, Optional

import torch


class JsonlLogger:
    def __init__(self, path: Optional[str], rank: int = 0, flush: bool = True):
        self.path = path
        self.rank = rank
        self.flush = flush
        self._f = None
        if path:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            self._f = open(path, "a", encoding="utf-8")

    def log(self, kind: str, **fields: Any) -> Dict[str, Any]:
        rec = {"wall_time": time.time(), "rank": self.rank, "kind": kind, **fields}
        if self._f is not None:
            self._f.write(json.dumps(rec, default=_jsonable) + "\n")
            if self.flush:
                self._f.flush()
        return rec

    def close(self) -> None:
        if self._f is not None:
            self._f.close()
            self._f = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def _jsonable(x):
    if isinstance(x, torch.Tensor):
        return x.tolist()
    if hasattr(x, "item"):
        return x.item()
    return str(x)


def read_jsonl(path: str) -> List[Dict[str, Any]]:
    with open(path, encoding="utf-8") as f:
        return [json.loads(line) for line in f if line.strip()]


class StepTimer:
    """Accumulates device time of bracketed regions: ``with timer: work()`` (events are only
    synchronised when :meth:`ms` is read)."""

    def __init__(self, device=None):
        self.device = torch.device(device) if device is not None else None
        self.cuda = self.device is not None and self.device.type == "cuda"
        self._pairs: List = []
        self._cpu_ms = 0.0

    def __enter__(self):
        if self.cuda:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            self._pairs.append((s, e))
        else:
            self._t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if self.cuda:
            self._pairs[-1][1].record()
        else:
            self._cpu_ms += 1e3 * (time.perf_counter() - self._t0)

    @property
    def count(self) -> int:
        return len(self._pairs) if self.cuda else int(self._cpu_ms > 0)

    def ms(self) -> float:
        if not self.cuda:
            return self._cpu_ms
        torch.cuda.synchronize(self.device)
        return sum(s.elapsed_time(e) for s, e in self._pairs)


def kernel_table(fn: Callable[[], None], steps: int = 3, top: int = 12) -> List[Dict[str, Any]]:
    """Per-kernel device time of ``fn`` (called ``steps`` times) from torch.profiler."""
    from torch.profiler import ProfilerActivity, profile
    acts = [ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(ProfilerActivity.CUDA)
    with profile(activities=acts) as prof:
        for _ in range(steps):
            fn()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    rows = []
    for ev in prof.key_averages():
        dev_us = getattr(ev, "device_time_total", None)
        if dev_us is None:
            dev_us = getattr(ev, "cuda_time_total", 0.0)
        if dev_us and dev_us > 0:
            rows.append(dict(name=ev.key, calls=ev.count, device_us_total=float(dev_us),
                             device_us_per_call=float(dev_us) / max(ev.count, 1)))
    rows.sort(key=lambda r: -r["device_us_total"])
    return rows[:top]


def engine_health(engine) -> Dict[str, float]:
    """Domain metrics over a batch (the reference's on-chain outputs, aggregated)."""
    from ..status import Status
    st = engine.status
    ok = (st == Status.OK) | (st == Status.ZERO_VARIANCE) if engine.mode == "fast" else st == Status.OK
    active = engine.consensus_active.bool()
    rel = engine.rel.double()
    if engine.mode == "exact":
        rel = rel / 1e6
    n_act = int(active.sum())
    return dict(
        instances=int(engine.B), consensus_active=n_act,
        ok_fraction=float(ok.double().mean()) if st.numel() else 0.0,
        rel1_mean=float(rel[active, 0].mean()) if n_act else 0.0,
        rel2_mean=float(rel[active, 1].mean()) if n_act else 0.0,
        rounds=int(getattr(engine, "rounds", 0)))


def algorithmic_bytes_per_round(n: int, d: int, storage_bytes: int = 2, updates: int = 0) -> int:
    """Lower bound of the HBM bytes one fast round must move (a data-flow floor, not a measurement):
    the [N, D] values read ONCE (the one-network window kernels need no second read), the round's
    outputs (consensus, skewness, kurtosis: 3 x D fp32; qr, reliable: N x 5 B; two reliabilities and a
    status), plus, for streaming configs, the ``updates`` fresh rows read and written into the state."""
    return n * d * storage_bytes + 3 * d * 4 + 5 * n + 12 + 2 * updates * d * storage_bytes
