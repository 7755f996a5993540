"""Observability utilities (svoc/utils/metrics.py) and the bench record contract on the CPU config."""
import json
import os
import subprocess
import sys

import torch

from svoc.config import ConsensusConfig
from svoc.engine import ConsensusEngine
from svoc.utils import metrics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_jsonl_roundtrip(tmp_path):
    p = tmp_path / "m" / "log.jsonl"
    with metrics.JsonlLogger(str(p), rank=3) as lg:
        lg.log("a", x=1, t=torch.tensor([1.5, 2.0]))
        lg.log("b", y="z")
    recs = metrics.read_jsonl(str(p))
    assert [r["kind"] for r in recs] == ["a", "b"] and recs[0]["rank"] == 3 and recs[0]["t"] == [1.5, 2.0]


def test_step_timer_cpu():
    t = metrics.StepTimer("cpu")
    with t:
        sum(range(20000))
    assert t.ms() > 0


def test_engine_health_exact():
    e = ConsensusEngine(ConsensusConfig(n_oracles=7, dimension=3, n_failing_oracles=2), 4, device="cpu", mode="exact")
    e.randomize(seed=1)
    e.run_round()
    h = metrics.engine_health(e)
    assert h["instances"] == 4 and h["consensus_active"] == int(e.consensus_active.sum())
    assert 0.0 <= h["rel2_mean"] <= 1.0


def test_bench_c1_record(tmp_path):
    log = tmp_path / "bench.jsonl"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "c1", "--steps", "20",
                        "--warmup", "2", "--log", str(log)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in out
    assert out["steps"] == 20 and out["value"] > 0 and out["config"]["ok_fraction"] == 1.0
    rec = metrics.read_jsonl(str(log))[-1]
    assert rec["kind"] == "bench" and rec["health"]["consensus_active"] == 1
