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


def _cpu_cfg(tmp_path):
    p = tmp_path / "cpu_small.yaml"
    p.write_text("name: cpu_small\nmodel: test N=16 D=64 streaming\nN: 16\nD: 64\nf: 2\nbatch: 8\n"
                 "update_frac: 0.25\ndevice: cpu\nmode: fast\n")
    return str(p)


def _run_dist(args, timeout=600):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py")] + args
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-4000:]
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


def _port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_dp_and_dshard_gloo(tmp_path):
    """The driver's multi-rank contract (torch.distributed.run, max over ranks, rank-0 JSON) on gloo."""
    cfg = _cpu_cfg(tmp_path)
    dp = _run_dist(["--config-file", cfg, "--gpus", "2", "--steps", "4", "--warmup", "1"])
    assert dp["n_gpus"] == 2 and dp["scaling"] == "weak" and dp["config"]["global_batch"] == 16
    assert dp["config"]["ok_fraction"] == 1.0
    ds = _run_dist(["--config-file", cfg, "--gpus", "2", "--steps", "4", "--warmup", "1", "--dshard"])
    assert ds["scaling"] == "strong" and ds["config"]["parallelism"] == "dshard2"
    assert ds["config"]["global_batch"] == 8 and ds["config"]["ok_fraction"] == 1.0


def test_bench_gpus_flag_spawns_ranks_gloo(tmp_path):
    """The driver's plain form `python bench.py --gpus 2` (no launcher) starts two ranks itself."""
    cfg = _cpu_cfg(tmp_path)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config-file", cfg, "--gpus", "2",
                        "--steps", "3", "--warmup", "1"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 16
    assert out["config"]["backend_world"] == 2 and len(out["config"]["rank_ms_per_step"]) == 2


def test_bench_gpus_8_spawns_eight_ranks_gloo(tmp_path):
    """The driver's 8-GPU form, `python bench.py --gpus 8`, rehearsed at world 8 on gloo: eight ranks, one
    JSON line from rank 0, the backend's own world size, per-rank step times and outcomes."""
    cfg = _cpu_cfg(tmp_path)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config-file", cfg, "--gpus", "8",
                        "--steps", "3", "--warmup", "1"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    c = out["config"]
    assert out["n_gpus"] == 8 and c["backend_world"] == 8 and c["parallelism"] == "dp8"
    assert c["global_batch"] == 8 * 8 and len(c["rank_ms_per_step"]) == 8 and len(c["rank_ok_fraction"]) == 8
    lo, hi = c["rank_ms_spread"]
    assert 0 < lo <= hi and abs(out["ms_per_step"] - hi) < 1e-6 * max(1.0, hi)   # the job time is the slowest rank
    assert all(o == 1.0 for o in c["rank_ok_fraction"]) and c["ok_fraction"] == 1.0


def test_bench_gpus_8_dshard_gloo(tmp_path):
    """`bench.py --gpus 8 --dshard` at world 8 on gloo: every rank holds a column slice (D = 64 over 8 ranks)
    of the same 8 instances, one packed all-reduce per round, deferred commits, strong scaling."""
    cfg = _cpu_cfg(tmp_path)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config-file", cfg, "--gpus", "8",
                        "--dshard", "--steps", "3", "--warmup", "1"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    c = out["config"]
    assert out["n_gpus"] == 8 and out["scaling"] == "strong" and c["parallelism"] == "dshard8"
    assert c["backend_world"] == 8 and c["global_batch"] == 8 and len(c["rank_ms_per_step"]) == 8
    assert c["ok_fraction"] == 1.0 and all(o == 1.0 for o in c["rank_ok_fraction"])
    assert c["hip_graph"] is False            # (CPU ranks: no graphs)


def test_bench_gpus_world_mismatch_fails(tmp_path):
    cfg = _cpu_cfg(tmp_path)
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config-file", cfg, "--gpus", "2",
                        "--steps", "2", "--warmup", "0"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_bench_fp32_storage_cpu(tmp_path):
    """bench.py --storage fp32: the fast engine over fp32 storage (CPU twin here), dtype reported."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config-file", _cpu_cfg(tmp_path),
                        "--storage", "fp32", "--steps", "4", "--warmup", "1"], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["dtype"] == "fp32" and out["config"]["storage"] == "fp32"
    assert out["value"] > 0 and out["config"]["ok_fraction"] == 1.0


def test_bench_exact_transactional_stream_cpu(tmp_path):
    """configs/c*_exact_stream.yaml's form: exact mode, every update its own transaction -- rounds/s
    counts one round per update (U per instance per step)."""
    p = tmp_path / "cpu_tx.yaml"
    p.write_text("name: cpu_tx\nmodel: test N=7 D=6 exact transactional stream\nN: 7\nD: 6\nf: 2\nbatch: 64\n"
                 "update_frac: 0.2857142857142857\ndevice: cpu\nmode: exact\ntransactional: true\n")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config-file", str(p), "--steps", "3",
                        "--warmup", "1"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    cfg = out["config"]
    assert cfg["transactional"] and cfg["engine_mode"] == "exact" and cfg["updates_per_instance_per_step"] == 2
    assert abs(out["value"] - cfg["oracle_updates_per_s"]) < 1e-6 * out["value"]   # one round per update
    assert abs(out["value"] * out["ms_per_step"] / 1e3 - 64 * 2) < 1e-6 * 128
    assert 0 < cfg["ok_fraction"] <= 1.0
