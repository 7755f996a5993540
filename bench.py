"""Headline benchmark: consensus updates/sec (N oracles x D dims, batched) at 1/2/4/8 MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c5] [--batch B]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Configs (BASELINE.json):
  c3 (default): 256 oracles x 4096 dims, streaming updates with failing-oracle masking, DP over
      independent instances.  One step on every rank = a batch of fresh predictions from 1/4 of the
      oracles of every local instance (synthetic stream, pre-generated in HBM, cycled) scattered into
      the state + one full two-pass consensus round per instance (fused HIP kernel) + an RCCL
      all-reduce of the step's health metrics (reliability sum, OK count).
  c2: 64 oracles x 1024 dims, 10k instances per GPU, one full consensus round per instance per step.
Weak scaling: per-GPU instances are fixed; ``value`` is the whole-job consensus rounds per second.
Synthetic data (Beta(20,20) honest oracles, U(0,1) failing), random state, bf16 storage / fp32 math.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # f = 0: with 4 oracles any f >= 1 leaves R <= 3 reliable and the contract's kurtosis divides
    # by (n-2)(n-3) = 0 (math.cairo:362) -- every round would revert
    "c1": dict(model="plumbing: 4 oracles x 2 dims, one exact (wsad) round per step on the CPU engine", N=4, D=2,
               f=0, batch=1, update_frac=0.0, device="cpu", mode="exact", dtype="int64-wsad"),
    "c3": dict(model="svoc-consensus N=256 D=4096 streaming (f=32, constrained)", N=256, D=4096, f=32,
               batch=1024, update_frac=0.25, pipeline=4),
    "c2": dict(model="svoc-consensus N=64 D=1024 batched (f=8, constrained)", N=64, D=1024, f=8,
               batch=10000, update_frac=0.0),
    "c4": dict(model="sentiment oracles: BERT-base (12x768, bf16) on 30-comment windows -> 7 oracles x 6 dims",
               N=7, D=6, f=2, batch=64, update_frac=1.0, seq_len=128),
    "c5": dict(model="deployed config 7 oracles x 6 dims, governance + reliability stream (1% instances vote/step)",
               N=7, D=6, f=2, batch=1 << 20, update_frac=1 / 7, gov_frac=0.01),
}
METRIC = "consensus updates/sec (N oracles x D dims, batched)"


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch_ranks(n: int) -> int:
    """Re-run this script as ``n`` ranks under torch.distributed.run (rendezvous on 127.0.0.1)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--config-file", default=None, help="YAML config (configs/*.yaml); overrides --config")
    ap.add_argument("--batch", type=int, default=0, help="instances per GPU (default per config)")
    ap.add_argument("--wave-hint", type=int, default=0)
    ap.add_argument("--graph", type=int, default=1, help="capture the step in a HIP graph")
    ap.add_argument("--pipeline", type=int, default=-1,
                    help="streaming configs: overlap the update scatter of one instance range with the round "
                         "of the previous one over K ranges (ConsensusEngine.step_pipelined); 1 = serial, "
                         "-1 = the config's default")
    ap.add_argument("--mode", default=None, choices=["fast", "exact"],
                    help="override the config's engine mode (exact = bit-exact wsad int64 path)")
    ap.add_argument("--storage", default=None, choices=["bf16", "fp32", "int64", "int32"],
                    help="engine value storage (exact mode: int64 default, int32 for constrained configs)")
    ap.add_argument("--dshard", action="store_true",
                    help="strong scaling: every rank holds a column slice of ALL instances (D-sharding, one "
                         "[B, N] qr all-reduce per round) instead of its own instances (DP, default)")
    ap.add_argument("--backend", default=None, help="torch.distributed backend (default: nccl = RCCL on GPU)")
    ap.add_argument("--log", default=None, help="append the result record to this JSON-lines file")
    ap.add_argument("--kernel-table", type=int, default=0, help="profile N extra steps (torch.profiler) "
                    "after the timed region and add the per-kernel table to the log record")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python bench.py --gpus N` without a launcher: start N ranks (one process per GPU) under
        # torch.distributed.run as a child and exit with its code.  Nothing here has touched the GPU.
        sys.exit(_launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch one rank per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.config_file:
        import yaml
        with open(args.config_file, encoding="utf-8") as f:
            doc = yaml.safe_load(f)
        args.config = doc.pop("name")
        doc.pop("baseline_config", None)
        CONFIGS[args.config] = {**CONFIGS.get(args.config, {}), **doc}
    c = CONFIGS[args.config]
    dev = torch.device("cuda", local) if c.get("device", "cuda") == "cuda" else torch.device("cpu")
    if world > 1:
        if dev.type == "cuda":
            torch.cuda.set_device(local)
            dist.init_process_group(args.backend or "nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend or "gloo")
    dshard = args.dshard   # world 1: the split-kernel path without collectives (its overhead)

    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    from svoc.parallel.dp import DataParallelConsensus

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    B = args.batch or c["batch"]
    D_local, lo = c["D"], 0
    if dshard:
        from svoc.parallel.dshard import run_round_sharded, shard_bounds
        lo, hi = shard_bounds(c["D"], rank, world)
        D_local = hi - lo
    cfg = ConsensusConfig(n_oracles=c["N"], dimension=D_local, n_failing_oracles=c["f"], constrained=True)
    mode = args.mode or c.get("mode", "fast")
    if dshard and args.config in ("c4", "c5"):
        raise SystemExit("--dshard is for the column-sharded configs (c2, c3, fast or exact)")
    eng = ConsensusEngine(cfg, batch=B, device=dev, mode=mode, storage=args.storage)
    eng.wave_hint = args.wave_hint
    dp = DataParallelConsensus(eng, rank=rank, world=world)
    eng.randomize(seed=1000 + (0 if dshard else rank))

    # synthetic update stream resident in HBM: `pool` steps of updates, cycled
    U_per_inst = int(round(c["update_frac"] * c["N"]))
    stream = pipe = gov = None
    extra = {}
    if args.config == "c4":
        from svoc.models import corpus
        from svoc.models.sentiment_oracle import SentimentOraclePipeline
        pipe = SentimentOraclePipeline(eng, seed=0)
        g = torch.Generator(device=dev).manual_seed(rank)
        toks = [corpus.synthetic_token_batch(B * 30, c["seq_len"], 50265, g, dev) for _ in range(2)]
        from svoc.models.encoder import flops_for_lengths
        extra["comments_per_step"] = B * 30
        lens = toks[0][1].sum(1).tolist()
        extra["real_tokens_per_step"] = int(sum(lens))
        extra["padded_tokens_per_step"] = B * 30 * c["seq_len"]
        # the packed path computes real tokens only (as the reference pipeline, one comment at a time)
        extra["encoder_gflop_per_step"] = flops_for_lengths(pipe.encoder.cfg, lens) / 1e9
    elif U_per_inst:
        from svoc.stream import SyntheticUpdateStream
        # D-sharding: every rank streams the same updates (same seed), its own column slice of them
        stream = SyntheticUpdateStream(B, c["N"], D_local, U_per_inst, c["f"], pool=2, device=dev,
                                       seed=(0 if dshard else rank),
                                       dtype=torch.int64 if mode == "exact" else torch.bfloat16)
    if args.config == "c5":
        from svoc.codec import address_to_limbs
        from svoc.governance import Governance
        gov = Governance(B, 3, c["N"], dev, True, 2)
        gov.admins.copy_(torch.tensor([address_to_limbs(1000 + a) for a in range(3)], device=dev).expand(B, 3, 4))
        ora = torch.tensor([address_to_limbs(5000 + o) for o in range(c["N"])], device=dev)
        gov.oracle_addr.copy_(ora.expand(B, c["N"], 4))
        from svoc.stream import governance_stream
        gov_batches = governance_stream(B, c["N"], [1000, 1001, 1002], dev, seed=rank, frac=c["gov_frac"])
        K = gov_batches[0][0].numel()
        extra["governance_actions_per_step"] = K
        extra["state_bytes_per_instance"] = eng.bytes_per_instance(c["N"], c["D"], "fast") + 3 * 4 * 8 + 3 * 8 + 3 * (1 + 4 + 32) + c["N"] * 32
        extra["instances_per_288GB"] = int(288e9 // extra["state_bytes_per_instance"])

    pipeline = args.pipeline if args.pipeline >= 0 else c.get("pipeline", 1)
    if dshard or mode != "fast" or dev.type != "cuda":
        pipeline = 1
    extra["pipeline_chunks"] = pipeline

    def run_round():
        if dshard:
            run_round_sharded(eng, c["D"], world=world)   # includes the qr all-reduce
        else:
            eng.run_round(only_touched=True)

    def step(i):  # device-only work (capturable)
        if pipe is not None:
            pipe.fetch(*toks[i % 2])
        elif stream is not None:
            inst, orc, vals = stream.batch(i)
            if pipeline > 1:   # the stream has distinct (instance, oracle), grouped by instance
                eng.step_pipelined(inst, orc, vals, U_per_inst, chunks=pipeline)
            else:
                eng.apply_updates(inst, orc, vals, unique=True)
                run_round()
        else:
            eng.touched.fill_(1)
            run_round()
        if gov is not None:
            gov.submit_tensors(*gov_batches[i % len(gov_batches)])
        dp.accumulate()

    for i in range(args.warmup):
        step(i)
        dp.reduce()
    sync()

    graph = None
    if args.graph and dev.type == "cuda" and not (dshard and world > 1):   # (no collectives in a graph)
        # the stream cycles with period `pool`: capture one period and replay it
        import math
        period = 1
        for k in (stream.pool if stream is not None else 1, len(gov_batches) if gov is not None else 1,
                  2 if pipe is not None else 1):
            period = period * k // math.gcd(period, k)
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for i in range(period):
                step(i)
        torch.cuda.current_stream(dev).wait_stream(s)
        sync()
        try:
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                for i in range(period):
                    step(i)
            graph_period = period
        except Exception as e:  # graph capture is an optimisation; eager stays correct
            if rank == 0:
                print(f"[bench] graph capture failed ({e}); running eager", file=sys.stderr)
            graph = None

    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    if graph is not None:
        reps, rem = divmod(args.steps, graph_period)
        for _ in range(reps):
            graph.replay()
            dp.reduce()            # one RCCL all-reduce of the step metrics per replay
        for i in range(rem):       # exactly K steps: the tail of a period runs eagerly
            step(i)
            dp.reduce()
        steps_done = args.steps
    else:
        for i in range(args.steps):
            step(i)
            dp.reduce()
        steps_done = args.steps
    sync()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    el = float(elapsed.item())
    ms_per_step = 1e3 * el / steps_done
    rounds = B * (1 if dshard else world) * steps_done   # D-sharding: all ranks share the same B instances
    value = rounds / el
    ok = dp.global_ok_fraction()
    if rank == 0:
        out = {
            "metric": METRIC, "value": value, "unit": "consensus rounds/s", "n_gpus": world,
            "steps": steps_done, "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
            "scaling": "strong" if dshard else "weak", "vs_baseline": None,
            "dtype": f"{eng.storage}-wsad" if mode == "exact" else ("fp32-storage" if eng.storage == "fp32" else c.get("dtype", "bf16")), "data": "synthetic",
            "config": {"model": c["model"], "global_batch": B * (1 if dshard else world), "seq_len": c["D"],
                       "parallelism": f"dshard{world}" if dshard else f"dp{world}", "engine_mode": mode, "n_oracles": c["N"], "dimension": c["D"],
                       "n_failing": c["f"], "updates_per_instance_per_step": U_per_inst,
                       "oracle_updates_per_s": (U_per_inst * rounds / el) if U_per_inst else 0.0,
                       "hip_graph": graph is not None, "ok_fraction": ok, **extra},
        }
        if args.config in ("c2", "c3"):
            from svoc.utils.metrics import algorithmic_bytes_per_round
            out["config"]["hbm_gbps_algorithmic"] = algorithmic_bytes_per_round(c["N"], c["D"], eng.values.element_size()) * rounds / el / 1e9
        print(json.dumps(out))
        if args.log:
            from svoc.utils.metrics import JsonlLogger, engine_health, kernel_table
            rec = dict(out)
            rec["health"] = engine_health(eng)
            if args.kernel_table:
                rec["kernels"] = kernel_table(lambda: step(0), steps=args.kernel_table)
            with JsonlLogger(args.log, rank) as lg:
                lg.log("bench", **rec)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
