"""Headline benchmark: consensus updates/sec (N oracles x D dims, batched) at 1/2/4/8 MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c5|c4|c1] [--batch B]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Configs (BASELINE.json):
  c3 (default): 256 oracles x 4096 dims, streaming updates with failing-oracle masking, DP over
      independent instances.  One step on every rank = a batch of fresh predictions from 1/4 of the
      oracles of every local instance (synthetic stream, pre-generated in HBM, cycled) scattered into
      the state + one full two-pass consensus round per instance (fused HIP kernel).  The step's
      health metrics (reliability sum, OK count) are folded on the device every step and all-reduced
      over RCCL once per graph replay (``graph_steps`` steps, reported on the line).  Storage: fp32 -- the
      reference computes on the 1e-6 wsad grid (contract/src/signed_decimal.cairo:82-83) and fp32 holds
      every grid value of [0, 1] exactly; the bf16-storage step is measured too and reported as the
      extra field ``config.alt_storage``.
  c2: 64 oracles x 1024 dims, 10k instances per GPU (bf16, as BASELINE.json names it; fp32 storage
      reported as ``config.alt_storage``), one full consensus round per instance per step.
Weak scaling: per-GPU instances are fixed; ``value`` is the whole-job consensus rounds per second.
Synthetic data (Beta(20,20) honest oracles, U(0,1) failing), random state.
"""
from __future__ import annotations

import argparse
import json
import math
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
               batch=1024, update_frac=0.25, pipeline=2, storage="fp32", alt_storage="bf16"),
    "c2": dict(model="svoc-consensus N=64 D=1024 batched (f=8, constrained)", N=64, D=1024, f=8,
               batch=10000, update_frac=0.0, storage="bf16", alt_storage="fp32"),
    "c4": dict(model="sentiment oracles: RoBERTa-base (BERT-base sized 12x768, erf GELU, bf16) on 30-comment windows -> 7 oracles x 6 dims",
               N=7, D=6, f=2, batch=64, update_frac=1.0, seq_len=128, alt_precision="fp32"),
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


def _collectives_capturable(dev) -> bool:
    """Whether an all-reduce of this process group can be captured in a HIP graph (collective: every rank
    runs it; the verdict is agreed by a MIN all-reduce so all ranks take the same path)."""
    ok = True
    buf = torch.ones(16, device=dev)
    try:
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            dist.all_reduce(buf)                  # warm the communicator on the capture stream
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            dist.all_reduce(buf)
        g.replay()
        torch.cuda.synchronize(dev)
        del g
    except Exception as e:  # capture is an optimisation; eager stays correct
        print(f"[bench] collective capture unavailable ({e}); D-shard steps run eagerly", file=sys.stderr)
        ok = False
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return bool(flag.item())


def _dtype_name(mode: str, storage: str, c: dict) -> str:
    if mode == "exact":
        return f"{storage}-wsad"
    return {"fp32": "fp32", "bf16": "bf16"}.get(storage, c.get("dtype", "bf16"))


_MARK_SEQ = 0   # timed regions bracketed by marker kernels so far (--markers)


def measure(args, c, storage, dev, rank, world, dshard, enc_dtype=None, enc_pool=None):
    """Build the engine + update source for one storage dtype, warm up, time exactly args.steps steps
    (barrier + device sync on both sides) and gather every rank's time and round outcomes."""
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    from svoc.parallel.dp import DataParallelConsensus

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    B = args.batch or c["batch"]
    D_local = c["D"]
    if dshard:
        from svoc.parallel.dshard import flush_sharded, run_round_sharded, shard_bounds
        lo, hi = shard_bounds(c["D"], rank, world)
        D_local = hi - lo
    # (constrained: false -- the reference's R^M mode, contract.cairo:370-434; max_spread in real units)
    cfg = ConsensusConfig(n_oracles=c["N"], dimension=D_local, n_failing_oracles=c["f"],
                          constrained=bool(c.get("constrained", True)),
                          unconstrained_max_spread=float(c.get("max_spread", 1.0)))
    mode = args.mode or c.get("mode", "fast")
    eng = ConsensusEngine(cfg, batch=B, device=dev, mode=mode, storage=storage)
    eng.wave_hint = args.wave_hint
    if mode == "fast":
        # transactional steps (default): a reverted round restores its instance's pre-batch rows
        eng.transactional = bool(args.transactional)
    dp = DataParallelConsensus(eng, rank=rank, world=world)
    eng.randomize(seed=1000 + (0 if dshard else rank))
    if c.get("price_centre") is not None and mode == "exact":
        # price-like unconstrained columns: the [0, 1] draws mapped onto centre +- spread real units
        sp, ce = float(c.get("price_spread", 200.0)), float(c["price_centre"])
        eng.values.copy_(((eng.values.double() - 500_000.0) * (2.0 * sp) + ce * 1e6).round().to(eng.values.dtype))

    # synthetic update stream resident in HBM: `pool` steps of updates, cycled
    U_per_inst = int(round(c["update_frac"] * c["N"]))
    stream = pipe = gov = None
    extra = {}
    if args.config == "c4":
        from svoc.models import corpus
        from svoc.models.sentiment_oracle import SentimentOraclePipeline
        enc = None
        if enc_dtype is not None or enc_pool is not None:
            # the reference's precision (HF pipeline, fp32 weights: oracle_scheduler.py:23-25): fp32 GEMMs over the
            # packed tokens, the fp32 encoder kernels (mfma_f32_32x32x2_f32 attention, fp32 LayerNorms); or the
            # reference's classifier head (RobertaClassificationHead on the <s> state: pool="cls")
            from svoc.models.encoder import EncoderConfig
            from svoc.models.encoder import build as build_encoder
            enc = build_encoder(dev, enc_dtype or torch.bfloat16, 0, EncoderConfig(pool=enc_pool or "mean"))
        pipe = SentimentOraclePipeline(eng, encoder=enc, seed=0)
        from svoc.models import encoder as _encm
        extra["encoder_pool"] = pipe.encoder.cfg.pool
        extra["encoder_gelu"] = "tanh (GEMM epilogue)" if _encm.GELU_EPILOGUE else "erf"
        extra["encoder_packed"] = bool(pipe.encoder.packed)
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
        # one distinct batch per timed step (a period-2 stream would let any cross-round reuse
        # measure cached answers), within a 96 GB budget for the resident pool
        elem = 8 if mode == "exact" else eng.values.element_size()
        per_batch = B * U_per_inst * (D_local * elem + 16)
        pool = max(2, min(args.steps, int(96e9 // max(1, per_batch)))) if dev.type == "cuda" else 2
        if args.stream_pool > 0:   # (A/B: a fixed pool, e.g. round 4's period-2 stream)
            pool = args.stream_pool
        extra["stream_pool"] = pool
        stream = SyntheticUpdateStream(B, c["N"], D_local, U_per_inst, c["f"], pool=pool, device=dev,
                                       seed=(0 if dshard else rank),
                                       dtype=torch.int64 if mode == "exact" else eng.vdtype,
                                       # the state's failing oracles stay the failing ones (D-shard:
                                       # every rank's slice of the same rows, so the stream's own set)
                                       failing=None if (dshard or c.get("independent_failing")) else eng.failing_mask)
        # (independent_failing: the stream draws its own failing oracles, so U(0,1) rows land among the
        # engine's reliable ones -- reliable outliers every round: the exact kernels' hard case)
        extra["independent_failing"] = bool(c.get("independent_failing"))
    if args.config == "c5":
        from svoc.codec import address_to_limbs
        from svoc.governance import Governance
        gov = Governance(B, 3, c["N"], dev, True, 2)
        gov.admins.copy_(torch.tensor([address_to_limbs(1000 + a) for a in range(3)], device=dev).expand(B, 3, 4))
        ora = torch.tensor([address_to_limbs(5000 + o) for o in range(c["N"])], device=dev)
        gov.oracle_addr.copy_(ora.expand(B, c["N"], 4))
        from svoc.stream import governance_stream
        gov_batches = governance_stream(B, c["N"], [1000, 1001, 1002], dev, seed=rank, frac=c["gov_frac"])
        extra["governance_actions_per_step"] = gov_batches[0][0].numel()
        extra["state_bytes_per_instance"] = (eng.state_bytes_per_instance() + 3 * 4 * 8 + 3 * 8 + 3 * (1 + 4 + 32)
                                             + c["N"] * 32)
        extra["instances_per_288GB"] = int(288e9 // extra["state_bytes_per_instance"])

    transactional = bool(c.get("transactional")) and stream is not None
    if transactional and mode != "exact":
        raise SystemExit("transactional streaming is the exact engine's per-update replay (mode: exact)")
    extra["transactional"] = transactional
    if mode == "fast" and stream is not None:
        extra["fast_transactional"] = eng.transactional
    pipeline = args.pipeline if args.pipeline >= 0 else c.get("pipeline", 1)
    if dshard or mode != "fast" or dev.type != "cuda":
        pipeline = 1
    extra["pipeline_chunks"] = pipeline

    def run_round():
        if dshard:
            # one packed all-reduce per round (qr partials + the previous round's status codes: the
            # previous round commits from it); the last round commits at flush()
            run_round_sharded(eng, c["D"], world=world, defer=world > 1)
        else:
            eng.run_round(only_touched=True)

    def step(i):  # device-only work (capturable)
        if pipe is not None:
            pipe.fetch(*toks[i % 2])
        elif stream is not None:
            inst, orc, vals = stream.batch(i)
            if transactional:   # exact: every update its own transaction (store + round, revert on failure)
                eng.step(inst, orc, vals, updates_per_instance=U_per_inst)
            elif pipeline > 1:   # the stream has distinct (instance, oracle), grouped by instance
                # consecutive steps overlap too (range 0's update beside the previous step's last
                # round); anything reading the state joins the streams first (engine.pipeline_join)
                eng.step_pipelined(inst, orc, vals, U_per_inst, chunks=pipeline, overlap=bool(args.overlap))
            else:
                eng.apply_updates(inst, orc, vals, unique=True)
                run_round()
        elif dshard:
            eng.touched.fill_(1)
            run_round()
        else:   # every active instance runs a round (the prologue ignores `touched`: no fill per step)
            eng.run_round(only_touched=False)
        if gov is not None:
            gov.submit_tensors(*gov_batches[i % len(gov_batches)])

    def flush():
        if dshard:
            flush_sharded(eng, world=world)

    def step_metrics():   # DP: one all-reduce of the round counters per call -- per graph replay (D-shard: every rank
        if not dshard:    # commits the same rounds, so the counters are reduced once, after the loop)
            dp.reduce()

    for i in range(args.warmup):
        step(i)
        step_metrics()
    flush()
    sync()

    graph = None
    graph_period = 1
    graph_ok = args.graph and dev.type == "cuda"
    if graph_ok and dshard and world > 1:
        # the D-shard round's RCCL all-reduce goes into the graph too (RCCL kernels are stream-capturable):
        # probe one captured all-reduce first, so a backend that cannot capture collectives runs eagerly
        graph_ok = _collectives_capturable(dev)
    extra["graph_collectives"] = bool(graph_ok and dshard and world > 1)
    if graph_ok:
        # the stream cycles with period `pool`: capture one period and replay it
        period = 1
        # (pipelined: a graph of at least 4 steps, so 3 of 4 step boundaries overlap; a pool of >= 4 steps
        # already overlaps all but one)
        sp = stream.pool if stream is not None else 1
        # (whole-batch rounds without a stream -- c2, the wide configs: every step is the same round of every
        # instance, so one graph holds up to 20 of them, as the streamed configs' graph holds its pool: the
        # metrics reduce runs once per replay either way)
        same = max(1, min(args.steps, 20)) if (stream is None and pipe is None and gov is None) else 1
        for k in (sp, len(gov_batches) if gov is not None else 1,
                  2 if pipe is not None else 1, 4 if (pipeline > 1 and sp < 4) else 1, same):
            period = period * k // math.gcd(period, k)
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        # (D-shard at world > 1: the streams only -- pipeline_join would commit the deferred round with a
        # collective; the graph's next round commits it from the engine's persistent pending buffers)
        join = eng._join_streams if (dshard and world > 1) else eng.pipeline_join
        with torch.cuda.stream(s):
            for i in range(period):
                step(i)
            join()
        torch.cuda.current_stream(dev).wait_stream(s)
        sync()
        try:
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                for i in range(period):
                    step(i)
                join()   # every forked stream rejoins the capture stream
            graph_period = period
            extra["graph_steps"] = period
        except Exception as e:  # graph capture is an optimisation; eager stays correct
            if rank == 0:
                print(f"[bench] graph capture failed ({e}); running eager", file=sys.stderr)
            graph = None

    # cross-step overlap happens only under graph replay: eager steps reduce the metrics every step, and
    # that joins the pipeline streams (engine.pipeline_join)
    extra["pipeline_overlap"] = bool(args.overlap) and pipeline > 1 and graph is not None
    fx0 = eng.metrics_fx.clone()   # this rank's round outcome counters before the timed steps
    if world > 1:
        dist.barrier()
    mark = None
    if getattr(args, "markers", False) and dev.type == "cuda":
        # (profiling only) a one-lane marker kernel on each side of the timed steps: tools/replay_kernels.py
        # keeps the trace's kernels between them -- the timed replay without setup, RNG or capture kernels
        global _MARK_SEQ
        _MARK_SEQ += 1
        mark = torch.zeros(1, dtype=torch.int32, device=dev)
        import svoc.ops as _svops
        _svops.ops().bench_marker(mark, 2 * _MARK_SEQ - 1)
    sync()
    t0 = time.perf_counter()
    if graph is not None:
        reps, rem = divmod(args.steps, graph_period)
        for _ in range(reps):
            graph.replay()
            step_metrics()         # one RCCL all-reduce of the step metrics per replay
        for i in range(rem):       # exactly K steps: the tail of a period runs eagerly
            step(i)
            step_metrics()
    else:
        for i in range(args.steps):
            step(i)
            step_metrics()
    flush()                        # (D-shard) the last round's commit: inside the timed region
    eng.pipeline_join()
    if mark is not None:
        _svops.ops().bench_marker(mark, 2 * _MARK_SEQ)
    sync()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    fx = (eng.metrics_fx - fx0).double()
    ns = eng.net_stats() if mode == "fast" else {"slab_networks": 0}
    if ns["slab_networks"]:
        # pruned window network (fp32, N = 256): share of slab networks whose exact check failed and reran
        # the full network (whole run, warm-up included)
        extra["pruned_net_fallback_rate"] = ns["fallbacks"] / ns["slab_networks"]
    if mode == "exact" and dev.type == "cuda":
        # exact rounds by kernel (whole run, warm-up included): the share handed to the i128 kernel and the share
        # the int64 wide-column kernel took (unconstrained columns spread past 2^30 wsad); the rest ran on the
        # column kernel
        xr = eng.exact_routing()
        if xr["processed"]:
            extra["exact_i128_share"] = xr["i128"] / xr["processed"]
            extra["exact_wide_column_share"] = xr["wide_column"] / xr["processed"]
    ok_local = float(fx[1] / fx[2]) if float(fx[2]) > 0 else 0.0
    mine = torch.tensor([t1 - t0, ok_local], dtype=torch.float64, device=dev)
    if world > 1:
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = torch.stack(allr).cpu()
    else:
        per_rank = mine[None].cpu()
    return dict(eng=eng, B=B, mode=mode, elapsed=float(per_rank[:, 0].max()),   # the slowest rank's time
                rounds_per_instance=U_per_inst if transactional else 1,
                U=U_per_inst, graph=graph is not None, extra=extra, step=step, storage=eng.storage,
                rank_ms=[1e3 * float(t) / args.steps for t in per_rank[:, 0]],
                rank_ok=[float(o) for o in per_rank[:, 1]], ok=dp.global_ok_fraction())


def _enc_fp32_gemm() -> str:
    from svoc.models import encoder
    return encoder.FP32_GEMM


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
    ap.add_argument("--overlap", type=int, default=1,
                    help="pipelined steps: overlap consecutive steps too (ConsensusEngine.step_pipelined "
                         "overlap=True); 0 = join the streams at the end of every step")
    ap.add_argument("--transactional", type=int, default=1,
                    help="fast streaming: save the rows each update overwrites and restore them for instances "
                         "whose round reverts (the reference's per-transaction atomicity); 0 = coalesced rows stay")
    ap.add_argument("--mode", default=None, choices=["fast", "exact"],
                    help="override the config's engine mode (exact = bit-exact wsad int64 path)")
    ap.add_argument("--storage", default=None, choices=["bf16", "fp32", "int64", "int32"],
                    help="engine value storage (default: the config's; exact mode: int64, int32 for constrained "
                         "configs).  Given explicitly, only that storage is measured (no alt_storage field)")
    ap.add_argument("--dshard", action="store_true",
                    help="strong scaling: every rank holds a column slice of ALL instances (D-sharding, one "
                         "[B, N] qr all-reduce per round) instead of its own instances (DP, default)")
    ap.add_argument("--backend", default=None, help="torch.distributed backend (default: nccl = RCCL on GPU)")
    ap.add_argument("--stream-pool", type=int, default=0,
                    help="streaming configs: distinct update batches cycled (0 = one per timed step, within 96 GB)")
    ap.add_argument("--log", default=None, help="append the result record to this JSON-lines file")
    ap.add_argument("--markers", action="store_true",
                    help="profiling: bracket each timed region with marker kernels (tools/replay_kernels.py)")
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
    # the world size the initialised backend reports (not just the launcher's environment)
    backend_world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    dshard = args.dshard   # world 1: the split-kernel path without collectives (its overhead)
    if dshard and args.config in ("c4", "c5"):
        raise SystemExit("--dshard is for the column-sharded configs (c2, c3, fast or exact)")

    from svoc.utils.metrics import algorithmic_bytes_per_round
    fast = (args.mode or c.get("mode", "fast")) == "fast"
    storage = args.storage or (c.get("storage") if fast else None)
    alt = c.get("alt_storage") if (fast and args.storage is None and dev.type == "cuda") else None
    scale = 1 if dshard else world   # D-sharding: all ranks share the same B instances

    def min_gbps(res, storage_bytes):
        # data-flow floor (one read of the values + outputs + the update rows in and out), not measured bytes
        rr = res["B"] * scale * args.steps
        return algorithmic_bytes_per_round(c["N"], c["D"], storage_bytes, res["U"]) * rr / res["elapsed"] / 1e9

    r = measure(args, c, storage, dev, rank, world, dshard)
    B, mode, el, U, eng = r["B"], r["mode"], r["elapsed"], r["U"], r["eng"]
    # transactional streaming: one round per update transaction (U per instance per step)
    rounds = B * scale * args.steps * r["rounds_per_instance"]
    out = {
        "metric": METRIC, "value": rounds / el, "unit": "consensus rounds/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * el / args.steps, "higher_is_better": True,
        "scaling": "strong" if dshard else "weak", "vs_baseline": None,
        "dtype": _dtype_name(mode, eng.storage, c), "data": "synthetic",
        "config": {"model": c["model"], "global_batch": B * scale, "seq_len": c["D"],
                   "parallelism": f"dshard{world}" if dshard else f"dp{world}", "engine_mode": mode,
                   "storage": eng.storage, "n_oracles": c["N"], "dimension": c["D"], "n_failing": c["f"],
                   "updates_per_instance_per_step": U, "oracle_updates_per_s": (U * B * scale * args.steps / el) if U else 0.0,
                   "hip_graph": r["graph"], "ok_fraction": r["ok"], "backend_world": backend_world,
                   "rank_ms_per_step": r["rank_ms"], "rank_ms_spread": [min(r["rank_ms"]), max(r["rank_ms"])],
                   "rank_ok_fraction": r["rank_ok"], **r["extra"]},
    }
    if args.config in ("c2", "c3") and mode == "fast":
        out["config"]["hbm_gbps_min_traffic"] = min_gbps(r, eng.values.element_size())
    log_eng, log_step = eng, r["step"]
    if alt:
        # the same step at the alternative storage dtype (a fresh engine; the first one is freed first)
        r = eng = None
        log_eng = log_step = None
        if dev.type == "cuda":
            torch.cuda.empty_cache()
        ra = measure(args, c, alt, dev, rank, world, dshard)
        out["config"]["alt_storage"] = {
            "storage": ra["storage"], "value": ra["B"] * scale * args.steps / ra["elapsed"],
            "ms_per_step": 1e3 * ra["elapsed"] / args.steps, "ok_fraction": ra["ok"],
            "hbm_gbps_min_traffic": min_gbps(ra, ra["eng"].values.element_size()),
            "rank_ms_spread": [min(ra["rank_ms"]), max(ra["rank_ms"])]}
        log_eng, log_step = ra["eng"], ra["step"]
    if args.config == "c3" and fast and args.storage is None and dev.type == "cuda" and not dshard:
        # the transaction-faithful form of the same stream: the EXACT engine (wsad, bit-identical to the
        # contract), every one of the 64 updates per instance its own transaction (store + full round +
        # revert on failure: contract.cairo:588-603).  Fixed 2 timed steps (1 warm-up): ~0.45 s each.
        import copy
        r = eng = None
        log_eng = log_step = None
        torch.cuda.empty_cache()
        ax = copy.copy(args)
        ax.steps, ax.warmup = 2, 1
        cx = {**c, "mode": "exact", "transactional": True}
        cx.pop("pipeline", None)
        rx = measure(ax, cx, None, dev, rank, world, dshard)
        out["config"]["exact_stream"] = {
            "engine": "exact (wsad)", "storage": rx["storage"], "transactions_per_instance_per_step": rx["U"],
            "value": rx["B"] * scale * ax.steps * rx["rounds_per_instance"] / rx["elapsed"],
            "unit": "consensus rounds/s (one per update transaction)", "steps": ax.steps, "warmup": ax.warmup,
            "ms_per_step": 1e3 * rx["elapsed"] / ax.steps, "ok_fraction": rx["ok"]}
        log_eng, log_step = rx["eng"], rx["step"]
    if c.get("alt_precision") == "fp32" and dev.type == "cuda":
        # c4 at the reference's precision: the same step with fp32 encoder weights / activations
        r = eng = None
        log_eng = log_step = None
        torch.cuda.empty_cache()
        rp = measure(args, c, storage, dev, rank, world, dshard, enc_dtype=torch.float32)
        out["config"]["alt_precision"] = {
            "encoder_dtype": "fp32", "value": rp["B"] * scale * args.steps / rp["elapsed"],
            "ms_per_step": 1e3 * rp["elapsed"] / args.steps, "ok_fraction": rp["ok"],
            "path": "packed tokens, fp32 MFMA attention + fp32 LayerNorm kernels, "
                    + ("fp32 GEMMs as six bf16 products of three-way bf16 splits (fp32 accumulate; "
                       "SVOC_FP32_GEMM=native: hipBLASLt fp32)" if _enc_fp32_gemm() == "bf16x6"
                       else "fp32 GEMMs (hipBLASLt)"),
            "fp32_gemm": _enc_fp32_gemm()}
        log_eng, log_step = rp["eng"], rp["step"]
    if args.config == "c4" and dev.type == "cuda":
        # the reference's head (client/oracle_scheduler.py:23-40: the <s> state through the classification
        # head, SamLowe/roberta-base-go_emotions) -- same encoder, <s> pooling instead of the masked mean
        r = eng = None
        log_eng = log_step = None
        torch.cuda.empty_cache()
        rc = measure(args, c, storage, dev, rank, world, dshard, enc_pool="cls")
        out["config"]["cls_pool"] = {
            "encoder_pool": "cls", "value": rc["B"] * scale * args.steps / rc["elapsed"],
            "ms_per_step": 1e3 * rc["elapsed"] / args.steps, "ok_fraction": rc["ok"]}
        log_eng, log_step = rc["eng"], rc["step"]
    if rank == 0:
        print(json.dumps(out))
        if args.log:
            from svoc.utils.metrics import JsonlLogger, engine_health, kernel_table
            rec = dict(out)
            rec["health"] = engine_health(log_eng)
            if args.kernel_table:
                rec["kernels"] = kernel_table(lambda: log_step(0), steps=args.kernel_table)
            with JsonlLogger(args.log, rank) as lg:
                lg.log("bench", **rec)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
