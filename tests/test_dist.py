"""Multi-process paths on CPU with the gloo backend (world sizes 2 and 4): DP and D-sharding."""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from svoc import ops as svops
from svoc.status import Status

pytestmark = pytest.mark.skipif(not svops.available(), reason="svoc/_C.so not built")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)


def _dp_worker(rank, world, port, outdir):
    _init(rank, world, port)
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    from svoc.parallel.dp import DataParallelConsensus
    cfg = ConsensusConfig(n_oracles=16, dimension=24, n_failing_oracles=2)
    e = ConsensusEngine(cfg, 3, device="cpu", mode="fast")
    dp = DataParallelConsensus(e, rank, world)
    e.randomize(seed=100 + rank)
    e.run_round()
    dp.accumulate()
    g = dp.reduce().clone()
    summ = dp.all_gather_summaries(k=4)
    torch.save(dict(g=g, summ=summ, ids=dp.global_ids(), local=e.consensus[:, :4].clone(),
                    rel=e.rel.clone()), os.path.join(outdir, f"dp{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_data_parallel_gloo(world):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_dp_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"dp{i}.pt"), weights_only=True) for i in range(world)]
    for k in range(1, world):
        assert torch.equal(r[0]["g"], r[k]["g"])
    assert r[0]["g"][2].item() == 3 * world            # world ranks x 3 instances processed
    # rel2 sum over committed rounds (fixed-point 2^-32 counters, all-reduced as integers)
    rel2 = torch.cat([r[k]["rel"][:, 1] for k in range(world)]).double().sum().item()
    assert abs(r[0]["g"][0].item() - rel2) < 1e-6 and r[0]["g"][1].item() == 3 * world
    full = r[0]["summ"]["consensus"]
    for k in range(world):
        assert torch.allclose(full[3 * k:3 * k + 3].float(), r[k]["local"].float())
        assert r[k]["ids"].tolist() == [3 * k, 3 * k + 1, 3 * k + 2]


def _ds_worker(rank, world, port, outdir, x, cfgd, storage="bf16"):
    _init(rank, world, port)
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    from svoc.parallel.dshard import run_round_sharded, shard_bounds
    cfg = ConsensusConfig(**cfgd)
    lo, hi = shard_bounds(cfg.dimension, rank, world)
    lcfg = ConsensusConfig(**{**cfgd, "dimension": hi - lo})
    e = ConsensusEngine(lcfg, x.shape[0], device="cpu", mode="fast", storage=storage)
    e.values[:, :, : hi - lo] = x[:, :, lo:hi]
    e.enabled.fill_(1); e.n_active.fill_(cfg.n_oracles); e.touched.fill_(1)
    run_round_sharded(e, cfg.dimension, world=world)
    torch.save(dict(cons=e.consensus.clone(), rel=e.rel.clone(), reliable=e.reliable.clone(),
                    skew=e.skew.clone(), st=e.status.clone(), lo=lo, hi=hi),
               os.path.join(outdir, f"ds{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("constrained,world,storage", [(True, 2, "bf16"), (False, 2, "bf16"), (True, 4, "bf16"),
                                                       (True, 2, "fp32"), (False, 3, "fp32")])
def test_dsharding_matches_single_process(constrained, world, storage):
    from helpers import beta_oracles, run_fast
    B, N, D, f = 4, 32, 40, 4
    x, _ = beta_oracles(B, N, D, f, seed=11, dtype=torch.bfloat16 if storage == "bf16" else torch.float32)
    x = x[:, :, :D].contiguous()
    ref = run_fast(x, D, f, constrained, 1.0)
    cfgd = dict(n_oracles=N, dimension=D, n_failing_oracles=f, constrained=constrained, unconstrained_max_spread=1.0)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_ds_worker, args=(world, _free_port(), d, x, cfgd, storage), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"ds{i}.pt"), weights_only=True) for i in range(world)]
    for s in r:
        assert torch.equal(s["st"], ref["status"])
        assert torch.equal(s["reliable"], ref["reliable"])
        torch.testing.assert_close(s["rel"], ref["rel"], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(s["cons"], ref["consensus"][:, s["lo"]:s["hi"]], rtol=0, atol=1e-6)
        torch.testing.assert_close(s["skew"], ref["skew"][:, s["lo"]:s["hi"]], rtol=1e-4, atol=1e-4)


def _ds_revert_worker(rank, world, port, outdir, x1, x2, cfgd):
    _init(rank, world, port)
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    from svoc.parallel.dshard import run_round_sharded, shard_bounds
    cfg = ConsensusConfig(**cfgd)
    lo, hi = shard_bounds(cfg.dimension, rank, world)
    e = ConsensusEngine(ConsensusConfig(**{**cfgd, "dimension": hi - lo}), x1.shape[0], device="cpu", mode="fast")
    out = {}
    for k, x in enumerate((x1, x2)):
        e.values[:, :, : hi - lo] = x[:, :, lo:hi]
        e.enabled.fill_(1); e.n_active.fill_(cfg.n_oracles); e.touched.fill_(1)
        run_round_sharded(e, cfg.dimension, world=world)
        out[k] = dict(cons=e.consensus.clone(), rel=e.rel.clone(), reliable=e.reliable.clone(), qr=e.qr.clone(),
                      skew=e.skew.clone(), kurt=e.kurt.clone(), st=e.status.clone(), act=e.consensus_active.clone(),
                      c1=e.c1.clone())
    torch.save(dict(out=out, lo=lo, hi=hi), os.path.join(outdir, f"dsr{rank}.pt"))
    dist.destroy_process_group()


def test_dsharding_revert_is_atomic_across_shards():
    """Zero variance in one shard's columns only: every shard reverts that instance (no output moves)."""
    from helpers import beta_oracles
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    B, N, D, f, world = 4, 32, 40, 4, 2
    x1, _ = beta_oracles(B, N, D, f, seed=21)
    x1 = x1[:, :, :D].contiguous()
    x2, _ = beta_oracles(B, N, D, f, seed=22)
    x2 = x2[:, :, :D].contiguous()
    x2[1, :, 2] = 0.5           # column 2 lives in shard 0: constant -> zero variance there only
    x2[3, :, 25] = 0.25         # column 25: shard 1 only
    cfgd = dict(n_oracles=N, dimension=D, n_failing_oracles=f, constrained=True)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_ds_revert_worker, args=(world, _free_port(), d, x1, x2, cfgd), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"dsr{i}.pt"), weights_only=True) for i in range(world)]
    # single-process reference (CPU fast engine, all columns)
    ref = ConsensusEngine(ConsensusConfig(**cfgd), B, device="cpu", mode="fast")
    snaps = []
    for x in (x1, x2):
        ref.values[:, :, :D] = x
        ref.enabled.fill_(1); ref.n_active.fill_(N); ref.touched.fill_(1)
        ref.run_round()
        snaps.append(dict(cons=ref.consensus.clone(), st=ref.status.clone(), rel=ref.rel.clone(), qr=ref.qr.clone(),
                          reliable=ref.reliable.clone(), skew=ref.skew.clone()))
    assert snaps[1]["st"].tolist() == [0, 32, 0, 32]
    for s in r:
        o1, o2 = s["out"][0], s["out"][1]
        assert o2["st"].tolist() == [0, 32, 0, 32]
        for inst in (1, 3):   # reverted: every output identical to round 1, bit for bit
            for k in ("cons", "rel", "reliable", "qr", "skew", "kurt", "c1"):
                assert torch.equal(o2[k][inst], o1[k][inst]), (k, inst)
        for inst in (0, 2):
            assert not torch.equal(o2["cons"][inst], o1["cons"][inst])
        assert torch.equal(o2["reliable"], snaps[1]["reliable"])
        torch.testing.assert_close(o2["cons"], snaps[1]["cons"][:, s["lo"]:s["hi"]], rtol=0, atol=1e-6)
        torch.testing.assert_close(o2["rel"], snaps[1]["rel"], rtol=1e-5, atol=1e-6)
    # the single-process engine reverts the same instances and leaves round 1's outputs
    for inst in (1, 3):
        assert torch.equal(snaps[1]["cons"][inst], snaps[0]["cons"][inst])
        assert torch.equal(snaps[1]["qr"][inst], snaps[0]["qr"][inst])


def _ds_defer_worker(rank, world, port, outdir, xs, cfgd, mode):
    """The same rounds eagerly committed and deferred (one collective per round, flush at the end),
    counting the all-reduces of the deferred run."""
    _init(rank, world, port)
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    from svoc.parallel import dshard
    cfg = ConsensusConfig(**cfgd)
    lo, hi = dshard.shard_bounds(cfg.dimension, rank, world)
    lcfg = ConsensusConfig(**{**cfgd, "dimension": hi - lo})
    # 0: eager commits; 1: deferred, flushed explicitly; 2: deferred, committed by a state reader (getter)
    engines = [ConsensusEngine(lcfg, xs[0].shape[0], device="cpu", mode=mode) for _ in range(3)]
    calls = []
    real = dist.all_reduce

    def counting(t, *a, **k):
        calls.append(tuple(t.shape))
        return real(t, *a, **k)

    out = []
    for j, e in enumerate(engines):
        dist.all_reduce = counting if j == 1 else real
        try:
            for x in xs:
                e.values[:, :, : hi - lo] = x[:, :, lo:hi]
                e.enabled.fill_(1); e.n_active.fill_(cfg.n_oracles); e.touched.fill_(1)
                dshard.run_round_sharded(e, cfg.dimension, world=world, defer=(j >= 1))
                if j == 1:
                    calls.append("round")
            if j == 2:
                e.get_consensus_value()          # engine.pipeline_join commits the pending round
                assert getattr(e, "_dshard_pending", None) is None
            else:
                dshard.flush_sharded(e, world=world)
        finally:
            dist.all_reduce = real
        out.append({k: getattr(e, k).clone() for k in ("consensus", "rel", "reliable", "qr", "skew", "kurt", "c1",
                                                       "status", "consensus_active", "touched", "metrics_fx")})
    torch.save(dict(out=out, calls=calls), os.path.join(outdir, f"dd{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["fast", "exact"])
def test_dsharding_deferred_commit_one_collective_per_round(mode):
    """defer=True: each round issues ONE all-reduce (qr partials + every rank's status codes packed in one
    SUM buffer; the previous round commits from it), plus one status MAX at flush -- and the state after
    the flush is identical to the eagerly committed rounds, reverts included."""
    from helpers import beta_oracles
    from svoc.config import WSAD
    B, N, D, f, world = 4, 16, 24, 2, 2
    xs = []
    for seed in (31, 32, 33):
        x, _ = beta_oracles(B, N, D, f, seed=seed)
        xs.append(x[:, :, :D].contiguous())
    xs[1][1, :, 2] = 0.5        # round 2: zero variance in shard 0's column 2 only -> instance 1 reverts
    xs[2][3, :, 20] = 0.25      # round 3: shard 1 only -> instance 3 reverts
    if mode == "exact":
        xs = [(x.double() * WSAD).to(torch.int64) for x in xs]
    cfgd = dict(n_oracles=N, dimension=D, n_failing_oracles=f, constrained=True)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_ds_defer_worker, args=(world, _free_port(), d, xs, cfgd, mode), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"dd{i}.pt"), weights_only=True) for i in range(world)]
    for s in r:
        eager, deferred, via_getter = s["out"]
        for k in eager:
            assert torch.equal(eager[k], deferred[k]), k
            assert torch.equal(eager[k], via_getter[k]), k
        assert eager["status"].tolist()[1] == 0 and eager["status"].tolist()[3] != 0
        # one collective per round, the packed [B, N + 2 * world] buffer; the flush's status MAX last
        assert s["calls"] == [(B, N + 2 * world), "round"] * 3 + [(B,)], s["calls"]


def _ds_defer_txn_worker(rank, world, port, outdir, xs, ups, cfgd):
    """Transactional fast engines, D-sharded: the same update batches and rounds committed eagerly and
    deferred.  A deferred round's revert must restore its batch's rows / enabled / n_active before the next
    batch lands (apply_updates flushes the pending verdict first)."""
    _init(rank, world, port)
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    from svoc.parallel import dshard
    cfg = ConsensusConfig(**cfgd)
    lo, hi = dshard.shard_bounds(cfg.dimension, rank, world)
    lcfg = ConsensusConfig(**{**cfgd, "dimension": hi - lo})
    out = []
    for defer in (False, True):
        e = ConsensusEngine(lcfg, xs.shape[0], device="cpu", mode="fast", storage="fp32")
        e.values[:, :, : hi - lo] = xs[:, :, lo:hi]
        e.enabled.fill_(1); e.n_active.fill_(cfg.n_oracles); e.touched.fill_(1)
        dshard.run_round_sharded(e, cfg.dimension, world=world, defer=defer)
        sts, snaps = [], []
        for inst, orc, rows in ups:
            sts.append(e.apply_updates(inst, orc, rows[:, lo:hi].contiguous()))
            snaps.append({k: getattr(e, k).clone() for k in ("values", "enabled", "n_active")})
            dshard.run_round_sharded(e, cfg.dimension, world=world, defer=defer)
        dshard.flush_sharded(e, world=world)
        out.append(dict(st=[s.clone() for s in sts], snaps=snaps,
                        **{k: getattr(e, k).clone() for k in ("values", "enabled", "n_active", "status", "consensus",
                                                             "rel", "reliable", "c1")}))
    torch.save(dict(out=out, lo=lo, hi=hi), os.path.join(outdir, f"dt{rank}.pt"))
    dist.destroy_process_group()


def test_dsharding_deferred_rounds_are_transactional():
    """A deferred D-shard round that reverts (zero variance in ONE shard's column) leaves no trace: its update
    batch's rows, enabled flags and n_active are restored on every rank before the next batch is stored, and
    the result equals the eagerly committed rounds bit for bit (statuses of every update included)."""
    from helpers import beta_oracles
    B, N, D, f, world = 4, 16, 24, 2, 2
    x, _ = beta_oracles(B, N, D, f, seed=41)
    x = x[:, :, :D].contiguous().float()
    g = torch.Generator().manual_seed(3)
    # batch 1: instance 1 -> every oracle, column 2 (shard 0) at one value: its round reverts; instance 0: two rows
    rows1 = torch.rand(N + 2, D, generator=g)
    rows1[:N, 2] = 0.5
    ups = [(torch.tensor([1] * N + [0, 0]), torch.cat([torch.arange(N), torch.tensor([3, 9])]), rows1),
           # batch 2: ordinary rows for instances 1 and 2 (lands on instance 1's restored rows)
           (torch.tensor([1, 2]), torch.tensor([3, 5]), torch.rand(2, D, generator=g))]
    cfgd = dict(n_oracles=N, dimension=D, n_failing_oracles=f, constrained=True)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_ds_defer_txn_worker, args=(world, _free_port(), d, x, ups, cfgd), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"dt{i}.pt"), weights_only=True) for i in range(world)]
    for s in r:
        eager, deferred = s["out"]
        for k in ("values", "enabled", "n_active", "status", "consensus", "rel", "reliable", "c1"):
            assert torch.equal(eager[k], deferred[k]), k
        for a, b in zip(eager["st"], deferred["st"]):
            assert torch.equal(a, b)
        assert (eager["st"][0][:N] == int(Status.ZERO_VARIANCE)).all() and eager["st"][0][N:].tolist() == [0, 0]
        # instance 1: batch 1 rolled back, then batch 2's row for oracle 3 stored on the original rows
        v1 = x[1, :, s["lo"]:s["hi"]].clone()
        v1[3] = ups[1][2][0, s["lo"]:s["hi"]]
        assert torch.equal(deferred["values"][1, :, : s["hi"] - s["lo"]], v1)


def _ds_exact_worker(rank, world, port, outdir, xs, cfgd):
    _init(rank, world, port)
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    from svoc.parallel.dshard import run_round_sharded, shard_bounds
    cfg = ConsensusConfig(**cfgd)
    lo, hi = shard_bounds(cfg.dimension, rank, world)
    e = ConsensusEngine(ConsensusConfig(**{**cfgd, "dimension": hi - lo}), xs[0].shape[0], device="cpu", mode="exact")
    out = []
    for x in xs:
        e.values.copy_(x[:, :, lo:hi].to(e.values.dtype))
        e.enabled.fill_(1); e.n_active.fill_(cfg.n_oracles); e.touched.fill_(1)
        run_round_sharded(e, cfg.dimension, world=world)
        out.append({k: getattr(e, k).clone() for k in ("consensus", "skew", "kurt", "rel", "qr", "reliable", "c1",
                                                        "status", "consensus_active")})
    torch.save(dict(out=out, lo=lo, hi=hi), os.path.join(outdir, f"dse{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("constrained,world,N,D,f", [(True, 2, 16, 11, 3), (True, 3, 16, 11, 3), (False, 2, 16, 11, 3),
                                                     (True, 2, 4096, 64, 512), (True, 4, 4096, 64, 512),
                                                     (True, 2, 512, 2048, 64), (True, 4, 512, 2048, 64)])
def test_dsharding_exact_bit_identical(constrained, world, N, D, f):
    """Exact (wsad) engine, D-sharded: every output of every round equals the single-process exact engine
    bit for bit (qr = the int64 sum of the shards' partials); a zero-variance column in one shard reverts
    the instance on every shard with the single-process code, leaving the previous round's outputs.
    4096 x 64 and 512 x 2048: the wide shapes (N > 256) of VERDICT r5 item 5."""
    from helpers import beta_oracles
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    B = 4 if N <= 256 else 2
    xs = []
    for seed in (31, 32):
        x, _ = beta_oracles(B, N, D, f, seed=seed, dtype=torch.float64)
        xs.append((x[:, :, :D] * 1e6).to(torch.int64).contiguous())
    xs[1][1, :, 1] = 500_000      # shard 0's column: zero variance -> that instance reverts
    if not constrained:
        xs = [x - 400_000 for x in xs]   # signed values (unconstrained domain)
    cfgd = dict(n_oracles=N, dimension=D, n_failing_oracles=f, constrained=constrained,
                unconstrained_max_spread=1.0)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_ds_exact_worker, args=(world, _free_port(), d, xs, cfgd), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"dse{i}.pt"), weights_only=True) for i in range(world)]
    ref = ConsensusEngine(ConsensusConfig(**cfgd), B, device="cpu", mode="exact")
    snaps = []
    for x in xs:
        ref.values.copy_(x.to(ref.values.dtype))
        ref.enabled.fill_(1); ref.n_active.fill_(N); ref.touched.fill_(1)
        ref.run_round()
        snaps.append({k: getattr(ref, k).clone() for k in ("consensus", "skew", "kurt", "rel", "qr", "reliable",
                                                            "c1", "status", "consensus_active")})
    assert snaps[0]["status"].tolist() == [0] * B
    others = [i for i in range(B) if i != 1]
    assert snaps[1]["status"][1].item() != 0 and snaps[1]["status"][others].tolist() == [0] * len(others)
    for s in r:
        lo, hi = s["lo"], s["hi"]
        for k, (o, ref_o) in enumerate(zip(s["out"], snaps)):
            for name in ("rel", "qr", "reliable", "status", "consensus_active"):
                assert torch.equal(o[name], ref_o[name]), (k, name)
            for name in ("consensus", "skew", "kurt", "c1"):
                assert torch.equal(o[name], ref_o[name][:, lo:hi]), (k, name)


def test_dsharding_exact_rejects_more_than_32_shards():
    """Exact D-sharding all-reduces int64 qr partials bounded below 2^58: more than 32 shards could wrap
    the sum, so the sharded round refuses."""
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    from svoc.parallel.dshard import MAX_EXACT_SHARDS, run_round_sharded
    e = ConsensusEngine(ConsensusConfig(n_oracles=8, dimension=4, n_failing_oracles=1, constrained=True), 2,
                        device="cpu", mode="exact")
    with pytest.raises(ValueError):
        run_round_sharded(e, 4 * (MAX_EXACT_SHARDS + 1), world=MAX_EXACT_SHARDS + 1)
