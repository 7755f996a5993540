"""Multi-process GPU paths on a one-GPU box: two ranks share cuda:0 through the gloo backend (RCCL
refuses two ranks on one device), exercising DP metrics/all-gather and D-sharding with HIP kernels,
plus the RCCL (`nccl`) backend itself at world size 1.  The 8-GPU RCCL run is the driver's scaling bench."""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port, backend="gloo"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)


def _dp_worker(rank, world, port, outdir):
    _init(rank, world, port)
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    from svoc.parallel.dp import DataParallelConsensus
    cfg = ConsensusConfig(n_oracles=64, dimension=256, n_failing_oracles=8)
    e = ConsensusEngine(cfg, 16, device="cuda", mode="fast")
    dp = DataParallelConsensus(e, rank, world)
    e.randomize(seed=7 + rank)
    e.run_round()
    g = dp.reduce().cpu().clone()
    summ = {k: v.cpu() for k, v in dp.all_gather_summaries(k=4).items()}
    torch.save(dict(g=g, summ=summ, local=e.consensus[:, :4].cpu().clone(), rel=e.rel.cpu().clone()),
               os.path.join(outdir, f"dp{rank}.pt"))
    dist.destroy_process_group()


def test_dp_two_ranks_on_one_gpu():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_dp_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"dp{i}.pt"), weights_only=True) for i in range(world)]
    assert torch.equal(r[0]["g"], r[1]["g"]) and r[0]["g"][2].item() == 32
    rel2 = torch.cat([r[0]["rel"][:, 1], r[1]["rel"][:, 1]]).double().sum().item()
    assert abs(r[0]["g"][0].item() - rel2) < 1e-5
    full = r[1]["summ"]["consensus"]
    torch.testing.assert_close(full[:16].float(), r[0]["local"].float())
    torch.testing.assert_close(full[16:].float(), r[1]["local"].float())


def _ds_worker(rank, world, port, outdir, x, cfgd):
    _init(rank, world, port)
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    from svoc.parallel.dshard import run_round_sharded, shard_bounds
    cfg = ConsensusConfig(**cfgd)
    lo, hi = shard_bounds(cfg.dimension, rank, world)
    e = ConsensusEngine(ConsensusConfig(**{**cfgd, "dimension": hi - lo}), x.shape[0], device="cuda", mode="fast")
    e.values[:, :, : hi - lo] = x[:, :, lo:hi].to("cuda", torch.bfloat16)
    e.enabled.fill_(1); e.n_active.fill_(cfg.n_oracles); e.touched.fill_(1)
    run_round_sharded(e, cfg.dimension, world=world)
    torch.save(dict(cons=e.consensus.cpu(), rel=e.rel.cpu(), reliable=e.reliable.cpu(), st=e.status.cpu(),
                    lo=lo, hi=hi), os.path.join(outdir, f"ds{rank}.pt"))
    dist.destroy_process_group()


def test_dsharding_two_ranks_on_one_gpu():
    from helpers import beta_oracles, run_fast
    B, N, D, f = 6, 128, 600, 16
    x, _ = beta_oracles(B, N, D, f, seed=5)
    x = x[:, :, :D].contiguous()
    ref = run_fast(x.cuda(), D, f, True, 1.0)
    cfgd = dict(n_oracles=N, dimension=D, n_failing_oracles=f, constrained=True)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_ds_worker, args=(2, _free_port(), d, x, cfgd), nprocs=2, join=True)
        r = [torch.load(os.path.join(d, f"ds{i}.pt"), weights_only=True) for i in range(2)]
    for s in r:
        assert torch.equal(s["st"], ref["status"].cpu())
        assert torch.equal(s["reliable"], ref["reliable"].cpu())
        torch.testing.assert_close(s["rel"], ref["rel"].cpu(), rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(s["cons"], ref["consensus"].cpu()[:, s["lo"]:s["hi"]], rtol=0, atol=1e-6)


def _rccl_worker(rank, world, port, outdir):
    _init(rank, world, port, backend="nccl")
    t = torch.arange(4, dtype=torch.int64, device="cuda")
    dist.all_reduce(t)
    torch.save(t.cpu(), os.path.join(outdir, "rccl.pt"))
    dist.destroy_process_group()


def test_rccl_backend_world1():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rccl_worker, args=(1, _free_port(), d), nprocs=1, join=True)
        assert torch.load(os.path.join(d, "rccl.pt"), weights_only=True).tolist() == [0, 1, 2, 3]


def _ds_exact_worker(rank, world, port, outdir, x, cfgd):
    _init(rank, world, port)
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    from svoc.parallel.dshard import run_round_sharded, shard_bounds
    cfg = ConsensusConfig(**cfgd)
    lo, hi = shard_bounds(cfg.dimension, rank, world)
    e = ConsensusEngine(ConsensusConfig(**{**cfgd, "dimension": hi - lo}), x.shape[0], device="cuda", mode="exact")
    e.values.copy_(x[:, :, lo:hi].to("cuda", e.values.dtype))
    e.enabled.fill_(1); e.n_active.fill_(cfg.n_oracles); e.touched.fill_(1)
    run_round_sharded(e, cfg.dimension, world=world)
    torch.save({k: getattr(e, k).cpu() for k in ("consensus", "skew", "kurt", "rel", "qr", "reliable", "status")}
               | dict(lo=lo, hi=hi), os.path.join(outdir, f"dse{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("constrained", [True, False])
def test_dsharding_exact_two_ranks_on_one_gpu(constrained):
    """Exact (wsad) D-sharding on the GPU split modes (column kernel, i128 kernel for what it hands over;
    unconstrained: signed values): bit-identical to one whole round."""
    from helpers import beta_oracles
    from svoc.config import ConsensusConfig
    from svoc.engine import ConsensusEngine
    B, N, D, f = 6, 64, 200, 8
    x, _ = beta_oracles(B, N, D, f, seed=9, dtype=torch.float64)
    x = (x[:, :, :D] * 1e6).to(torch.int64).contiguous()
    if not constrained:
        x = x * 3 - 1_500_000          # signed, wider than [0, 1e6]
    cfgd = dict(n_oracles=N, dimension=D, n_failing_oracles=f, constrained=constrained, unconstrained_max_spread=1.0)
    ref = ConsensusEngine(ConsensusConfig(**cfgd), B, device="cuda", mode="exact")
    ref.values.copy_(x.to("cuda", ref.values.dtype))
    ref.enabled.fill_(1); ref.n_active.fill_(N); ref.touched.fill_(1)
    ref.run_round()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_ds_exact_worker, args=(2, _free_port(), d, x, cfgd), nprocs=2, join=True)
        r = [torch.load(os.path.join(d, f"dse{i}.pt"), weights_only=True) for i in range(2)]
    assert (ref.status == 0).all()
    for s in r:
        for k in ("rel", "qr", "reliable", "status"):
            assert torch.equal(s[k], getattr(ref, k).cpu()), k
        for k in ("consensus", "skew", "kurt"):
            assert torch.equal(s[k], getattr(ref, k).cpu()[:, s["lo"]:s["hi"]]), k
