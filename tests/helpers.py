import torch

from svoc import ops as svops


def alloc_fast_out(B, N, D, device):
    f = dict(device=device)
    return dict(
        c1=torch.zeros(B, D, dtype=torch.float32, **f), consensus=torch.zeros(B, D, dtype=torch.float32, **f),
        skew=torch.zeros(B, D, dtype=torch.float32, **f), kurt=torch.zeros(B, D, dtype=torch.float32, **f),
        rel=torch.zeros(B, 2, dtype=torch.float32, **f), qr=torch.zeros(B, N, dtype=torch.float32, **f),
        reliable=torch.zeros(B, N, dtype=torch.uint8, **f), status=torch.full((B,), -1, dtype=torch.int32, **f))


def alloc_exact_out(B, N, D, device):
    f = dict(device=device, dtype=torch.int64)
    return dict(
        c1=torch.zeros(B, D, **f), consensus=torch.zeros(B, D, **f), skew=torch.zeros(B, D, **f),
        kurt=torch.zeros(B, D, **f), rel=torch.zeros(B, 2, **f), qr=torch.zeros(B, N, **f),
        reliable=torch.zeros(B, N, dtype=torch.uint8, device=device),
        status=torch.full((B,), -1, dtype=torch.int32, device=device))


def run_fast(values, D, n_failing, constrained, max_spread=1.0, active=None, wave_hint=0, legacy=False,
             work=None):
    B, N = values.shape[:2]
    o = alloc_fast_out(B, N, D, values.device)
    svops.ops().fast_round(values, active, D, n_failing, constrained, max_spread, o["c1"], o["consensus"],
                           o["skew"], o["kurt"], o["rel"], o["qr"], o["reliable"], o["status"], wave_hint,
                           0, 0, legacy, work)
    return o


def fast_work(B, D, device):
    return torch.empty(svops.fast_work_numel(B, D), dtype=torch.int32, device=device)


def run_exact(values, n_failing, constrained, max_spread=0, active=None, legacy=False):
    B, N, D = values.shape
    o = alloc_exact_out(B, N, D, values.device)
    svops.ops().exact_round(values, active, n_failing, constrained, max_spread, o["c1"], o["consensus"],
                            o["skew"], o["kurt"], o["rel"], o["qr"], o["reliable"], o["status"], legacy)
    return o


def beta_oracles(B, N, D, f, a=20.0, seed=0, device="cpu", dtype=torch.bfloat16, ld=None):
    """Honest oracles ~ Beta(a, a) per component, f failing ~ U(0,1), shuffled (notebook cell 3)."""
    g = torch.Generator().manual_seed(seed)
    # Beta(a, a) as Ga / (Ga + Gb), both gamma draws from g: a parametrisation is reproducible alone
    ga = torch._standard_gamma(torch.full((B, N, D), float(a)), generator=g)
    gb = torch._standard_gamma(torch.full((B, N, D), float(a)), generator=g)
    honest = ga / (ga + gb)
    fail = torch.rand(B, N, D, generator=g)
    is_fail = torch.zeros(B, N, dtype=torch.bool)
    for b in range(B):
        perm = torch.randperm(N, generator=g)[:f]
        is_fail[b, perm] = True
    x = torch.where(is_fail[:, :, None], fail, honest)
    ld = ld or ((D + 7) // 8) * 8
    out = torch.zeros(B, N, ld, dtype=dtype)
    out[:, :, :D] = x.to(dtype)
    return out.to(device), is_fail
