"""Which GELU does torch._addmm_activation(use_gelu=True) compute on this device: erf or tanh?"""
import torch
import torch.nn.functional as F

torch.manual_seed(0)
for dt in (torch.float32, torch.bfloat16):
    x = torch.randn(512, 768, device="cuda", dtype=dt)
    w = torch.randn(3072, 768, device="cuda", dtype=dt) * 0.05
    b = torch.randn(3072, device="cuda", dtype=dt) * 0.5
    y = torch._addmm_activation(b, x, w.t(), use_gelu=True).float()
    lin = F.linear(x, w, b).float()
    e = (y - F.gelu(lin)).abs().max().item()
    t = (y - F.gelu(lin, approximate="tanh")).abs().max().item()
    print(f"{dt}: max|epilogue - erf gelu| = {e:.3e}   max|epilogue - tanh gelu| = {t:.3e}   -> "
          f"{'tanh' if t < e else 'erf'}")
