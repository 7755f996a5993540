"""Probe: hipBLASLt GELU epilogue (torch._addmm_activation) vs Linear + F.gelu for the encoder FC1."""
import time

import torch
import torch.nn.functional as F

M, K, N = 245760, 768, 3072
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
b = torch.randn(N, device="cuda", dtype=torch.bfloat16) * 0.02


def bench(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t) / it


ref = F.gelu(F.linear(x, w, b))
print("linear+gelu      ms", bench(lambda: F.gelu(F.linear(x, w, b))))
print("linear+gelu(tanh)ms", bench(lambda: F.gelu(F.linear(x, w, b), approximate="tanh")))
try:
    out = torch._addmm_activation(b, x, w.t(), use_gelu=True)
    print("addmm_activation ms", bench(lambda: torch._addmm_activation(b, x, w.t(), use_gelu=True)))
    print("max |diff| vs exact gelu", (out.float() - ref.float()).abs().max().item())
except Exception as e:  # noqa: BLE001
    print("addmm_activation failed:", e)
print("linear only      ms", bench(lambda: F.linear(x, w, b)))
