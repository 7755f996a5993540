"""Probe: fp32 linear as native hipBLASLt fp32 GEMM vs three bf16 GEMMs with fp32 output (encoder._emul_linear)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from svoc import ops as svops
from svoc.models.encoder import _emul_linear


def t(fn, n=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def main():
    svops.load()
    M = 154065
    for K, N in ((768, 2304), (768, 768), (768, 3072), (3072, 768)):
        fc = torch.nn.Linear(K, N).cuda()
        x = torch.randn(M, K, device="cuda")
        xp = svops.ops().split3(x, False)
        xb = x.bfloat16()
        wb = fc.weight.bfloat16()
        fl = 2 * M * K * N
        r = {
            "fp32": t(lambda: torch.addmm(fc.bias, x, fc.weight.t())),
            "split": t(lambda: svops.ops().split3(x, False)),
            "emul": t(lambda: _emul_linear(xp, fc)),
            "bf16_out_bf16": t(lambda: torch.mm(xb, wb.t())),
            "bf16_out_f32": t(lambda: torch.mm(xb, wb.t(), out_dtype=torch.float32)),
            "bf16_3K_out_f32": t(lambda: torch.mm(xp, torch.cat([wb, wb, wb], 1).t(), out_dtype=torch.float32)),
        }
        print(K, N, {k: f"{v:.3f} ms ({fl / v / 1e9:.0f} TF/s eq)" for k, v in r.items()})


if __name__ == "__main__":
    main()
