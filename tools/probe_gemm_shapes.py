"""Probe: per-shape bf16 GEMM rates of the c4 encoder (BERT-base, 64 windows x 30 comments x 128 tokens)
under hipBLASLt vs rocBLAS, and with the weight stored as [N, K] (F.linear, "NT") vs pre-transposed
[K, N] ("NN").  One line per (shape, library, layout): ms and TFLOP/s.

    python tools/probe_gemm_shapes.py
"""
import time

import torch
import torch.nn.functional as F

M = 64 * 30 * 128
SHAPES = {"qkv": (768, 2304), "o": (768, 768), "fc1": (768, 3072), "fc2": (3072, 768)}


def bench(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t) / it


def main():
    torch.manual_seed(0)
    for name, (K, N) in SHAPES.items():
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        wt = w.t().contiguous()
        b = torch.randn(N, device="cuda", dtype=torch.bfloat16) * 0.02
        flop = 2.0 * M * K * N
        for lib in ("cublaslt", "cublas"):
            torch.backends.cuda.preferred_blas_library(lib)
            for layout, fn in (("NT", lambda: F.linear(x, w, b)),
                               ("NN", lambda: torch.addmm(b, x, wt))):
                ms = bench(fn)
                print(f"{name:4s} K={K:5d} N={N:5d} {lib:9s} {layout} {ms:8.3f} ms {flop / ms / 1e9:8.1f} TFLOP/s",
                      flush=True)
        del x, w, wt, b
    torch.backends.cuda.preferred_blas_library("cublaslt")


if __name__ == "__main__":
    main()
