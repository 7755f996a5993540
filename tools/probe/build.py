"""Tools-only build of the diagnostic kernels (not part of svoc/_C.so): tools/probe/_probe.so.

    python tools/probe/build.py        # then python tools/probe/qr_mfma_ab.py

qr_probe.hip: the VALU vs MFMA formulation of the quadratic-risk pass (the round-2 A/B recorded in
profiles/r2_qr_mfma_ab.json).  Loaded with ctypes (plain C ABI, device pointers + a HIP stream).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "_probe.so")


def build(force: bool = False) -> str:
    src = os.path.join(HERE, "qr_probe.hip")
    if force or not os.path.exists(OUT) or os.path.getmtime(src) > os.path.getmtime(OUT):
        rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
        subprocess.run([os.path.join(rocm, "bin", "hipcc"), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        "-shared", src, "-o", OUT], check=True)
    return OUT


def qr_probe(values, c1, qr, variant: int) -> None:
    """values: bf16 [B, N, ld] (cuda), c1: fp32 [B, D], qr: fp32 [B, N] (written)."""
    import torch
    lib = ctypes.CDLL(build())
    B, N, ld = values.shape
    D = c1.shape[1]
    stream = torch.cuda.current_stream(values.device).cuda_stream
    rc = lib.svoc_qr_probe(ctypes.c_void_p(values.data_ptr()), ctypes.c_void_p(c1.data_ptr()),
                           ctypes.c_void_p(qr.data_ptr()), B, N, D, ld, int(variant), ctypes.c_void_p(stream))
    if rc != 0:
        raise RuntimeError(f"svoc_qr_probe failed: {rc}")


if __name__ == "__main__":
    print(build(force=True))
