"""Build the in-tree extension ``svoc/_C.so`` (gfx950 HIP kernels + torch op bindings + C++ engines).

No hipify and no torch.utils.cpp_extension: ``.hip`` kernels are compiled by hipcc for gfx950 only,
host C++ by g++ against the PyTorch-ROCm headers, and everything is linked by hipcc into one shared
object next to the Python package (so it travels with the repo snapshot to the GPU box).

    python csrc/build.py [--force] [--jobs N] [--debug]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "obj")
OUT = os.path.join(ROOT, "svoc", "_C.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def torch_paths():
    import torch
    base = os.path.dirname(torch.__file__)
    return base, [os.path.join(base, "include"), os.path.join(base, "include", "torch", "csrc", "api", "include")]


def headers():
    return glob.glob(os.path.join(CSRC, "**", "*.hpp"), recursive=True)


def file_flags(src):
    """Extra hipcc flags a kernel source asks for in its header (``// svoc-hipcc-flags: ...``)."""
    with open(src, encoding="utf-8") as f:
        for _, line in zip(range(60), f):
            if "svoc-hipcc-flags:" in line:
                return line.split("svoc-hipcc-flags:", 1)[1].split()
    return []


def stale(obj, src, deps):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(p) > t for p in [src] + deps)


def run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}):\n{' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def build(force: bool = False, jobs: int = 8, debug: bool = False, verbose: bool = False) -> str:
    tbase, tinc = torch_paths()
    os.makedirs(BUILD, exist_ok=True)
    inc = ["-I" + os.path.join(CSRC, "include"), "-I" + CSRC]
    opt = ["-O0", "-g"] if debug else ["-O3"]
    hip_srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    cpp_srcs = sorted(glob.glob(os.path.join(CSRC, "engine", "*.cpp")) + glob.glob(os.path.join(CSRC, "bindings", "*.cpp")))
    deps = headers()
    jobs_list = []
    for src in hip_srcs:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        # per-file kernel flags: a "// svoc-hipcc-flags: ..." line in the source's header comment
        # SVOC_HIPCC_FLAGS: extra kernel flags for A/B builds of experimental variants
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", *opt, *inc, *file_flags(src),
               *os.environ.get("SVOC_HIPCC_FLAGS", "").split(), "-c", src, "-o", obj]
        jobs_list.append((src, obj, cmd))
    py_inc = sysconfig.get_paths()["include"]
    defs = ["-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-D_GLIBCXX_USE_CXX11_ABI=1", "-DTORCH_EXTENSION_NAME=_C"]
    for src in cpp_srcs:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        is_binding = os.sep + "bindings" + os.sep in src
        extra = [*(f"-I{p}" for p in tinc), f"-I{ROCM}/include", f"-I{py_inc}", *defs] if is_binding else [f"-I{ROCM}/include"]
        cmd = ["g++", "-std=c++17", "-fPIC", *opt, "-Wall", "-Wno-unused-function", *inc, *extra, "-c", src, "-o", obj]
        jobs_list.append((src, obj, cmd))
    todo = [j for j in jobs_list if force or stale(j[1], j[0], deps)]
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        futs = {ex.submit(run, cmd): src for src, obj, cmd in todo}
        for f in cf.as_completed(futs):
            out = f.result()
            if verbose and out.strip():
                print(out)
    objs = [j[1] for j in jobs_list]
    if force or todo or not os.path.exists(OUT) or any(os.path.getmtime(o) > os.path.getmtime(OUT) for o in objs):
        tmp = OUT + ".tmp"
        link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp,
                f"-L{tbase}/lib", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
                f"-Wl,-rpath,{tbase}/lib", "-lpthread"]
        run(link)
        os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    print(build(a.force, a.jobs, a.debug, a.verbose))
