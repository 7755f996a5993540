"""Native op loader: ``torch.ops.svoc.*`` from the in-tree ``svoc/_C.so``.

The shared object holds the gfx950 HIP kernels (csrc/kernels/*.hip), the bit-exact C++ CPU engines
(csrc/engine) and the torch bindings (csrc/bindings).  There is deliberately no silent fallback: if
the extension is missing on a GPU box every op raises, so a "passing" GPU run can never be a hidden
eager-PyTorch run.  Build with ``python csrc/build.py`` (or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import os
import threading

import torch

_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_C.so")
_lock = threading.Lock()
_loaded = False


class NativeExtensionMissing(RuntimeError):
    pass


def load(build_if_missing: bool = False) -> None:
    """Load ``svoc/_C.so`` into torch.ops (idempotent)."""
    global _loaded
    if _loaded:
        return
    with _lock:
        if _loaded:
            return
        if not os.path.exists(_LIB):
            if build_if_missing:
                from csrc_build import build  # type: ignore  # pragma: no cover
                build()
            else:
                raise NativeExtensionMissing(
                    f"{_LIB} not built: run `python csrc/build.py` (no eager fallback by design)")
        torch.ops.load_library(_LIB)
        _loaded = True


def available() -> bool:
    try:
        load()
        return True
    except Exception:
        return False


def lib_path() -> str:
    return _LIB


def ops():
    load()
    return torch.ops.svoc


from . import torch_ref  # noqa: E402,F401
