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


def fast_work_words(D: int) -> int:
    """u32 words per instance of the window kernel's workspace (csrc/include/svoc/launch.hpp)."""
    pairs = ((D + 1) // 2 + 255) // 256 * 256
    return pairs * 2 * (2 * 17 + 4 + 1 + 3)   # fp32 window layout (the larger of the two)


def fast_work_numel(B: int, D: int) -> int:
    """Total int32 elements of the window kernel's workspace (B instances)."""
    return B * fast_work_words(D)


def fast_work_applies(N: int, D: int, n_failing: int) -> bool:
    """Whether the default GPU fast round needs the workspace: every kernel but the small-instance
    one (N <= 16 and D <= 128) keeps its window state and staged pass-2 outputs there."""
    return N > 16 or D > 128



def fast_win_h(N: int, f: int) -> int:
    """Window half-width of the one-network kernels (launch.hpp fast_win_h): 5, 17, or 0 (no window)."""
    R = N - f
    a = N // 2 - R // 2
    if a + 1 <= 5 and f - a + 1 <= 5:
        return 5
    if a + 1 <= 17 and f - a + 1 <= 17:
        return 17
    return 0


def pruned_window_applies(N: int, n_failing: int, constrained: bool, storage: str) -> bool:
    """The fp32 window kernel's pruned network runs (N = 256, H = 17, constrained; csrc/kernels/
    consensus_fast_winf.hip + sortnet.hpp window_group_pruned) -- on every full 64-column slab step."""
    return storage == "fp32" and constrained and N == 256 and 0 <= n_failing <= 32 and fast_win_h(N, n_failing) == 17
