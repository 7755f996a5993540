"""felt252 <-> wsad <-> float codecs (the contract ABI value encoding).

* wsad: i128 scaled by 1e6 (contract/src/signed_decimal.cairo:82-83).
* felt252 at the ABI: a negative i128 ``x`` travels as ``P + x`` with the Stark prime
  ``P = 2**251 + 17 * 2**192 + 1`` (client/contract.py:35-53; test_math.cairo:95-97).
* ``float_to_fwsad`` truncates toward zero like ``int(x * 1e6)`` (client/contract.py:48-53), and
  ``fwsad_to_float`` treats any felt above ``2**127 - 1`` as negative (client/contract.py:41-46).

Vectorised versions operate on torch tensors / numpy arrays so the engine can import/export whole
[B, D] batches in one call.
"""
from __future__ import annotations

from typing import Iterable, List, Sequence

import numpy as np
import torch

from .status import ConsensusRevert, Status

WSAD = 1_000_000
FELT_P = 3618502788666131213697322783095070105623107215331596699973092056135872020481  # 2^251+17*2^192+1
I128_MAX = (1 << 127) - 1
I128_MIN = -(1 << 127)


def i128_to_felt(x: int) -> int:
    """``I128SignedBasics::as_felt`` (signed_decimal.cairo:26-28): negative -> P + x."""
    if x < I128_MIN or x > I128_MAX:
        raise ConsensusRevert(Status.OVERFLOW, "not an i128")
    return x + FELT_P if x < 0 else x


def felt_to_i128(f: int) -> int:
    """felt252 -> i128 ``try_into`` (signed_decimal.cairo:47-49): fails outside the i128 range."""
    if not (0 <= f < FELT_P):
        raise ConsensusRevert(Status.FELT_RANGE, "not a felt252")
    x = f - FELT_P if f > FELT_P // 2 else f
    if x < I128_MIN or x > I128_MAX:
        raise ConsensusRevert(Status.FELT_RANGE, "felt252 does not fit in i128")
    return x


def float_to_wsad(x: float) -> int:
    """``int(x * 1e6)``: truncation toward zero (client/contract.py:49)."""
    return int(x * 1e6)


def wsad_to_float(w: int) -> float:
    return float(w) * 1e-6


def float_to_fwsad(x: float) -> int:
    """client/contract.py:48-53."""
    w = float_to_wsad(x)
    return w + FELT_P if w < 0 else w


def fwsad_to_float(f: int) -> float:
    """client/contract.py:41-46."""
    return float((f - FELT_P) if f > I128_MAX else f) * 1e-6


def as_felt(vec: Sequence[int]) -> List[int]:
    """``WsadVector::as_felt`` (math.cairo:20-35)."""
    return [i128_to_felt(int(v)) for v in vec]


def as_wsad(vec: Sequence[int]) -> List[int]:
    """``FeltVector::as_wsad`` (math.cairo:37-50)."""
    return [felt_to_i128(int(v)) for v in vec]


def wsad_to_string(w: int, decimals: int = 6) -> str:
    """``utils.cairo:283-297`` style pretty printer: sign, integer part, fixed decimals."""
    sign = "-" if w < 0 else ""
    a = abs(int(w))
    s = f"{sign}{a // WSAD}.{a % WSAD:06d}"
    return s[: len(s) - (6 - decimals)] if decimals < 6 else s


# ---- batched -----------------------------------------------------------------------------------

def floats_to_wsad_tensor(x) -> torch.Tensor:
    """Vectorised ``int(x * 1e6)`` (truncation toward zero) -> int64 tensor."""
    t = torch.as_tensor(x, dtype=torch.float64)
    return torch.trunc(t * 1e6).to(torch.int64)


def wsad_tensor_to_floats(w: torch.Tensor) -> torch.Tensor:
    return w.to(torch.float64) * 1e-6


def felts_to_wsad_tensor(felts: Iterable[Iterable[int]]) -> torch.Tensor:
    """[[felt]] -> int64 wsad tensor (raises FELT_RANGE / OVERFLOW for values outside int64)."""
    rows = [[felt_to_i128(int(f)) for f in r] for r in felts]
    arr = np.array(rows, dtype=object)
    if arr.size and (max(map(int, arr.ravel())) > np.iinfo(np.int64).max or
                     min(map(int, arr.ravel())) < np.iinfo(np.int64).min):
        raise ConsensusRevert(Status.OVERFLOW, "engine storage is int64 wsad")
    return torch.tensor(rows, dtype=torch.int64)


def wsad_tensor_to_felts(w: torch.Tensor) -> List[List[int]]:
    w = w.detach().cpu()
    if w.dim() == 1:
        return [i128_to_felt(int(v)) for v in w.tolist()]
    return [[i128_to_felt(int(v)) for v in r] for r in w.tolist()]


def address_to_limbs(addr: int) -> List[int]:
    """252-bit address -> 4 little-endian signed 64-bit limbs (device storage of ContractAddress)."""
    if not (0 <= addr < (1 << 256)):
        raise ValueError("address out of range")
    limbs = [(addr >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)]
    return [l - (1 << 64) if l >= (1 << 63) else l for l in limbs]


def limbs_to_address(limbs: Sequence[int]) -> int:
    return sum((int(l) & 0xFFFFFFFFFFFFFFFF) << (64 * i) for i, l in enumerate(limbs))


def shortstring(s: str) -> int:
    """Cairo short string literal ('Akashi') -> felt (big-endian ASCII)."""
    return int.from_bytes(s.encode("ascii"), "big")
