"""``.svoc`` checkpoints of a whole :class:`ConsensusService` (engine state + governance).

The byte format is implemented natively (csrc/engine/svoc_io.cpp: CRC-checked typed sections,
atomic rename on write).  Sections follow the field order of the contract ``Storage`` struct
(contract/src/contract.cairo:80-102); wsad integers are widened to i128 and addresses written as
32-byte big-endian felts, so an exact-mode checkpoint carries exactly the contract's values.
Restoring a checkpoint and continuing gives bit-identical results to never having stopped
(tests/test_state.py).
"""
from __future__ import annotations

import json
from typing import Dict

import torch

from . import ops as svops
from .config import ConsensusConfig

FORMAT = "svoc-state/1"


def save(svc, path: str) -> None:
    e, g = svc.engine, svc.gov
    e.pipeline_join()
    D = e.D
    exact = e.mode == "exact"
    num = "i128" if exact else ""
    meta = dict(format=FORMAT, mode=e.mode, batch=e.B, config=svc.cfg.to_dict(),
                value_dtype=str(e.vdtype).replace("torch.", ""), storage=e.storage, rounds=e.rounds)
    secs = [
        ("admins", g.admins, "felt"),
        ("unconstrained_max_spread", torch.tensor([svc.cfg.max_spread_wsad], dtype=torch.int64), "i128"),
        ("oracle_address", g.oracle_addr, "felt"),
        ("enabled", e.enabled, ""),
        ("reliable", e.reliable, ""),
        ("oracles_values", e.values[:, :, :D].to(torch.int64 if exact else e.vdtype).contiguous(), num),
        ("n_active_oracles", e.n_active, ""),
        ("consensus_active", e.consensus_active.to(torch.uint8), ""),
        ("vote_matrix_columns", g.votes, ""),
        ("proposition_tag", g.prop_tag, ""),
        ("proposition_oracle_index", g.prop_idx, ""),
        ("proposition_address", g.prop_addr, "felt"),
        ("consensus_value", e.consensus, num),
        ("consensus_reliability_second_pass", e.rel[:, 1].contiguous(), num),
        ("consensus_reliability_first_pass", e.rel[:, 0].contiguous(), num),
        ("skewness", e.skew, num),
        ("kurtosis", e.kurt, num),
        # engine diagnostics (not contract storage)
        ("essence_first_pass", e.c1, num),
        ("quadratic_risk", e.qr, num),
        ("status", e.status, ""),
        ("touched", e.touched, ""),   # instances whose stored updates still await their round
    ]
    if e.mode == "fast" and e._pending:
        # update batches awaiting their round (transactional steps): the pre-image their revert restores
        e._pending.fold()
        pv, pe, pn = e._pending.dense
        secs += [("pending_pre_values", pv[:, :, :D].contiguous(), ""), ("pending_pre_enabled", pe, ""),
                 ("pending_pre_n_active", pn, ""), ("pending_rows", e._pending.rows.to(torch.uint8), "")]
    svops.ops().save_state(path, json.dumps(meta), [s[0] for s in secs],
                           [s[1].detach().cpu().contiguous() for s in secs], [s[2] for s in secs])


_DTYPE_STORAGE = {"float32": "fp32", "bfloat16": "bf16", "int64": "int64", "int32": "int32"}


def storage_of(meta: dict):
    """Storage name of a checkpoint.  Checkpoints written before the 'storage' key existed carry only
    value_dtype: map it, so an fp32 fast checkpoint is not silently restored at bf16."""
    if meta.get("storage"):
        return meta["storage"]
    return _DTYPE_STORAGE.get(str(meta.get("value_dtype", "")))


def load(path: str, device="cpu"):
    """Rebuild a :class:`svoc.api.ConsensusService` from a checkpoint."""
    from .api import ConsensusService
    meta_s, names, tensors = svops.ops().load_state(path)
    meta = json.loads(meta_s)
    if meta.get("format") != FORMAT:
        raise ValueError("not an svoc-state/1 checkpoint")
    t: Dict[str, torch.Tensor] = dict(zip(names, tensors))
    cfg = ConsensusConfig.from_dict(meta["config"])
    B = int(meta["batch"])
    # placeholder addresses, then the checkpoint's limb tensors copied in directly (no per-instance
    # host conversion: a 1M-instance checkpoint restores in seconds)
    svc = ConsensusService(cfg, B, [0] * cfg.n_admins, [0] * cfg.n_oracles, device=device, mode=meta["mode"],
                           storage=storage_of(meta))
    e, g = svc.engine, svc.gov
    dev = e.device
    if cfg.n_admins:
        g.admins.copy_(t["admins"].to(dev))
    g.oracle_addr.copy_(t["oracle_address"].to(dev))
    g._oracle_cache = None
    e.values[:, :, : e.D].copy_(t["oracles_values"].to(dev, e.vdtype))
    e.enabled.copy_(t["enabled"].to(dev))
    e.reliable.copy_(t["reliable"].to(dev))
    e.n_active.copy_(t["n_active_oracles"].to(dev))
    e._all_active = False   # (the fused streaming path re-checks activation)
    e.consensus_active.copy_(t["consensus_active"].to(dev).bool())
    g.votes.copy_(t["vote_matrix_columns"].to(dev))
    g.prop_tag.copy_(t["proposition_tag"].to(dev))
    g.prop_idx.copy_(t["proposition_oracle_index"].to(dev))
    g.prop_addr.copy_(t["proposition_address"].to(dev))
    e.consensus.copy_(t["consensus_value"].to(dev, e.consensus.dtype))
    e.rel[:, 1].copy_(t["consensus_reliability_second_pass"].to(dev, e.rel.dtype))
    e.rel[:, 0].copy_(t["consensus_reliability_first_pass"].to(dev, e.rel.dtype))
    e.skew.copy_(t["skewness"].to(dev, e.skew.dtype))
    e.kurt.copy_(t["kurtosis"].to(dev, e.kurt.dtype))
    e.c1.copy_(t["essence_first_pass"].to(dev, e.c1.dtype))
    e.qr.copy_(t["quadratic_risk"].to(dev, e.qr.dtype))
    e.status.copy_(t["status"].to(dev))
    e.rounds = int(meta.get("rounds", 0))
    if "touched" in t:
        e.touched.copy_(t["touched"].to(dev))
    if "pending_pre_values" in t and e.mode == "fast":
        pv = e.values.clone()
        pv[:, :, : e.D].copy_(t["pending_pre_values"].to(dev, e.vdtype))
        e._pending.dense = (pv, t["pending_pre_enabled"].to(dev).clone(), t["pending_pre_n_active"].to(dev).clone())
        # (checkpoints from before the row mask: every row of a reverted instance)
        e._pending.rows = (t["pending_rows"].to(dev).bool() if "pending_rows" in t
                           else torch.ones(e.B, e.N, dtype=torch.bool, device=dev))
    return svc
