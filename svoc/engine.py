"""Batched consensus engine: B independent reference contracts as device-resident SoA tensors.

One *instance* = one ``OracleConsensusNDS`` contract (contract/src/contract.cairo:38-832).  The state
mirrors its ``Storage`` struct (contract.cairo:80-102) as tensors with a leading batch dimension:

    values[B, N, ld]      oracles_values (bf16 / fp32 in fast mode, int64 wsad in exact mode)
    enabled[B, N]         OracleInfo.enabled          reliable[B, N]   OracleInfo.reliable
    n_active[B]           n_active_oracles            consensus_active[B]
    consensus[B, D]       consensus_value             rel[B, 2]        first / second pass reliability
    skew[B, D], kurt[B, D]

Two numeric modes share one semantics:

* ``exact``: int64 wsad storage (or ``storage="int32"`` for constrained configs: every value is in
  [0, 1e6], half the bytes), the bit-exact HIP kernels -- the column-parallel one
  (csrc/kernels/consensus_wsad.hip) for the rounds it can prove, the i128 one
  (csrc/kernels/consensus_exact.hip) for the rest -- or the C++ CPU engine; updates are transactions
  (a reverted round rolls the update back, exactly like a reverted Starknet tx) and are replayed in
  order per instance.
* ``fast``: fp32 math over bf16 storage (the fused kernels csrc/kernels/consensus_fast_*.hip) or fp32
  storage (``storage="fp32"``: reference resolution, csrc/kernels/consensus_fast_f32.hip).
  Updates inside one step are coalesced (last writer wins) -- exact for the reference because a
  round is a pure function of the current values (survey §2.8-13).  Steps are transactional per
  instance (``transactional=True``, the default): the update kernels save every row they overwrite, and
  a round that reverts restores that instance's rows, ``enabled`` flags and ``n_active`` to their
  pre-batch state and reports the round's code as the status of each of its updates
  (contract.cairo:588-603: the reverted transaction leaves no trace); its consensus outputs stay
  untouched as well.  (Coalescing differs from the reference's one-transaction-per-update replay only
  when a revert happens: the whole batch of that instance reverts.)

Steady-state steps issue no host synchronisation, so they can be captured in a HIP graph.
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Sequence

import numpy as np
import torch

from . import ops as svops
from .config import WSAD, ConsensusConfig
from .status import Status


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


class _PendingBatches:
    """Rollback information of the fast engine's update batches that await their round (transactional steps).

    Each ``apply_updates`` call adds its saved rows / ``enabled`` flags ([U, D] + [U]); the next round restores
    them for the instances it reverts (latest batch first) and gives those updates the round's status.  Many
    batches before one round are folded into one dense pre-image of the state -- ``values``, ``enabled`` and
    ``n_active`` as they were before the first pending batch -- so the memory held stays bounded by one state
    copy (the folded batches keep only their [U] instance / oracle ids and status tensors).  A revert restores
    only the rows (and ``enabled`` flags) the pending batches touched, folded or not, so both forms leave the same
    state: a direct write to other rows of the instance stands.  A checkpoint written while batches are pending
    stores that pre-image (svoc.state), so a round after a reload reverts to the same rows.
    """

    FOLD_AT = 8   # pending batches kept as saved rows before they are folded into the dense pre-image

    def __init__(self, eng: "ConsensusEngine"):
        self.e = eng
        self.entries = []      # (inst, oracle, st, saved, saved_en), batch order
        self.dense = None      # (values, enabled, n_active) before the first folded batch
        self.folded_st = []    # (inst, st) of the folded batches
        self.rows = None       # [B, N] bool: the rows the folded batches touched (restored on a revert)

    def __bool__(self) -> bool:
        return bool(self.entries) or self.dense is not None

    def add(self, inst: torch.Tensor, oracle: torch.Tensor, st: torch.Tensor):
        saved, saved_en, _ = self.e._save_buffer(("pending", len(self.entries)), inst.numel())
        self.entries.append((inst, oracle, st, saved, saved_en))
        return saved, saved_en

    def maybe_fold(self) -> None:
        if len(self.entries) > self.FOLD_AT:
            self.fold()

    def fold(self) -> None:
        """Fold the saved rows of every pending batch into the dense pre-image (one state copy)."""
        e = self.e
        if self.dense is None:
            pv, pe, pn = e.values.clone(), e.enabled.clone(), e.n_active.clone()
            revert_all = torch.full_like(e.status, int(Status.ZERO_VARIANCE))
            every = torch.ones_like(e._active)
            for inst, oracle, st, saved, saved_en in reversed(self.entries):
                e._ops.restore_updates(pv, pe, pn, inst, oracle, st.clone(), saved, saved_en, revert_all, every)
            self.dense = (pv, pe, pn)
        self._mark(self.entries)
        self.folded_st += [(inst, st) for inst, _, st, _, _ in self.entries]
        self.entries = []

    def _mark(self, entries) -> None:
        e = self.e
        if self.rows is None:
            self.rows = torch.zeros(e.B, e.N, dtype=torch.bool, device=e.device)
        for inst, oracle, *_ in entries:
            ok = (inst >= 0) & (inst < e.B) & (oracle >= 0) & (oracle < e.N)
            ic, oc = inst.clamp(0, e.B - 1), oracle.clamp(0, e.N - 1)
            self.rows[ic, oc] = self.rows[ic, oc] | ok

    def restore(self, status: torch.Tensor, active: torch.Tensor) -> None:
        """Roll back the pending batches of the instances whose round ran (``active``) and reverted."""
        e = self.e
        e._all_active = False   # (a reverted first commit lowers n_active: the fused path re-checks)
        if self.dense is None:
            for inst, oracle, st, saved, saved_en in reversed(self.entries):
                e._ops.restore_updates(e.values, e.enabled, e.n_active, inst, oracle, st, saved, saved_en,
                                       status, active)
        else:
            rev = (active != 0) & (status != int(Status.OK))
            pv, pe, pn = self.dense
            self._mark(self.entries)
            # only the rows the pending batches touched go back to the pre-image (the unfolded path's rows)
            m = rev[:, None] & self.rows
            e.values.copy_(torch.where(m[:, :, None], pv, e.values))
            e.enabled.copy_(torch.where(m, pe, e.enabled))
            e.n_active.copy_(torch.where(rev, pn, e.n_active))
            for inst, st in self.folded_st + [(x[0], x[2]) for x in self.entries]:
                ok = (inst >= 0) & (inst < e.B)
                ic = inst.clamp(0, e.B - 1)
                st.copy_(torch.where((st == int(Status.OK)) & ok & rev[ic], status[ic].to(st.dtype), st))
        self.entries, self.dense, self.folded_st, self.rows = [], None, [], None


class ConsensusEngine:
    def __init__(self, cfg: ConsensusConfig, batch: int, device="cuda", mode: str = "fast",
                 storage: Optional[str] = None):
        cfg.validate()
        if mode not in ("fast", "exact"):
            raise ValueError("mode must be 'fast' or 'exact'")
        self.cfg = cfg
        self.B = int(batch)
        self.N = cfg.n_oracles
        self.D = cfg.dimension
        self.mode = mode
        self.device = torch.device(device)
        self._ops = svops.ops()
        B, N, D = self.B, self.N, self.D
        dev = self.device
        if mode == "fast":
            self.vdtype = {"bf16": torch.bfloat16, "fp32": torch.float32}[storage or "bf16"]
            self.ld = _round_up(D, 8)              # 16-B rows for global_load_lds
            odt = torch.float32
        else:
            # constrained values are validated to [0, 1e6] on every update (contract.cairo:591-593), so
            # int32 storage is lossless there (half the bytes of int64); unconstrained wsad stays int64
            default = "int32" if cfg.constrained else "int64"
            self.vdtype = {"int64": torch.int64, "int32": torch.int32}[storage or default]
            if self.vdtype == torch.int32 and not cfg.constrained:
                raise ValueError("int32 wsad storage is for constrained configs (values in [0, 1e6])")
            self.ld = D
            odt = torch.int64
        self.storage = {torch.bfloat16: "bf16", torch.float32: "fp32", torch.int64: "int64",
                        torch.int32: "int32"}[self.vdtype]
        self.values = torch.zeros(B, N, self.ld, dtype=self.vdtype, device=dev)
        self.enabled = torch.zeros(B, N, dtype=torch.uint8, device=dev)
        self.n_active = torch.zeros(B, dtype=torch.int32, device=dev)
        self.reliable = torch.ones(B, N, dtype=torch.uint8, device=dev)   # constructor: reliable=true
        self.consensus_active = torch.zeros(B, dtype=torch.bool, device=dev)
        self.c1 = torch.zeros(B, D, dtype=odt, device=dev)
        self.consensus = torch.zeros(B, D, dtype=odt, device=dev)
        self.skew = torch.zeros(B, D, dtype=odt, device=dev)
        self.kurt = torch.zeros(B, D, dtype=odt, device=dev)
        self.rel = torch.zeros(B, 2, dtype=odt, device=dev)
        self.qr = torch.zeros(B, N, dtype=odt, device=dev)
        self.status = torch.full((B,), int(Status.NOT_ACTIVE), dtype=torch.int32, device=dev)
        self.touched = torch.zeros(B, dtype=torch.uint8, device=dev)
        self._winner = torch.full((B, N), -1, dtype=torch.int32, device=dev)
        self._active = torch.zeros(B, dtype=torch.uint8, device=dev)
        self.wave_hint = 0
        self.rounds = 0
        self.failing_mask: Optional[torch.Tensor] = None   # [B, N] set by randomize()
        self._work = None   # window-kernel workspace (GPU fast mode), allocated on first use
        # transactional fast steps: the rows each apply_updates call overwrote, restored by the next round
        # for the instances whose round reverts (engine docstring)
        self.transactional = mode == "fast"
        # pruned window network (fp32, N = 256): slab networks that failed the exact check and reran the
        # full network, counted by the kernel (net_stats)
        self._net_fb = torch.zeros(1, dtype=torch.int32, device=dev) if (mode == "fast" and dev.type == "cuda") else None
        # exact rounds on the GPU: [rounds committed by the wide-column unconstrained kernel, rounds handed to the
        # i128 kernel] (consensus_wsadx.hip; exact_routing)
        self._xstats = torch.zeros(2, dtype=torch.int32, device=dev) if (mode == "exact" and dev.type == "cuda") else None
        self._pending = _PendingBatches(self)
        self._save_bufs: Dict[tuple, tuple] = {}
        # health counters folded in by every round's epilogue: [rel2 sum (2^-32 units fast / wsad
        # exact), committed, processed, reverted]
        self.metrics_fx = torch.zeros(4, dtype=torch.int64, device=dev)

    # ------------------------------------------------------------------ sizing
    @staticmethod
    def bytes_per_instance(n: int, d: int, mode: str = "fast", storage: Optional[str] = None) -> int:
        """HBM bytes of state per instance (survey §7.6 sizing).  ``storage``: the value dtype
        ("bf16" / "fp32" fast, "int64" / "int32" exact; default bf16 fast, int64 exact); the legacy
        mode name "exact32" means exact with int32 storage."""
        if mode == "exact32":
            mode, storage = "exact", storage or "int32"
        s = {"bf16": 2, "fp32": 4, "int64": 8, "int32": 4}[storage or ("bf16" if mode == "fast" else "int64")]
        o = 4 if mode == "fast" else 8
        ld = _round_up(d, 8) if mode == "fast" else d
        return n * ld * s + 4 * d * o + n * (1 + 1 + o + 4) + 2 * o + 4 + 4 + 2

    def state_bytes_per_instance(self) -> int:
        """bytes_per_instance for this engine's own mode and storage dtype."""
        return self.bytes_per_instance(self.N, self.D, self.mode, self.storage)

    # ------------------------------------------------------------------ updates
    def _as_storage(self, vals: torch.Tensor) -> torch.Tensor:
        if self.mode == "exact":
            if vals.dtype.is_floating_point:
                raise TypeError("exact mode takes int64 wsad values (use svoc.codec.float_to_wsad)")
            v = vals.to(self.device, torch.int64)
            if self.vdtype == torch.int32:   # out of int32 -> -1: rejected by the interval check, not wrapped
                v = torch.where((v < -(2 ** 31)) | (v >= 2 ** 31), torch.full_like(v, -1), v)
            return v.to(self.vdtype).contiguous()
        return vals.to(self.device, self.vdtype).contiguous()

    def apply_updates(self, inst: torch.Tensor, oracle: torch.Tensor, vals: torch.Tensor,
                      unique: bool = False, _joined: bool = False, save=None) -> torch.Tensor:
        """Store a batch of predictions (no consensus). Returns the per-update status [U] (device).

        ``unique=True``: the caller guarantees distinct (instance, oracle) pairs in the batch, so the GPU
        validates and stores in one pass (no last-writer resolution)."""
        inst = torch.as_tensor(inst, dtype=torch.int64, device=self.device).contiguous()
        oracle = torch.as_tensor(oracle, dtype=torch.int64, device=self.device).contiguous()
        if not _joined:
            # (streams only: a pending D-shard round's commit writes outputs, not the stored rows, and
            # its pass 2 has already read them -- updates may land before it)
            self._join_streams()
            if self.transactional and getattr(self, "_dshard_pending", None) is not None:
                # ... unless the pending round's reverted instances must roll their rows back: its verdict
                # (one status all-reduce) and the restore come first, then this batch lands on the
                # restored rows (svoc.parallel.dshard, deferred rounds)
                self.pipeline_join()
        vals = self._as_storage(torch.as_tensor(vals))
        if vals.dim() != 2 or vals.shape[1] != self.D:
            raise ValueError(f"predictions must be [U, {self.D}]")
        saved = saved_en = None
        if save is not None:      # (saved rows, saved enabled flags, status out) of step_pipelined
            saved, saved_en, st = save
        else:
            st = torch.empty(inst.numel(), dtype=torch.int32, device=self.device)
            if self.transactional:
                saved, saved_en = self._pending.add(inst, oracle, st)
        self._ops.apply_updates(self.values, self.enabled, self.n_active, self.touched, self._winner,
                                inst, oracle, vals, self.cfg.constrained, st, bool(unique), saved, saved_en)
        if save is None and self.transactional:
            self._pending.maybe_fold()
        return st

    def _save_buffer(self, key, U: int):
        """Reusable [U, D] / [U] save buffers of the transactional update path (stable across steps, so
        a captured HIP graph replays into the same memory)."""
        buf = self._save_bufs.get(key)
        if buf is None or buf[0].shape[0] < U:
            buf = (torch.empty(U, self.D, dtype=self.vdtype, device=self.device),
                   torch.empty(U, dtype=torch.uint8, device=self.device),
                   torch.empty(U, dtype=torch.int32, device=self.device))
            self._save_bufs[key] = buf
        return buf[0][:U], buf[1][:U], buf[2][:U]

    def _restore(self, entries, status=None) -> None:
        """Roll back the saved updates of the instances whose round ran and reverted (latest batch first)."""
        status = self.status if status is None else status
        self._all_active = False   # (a reverted first commit lowers n_active: the fused path re-checks)
        for inst, oracle, st, saved, saved_en in reversed(entries):
            self._ops.restore_updates(self.values, self.enabled, self.n_active, inst, oracle, st, saved, saved_en,
                                      status, self._active)

    def _restore_pending(self, status=None) -> None:
        if self._pending:
            self._pending.restore(self.status if status is None else status, self._active)

    # ------------------------------------------------------------------ rounds
    def run_round(self, only_touched: bool = True) -> None:
        """Consensus round for every instance that is fully active (and touched, by default).

        Three launches: the prologue selects the instances (n_active == N, touched), the fused
        round kernel, and the epilogue commits consensus_active, clears touched and folds the
        round's health counters into :attr:`metrics_fx` (integers: deterministic sums)."""
        self.pipeline_join()
        self._ops.round_prologue(self.n_active, self.touched, self.N, bool(only_touched), self._active)
        mx = self.cfg.unconstrained_max_spread
        if self.mode == "fast":
            self._ops.fast_round(self.values, self._active, self.D, self.cfg.n_failing_oracles,
                                 self.cfg.constrained, float(mx), self.c1, self.consensus, self.skew,
                                 self.kurt, self.rel, self.qr, self.reliable, self.status, self.wave_hint,
                                 0, 0, self.cfg.legacy, self.work(), self._net_fb)
            self._restore_pending()
        else:
            self._ops.exact_round(self.values, self._active, self.cfg.n_failing_oracles, self.cfg.constrained,
                                  self.cfg.max_spread_wsad, self.c1, self.consensus, self.skew, self.kurt,
                                  self.rel, self.qr, self.reliable, self.status, self.cfg.legacy,
                                  stats=self._xstats)
        self._ops.round_epilogue(self._active, self.status, self.rel, self.consensus_active, self.touched,
                                 self.metrics_fx)
        self.rounds += 1

    def _run_round_range(self, b0: int, b1: int, only_touched: bool = True, restore=None, U: int = 0) -> None:
        """run_round over instances [b0, b1) only (views of the state; fast mode); ``restore``: the
        range's saved update batch (inst, oracle, st, saved, saved_en), rolled back where it reverted --
        by the round kernel itself when ``U`` (updates per instance, instance-grouped) is given and the
        kernel supports it (:meth:`_kernel_rollback_ok`), else by the restore kernel after it."""
        sl = slice(b0, b1)
        self._ops.round_prologue(self.n_active[sl], self.touched[sl], self.N, bool(only_touched), self._active[sl])
        w = self.work()
        if w is not None:
            words = w.numel() // self.B
            w = w[b0 * words:b1 * words]
        args = (self.values[sl], self._active[sl], self.D, self.cfg.n_failing_oracles,
                self.cfg.constrained, float(self.cfg.unconstrained_max_spread), self.c1[sl],
                self.consensus[sl], self.skew[sl], self.kurt[sl], self.rel[sl], self.qr[sl],
                self.reliable[sl], self.status[sl], self.wave_hint, 0, 0, self.cfg.legacy, w, self._net_fb)
        if restore is not None and U > 0:
            _, oracle, st, saved, saved_en = restore
            self._all_active = False   # (a reverted first commit lowers n_active)
            self._ops.fast_round(*args, None, oracle.contiguous(), st, U, saved, saved_en, self.enabled[sl],
                                 self.n_active[sl])
        else:
            self._ops.fast_round(*args)
            if restore is not None:
                self._restore([restore])
        self._ops.round_epilogue(self._active[sl], self.status[sl], self.rel[sl], self.consensus_active[sl],
                                 self.touched[sl], self.metrics_fx)

    def _kernel_rollback_ok(self, U: int) -> bool:
        """Whether the round kernel itself rolls back a reverted instance's saved batch (FastParams.rst_saved):
        the bf16 window kernel -- whole constrained rounds, 16 < N <= 256 (or D > 128: not the small-instance
        kernel), f <= 32 with a window, U updates per instance."""
        f = self.cfg.n_failing_oracles
        if os.environ.get("SVOC_KERNEL_ROLLBACK", "1") == "0":   # (A/B: the restore kernel instead)
            return False
        return (self.mode == "fast" and self.device.type == "cuda" and self.vdtype == torch.bfloat16
                and self.cfg.constrained and not self.cfg.legacy and self.wave_hint == 0
                and 2 <= self.N <= 256 and (self.N > 16 or self.D > 128) and 0 <= f <= 32 and f <= self.N - 2
                and bool(svops.fast_win_h(self.N, f)) and self.work() is not None and 0 < U)

    def _fused_ok(self, inst, oracle, vals, U: int) -> bool:
        """Whether a pipelined step can take the fused transactional path: fp32 storage on the GPU, whole
        constrained rounds through the window kernel (N <= 256, f <= 32), at most 256 updates per instance
        (instance-grouped batch, as step_pipelined requires), fp32 rows of exactly D columns, and every
        instance already active (the fused round covers no activation; checked once, then tracked).
        (bf16 storage takes the generic path: the same fusion in the bf16 window kernel measured slower than
        saving the rows, profiles/r4_c3_bf16_txn_ab.txt.)"""
        if os.environ.get("SVOC_FUSED_TXN", "1") == "0":   # (A/B: the generic path instead)
            return False
        if not (self.mode == "fast" and self.device.type == "cuda" and self.vdtype == torch.float32
                and self.cfg.constrained and 2 <= self.N <= 256 and 0 <= self.cfg.n_failing_oracles <= 32
                and self.cfg.n_failing_oracles <= self.N - 2 and svops.fast_win_h(self.N, self.cfg.n_failing_oracles)
                and 0 < U <= 256 and vals.dtype == self.vdtype and vals.dim() == 2 and vals.shape[1] == self.D
                and oracle.dtype == torch.int64 and not self.cfg.legacy
                # (the kernel's 32-bit batch offsets and 24-bit row-offset multiplies: svoc_fast_round_f32_win)
                and U * self.D * 4 < (1 << 31) and self.ld * 4 < (1 << 24)):
            return False
        if not getattr(self, "_all_active", False):
            if torch.cuda.is_current_stream_capturing():
                return False
            self._all_active = bool((self.n_active == self.N).all())
        return self._all_active

    def _status_buffer(self, U: int) -> torch.Tensor:
        buf = self._save_bufs.get(("st",))
        if buf is None or buf.shape[0] < U:
            buf = torch.empty(U, dtype=torch.int32, device=self.device)
            self._save_bufs[("st",)] = buf
        return buf[:U]

    def _run_round_range_fused(self, b0: int, b1: int, oracle: torch.Tensor, rows: torch.Tensor, st: torch.Tensor,
                               U: int) -> None:
        """Fused transactional round over instances [b0, b1): every instance is active and each has U
        updates (rows b * U ..); the window kernel reads the updated rows from `rows`, writes each update's
        transaction status to `st`, and the commit kernel stores the accepted rows (a reverted round's rows
        never reach the state)."""
        sl = slice(b0, b1)
        self._ops.round_prologue(self.n_active[sl], self.touched[sl], self.N, False, self._active[sl])
        w = self.work()
        words = w.numel() // self.B
        w = w[b0 * words:b1 * words]
        self._ops.fast_round(self.values[sl], self._active[sl], self.D, self.cfg.n_failing_oracles,
                             self.cfg.constrained, float(self.cfg.unconstrained_max_spread), self.c1[sl],
                             self.consensus[sl], self.skew[sl], self.kurt[sl], self.rel[sl], self.qr[sl],
                             self.reliable[sl], self.status[sl], self.wave_hint, 0, 0, self.cfg.legacy, w,
                             self._net_fb, rows, oracle.contiguous(), st, U)
        self._ops.commit_updates(rows, oracle, st, self.values[sl], U)
        self._ops.round_epilogue(self._active[sl], self.status[sl], self.rel[sl], self.consensus_active[sl],
                                 self.touched[sl], self.metrics_fx)

    def step_pipelined(self, inst: torch.Tensor, oracle: torch.Tensor, vals: torch.Tensor,
                       updates_per_instance: int, chunks: int = 2, overlap: bool = False) -> None:
        """apply_updates(unique=True) + run_round, pipelined over ``chunks`` instance ranges on HIP streams.

        The update scatter is HBM-bound and the round kernel VALU-bound, so they overlap: the updates of
        range k+1 (one update stream, in order) run while the round of range k runs on its own stream.
        The batch must be grouped by instance, ``updates_per_instance`` distinct oracles per instance in
        instance order (SyntheticUpdateStream's layout).  Same results as ``apply_updates(...,
        unique=True); run_round()`` (ranges are disjoint instances).  GPU fast mode only;
        graph-capturable (fork/join through stream waits / events).

        ``overlap=True`` also overlaps consecutive steps: every range runs on its own stream (its update,
        then its round), the streams are not joined back at the end, so the next call's update of range
        k queues behind this call's round of range k (the one kernel that reads those rows) and runs
        beside the other ranges' rounds.  The engine is then "open": :meth:`pipeline_join` (called by
        every other engine method) joins the streams into the current stream before anything else
        touches the state."""
        U = int(updates_per_instance)
        # the batch goes to kernels that dereference it directly (the fused round, the commit and restore
        # kernels): indices as int64 and rows in the storage dtype, all on the state's device
        inst = torch.as_tensor(inst, dtype=torch.int64, device=self.device).reshape(-1).contiguous()
        oracle = torch.as_tensor(oracle, dtype=torch.int64, device=self.device).reshape(-1).contiguous()
        vals = self._as_storage(torch.as_tensor(vals))
        # (a lone apply_updates before this step is still awaiting its round: one round must cover both)
        if self.mode != "fast" or self.device.type != "cuda" or chunks <= 1 or self._pending:
            self.pipeline_join()
            self.apply_updates(inst, oracle, vals, unique=True)
            self.run_round()
            return
        if inst.numel() != self.B * U:
            raise ValueError("step_pipelined: expects updates_per_instance updates for every instance")
        cur = torch.cuda.current_stream(self.device)
        if getattr(self, "_pipe_streams", None) is None or len(self._pipe_streams) != chunks + 1:
            self.pipeline_join()
            self._pipe_streams = [torch.cuda.Stream(self.device) for _ in range(chunks + 1)]
        su, sc = self._pipe_streams[0], self._pipe_streams[1:]
        step = (self.B + chunks - 1) // chunks
        ranges = [(k * step, min(self.B, (k + 1) * step)) for k in range(chunks) if k * step < self.B]
        # fused transactional streaming (fp32 window kernel): the round reads the updated rows from the batch
        # and a commit kernel copies the accepted ones -- no saved copy, no restore (_fused_ok)
        fused = self.transactional and self._fused_ok(inst, oracle, vals, U)
        kroll = self.transactional and not fused and self._kernel_rollback_ok(U)
        # per-step buffers live in the engine (the side streams use them after this returns): saved rows,
        # saved enabled flags and the update statuses, one slice per range
        if fused:
            sv_all = sen_all = None
            st_all = self._status_buffer(inst.numel())
            vals = vals.contiguous()
        else:
            sv_all, sen_all, st_all = (self._save_buffer(("pipe",), inst.numel()) if self.transactional
                                       else (None,) * 3)

        def upd(k, b0, b1):
            sl = slice(b0 * U, b1 * U)
            if fused:
                return   # (the round reads the batch; the commit after it stores the accepted rows)
            if self.transactional:
                self.apply_updates(inst[sl], oracle[sl], vals[sl], unique=True, _joined=True,
                                   save=(sv_all[sl], sen_all[sl], st_all[sl]))
            else:
                self.apply_updates(inst[sl], oracle[sl], vals[sl], unique=True, _joined=True)

        def rnd(k, b0, b1):
            sl = slice(b0 * U, b1 * U)
            if fused:
                self._run_round_range_fused(b0, b1, oracle[sl], vals[sl], st_all[sl], U)
                return
            rest = (inst[sl], oracle[sl], st_all[sl], sv_all[sl], sen_all[sl]) if self.transactional else None
            self._run_round_range(b0, b1, restore=rest, U=U if (rest is not None and kroll) else 0)
        if overlap:
            # range k lives on stream sc[k] alone (update, then round; the next step's update of range k
            # queues behind this round on the same stream: no cross-stream waits).  The streams start
            # staggered by one update (sc[k] waits for range k-1's update once, after a join), so each
            # range's update runs beside another range's round, also across steps.
            fresh = not getattr(self, "_pipe_open", False)
            for k, (b0, b1) in enumerate(ranges):
                sc[k].wait_stream(cur)
                if fresh and k > 0:
                    sc[k].wait_stream(sc[k - 1])     # holds only range k-1's update at this point
                with torch.cuda.stream(sc[k]):
                    upd(k, b0, b1)
            for k, (b0, b1) in enumerate(ranges):
                with torch.cuda.stream(sc[k]):
                    rnd(k, b0, b1)
            # the side streams still read the caller's batch after this returns: hold it until the join
            # (after which the current stream is ordered behind every read, so the caching allocator may
            # hand its blocks out again)
            held = getattr(self, "_pipe_held", None) or []
            held.append((inst, oracle, vals))
            self._pipe_held = held
            self.rounds += 1
            self._pipe_open = True
            return
        su.wait_stream(cur)
        for k, (b0, b1) in enumerate(ranges):
            with torch.cuda.stream(su):
                upd(k, b0, b1)
            sc[k].wait_stream(su)
            with torch.cuda.stream(sc[k]):
                rnd(k, b0, b1)
        self.rounds += 1
        for s in self._pipe_streams:
            cur.wait_stream(s)

    def pipeline_join(self) -> None:
        """Join the streams of an open (``overlap=True``) pipelined step into the current stream, and
        commit a deferred D-sharded round (svoc.parallel.dshard, ``defer=True``): every reader of the
        state (getters, metrics, checkpoints, the next update) goes through here.  With a D-shard round
        pending this is a collective (one status all-reduce): every rank of the shard group must read."""
        self._join_streams()
        if getattr(self, "_dshard_pending", None) is not None:
            from .parallel.dshard import flush_sharded
            group, world = self._dshard_ctx
            flush_sharded(self, group=group, world=world)

    def _join_streams(self) -> None:
        if getattr(self, "_pipe_open", False):
            cur = torch.cuda.current_stream(self.device)
            for s in self._pipe_streams:
                cur.wait_stream(s)
            self._pipe_open = False
            self._pipe_held = None

    def work(self) -> Optional[torch.Tensor]:
        """Workspace of the one-network window kernel (34 window keys + 8 power sums + 2 cleanup
        list slots per column pair: 176 B per column pair and instance); None where that kernel does not run (CPU, small
        instances, more than 32 failing oracles)."""
        if self.mode != "fast" or self.device.type != "cuda":
            return None
        if self.vdtype == torch.bfloat16 and not svops.fast_work_applies(self.N, self.D, self.cfg.n_failing_oracles):
            return None   # (the fp32 kernel always stages its pass-2 outputs there)
        if self._work is None:
            self._work = torch.empty(svops.fast_work_numel(self.B, self.D), dtype=torch.int32,
                                     device=self.device)
        return self._work

    def net_stats(self) -> Dict[str, int]:
        """Pruned window network counters (fp32 storage, N = 256; sortnet.hpp window_group_pruned):
        ``slab_networks`` run so far (processed rounds x full 64-column slab steps x 4 waves) and the
        ``fallbacks`` among them whose exact check failed (the full network reran for that wave)."""
        self.pipeline_join()
        if self._net_fb is None or not svops.pruned_window_applies(self.N, self.cfg.n_failing_oracles,
                                                                  self.cfg.constrained, self.storage):
            return {"slab_networks": 0, "fallbacks": 0}
        processed = int(self.metrics_fx[2].item())
        return {"slab_networks": processed * (self.D // 64) * 4, "fallbacks": int(self._net_fb.item())}

    def exact_routing(self) -> Dict[str, int]:
        """Exact engine on the GPU: how the rounds so far were computed -- ``processed`` rounds, of which
        ``wide_column`` committed by the int64 wide-column kernel (unconstrained columns spread past 2^30 wsad,
        consensus_wsadx.hip) and ``i128`` handed to the i128 kernel (out of every column kernel's domain, or
        reverting where the wide-column kernel cannot name the status); the rest ran on the column kernel."""
        self.pipeline_join()
        processed = int(self.metrics_fx[2].item())
        if self._xstats is None:
            return {"processed": processed, "wide_column": 0, "i128": 0}
        x = self._xstats.tolist()
        return {"processed": processed, "wide_column": int(x[0]), "i128": int(x[1])}

    def metrics(self) -> torch.Tensor:
        """[sum rel2 of committed rounds, committed, processed, reverted] as float64 (device)."""
        self.pipeline_join()
        m = self.metrics_fx.double()
        m[0] *= (2.0 ** -32) if self.mode == "fast" else 1e-6
        return m

    def step(self, inst, oracle, vals, updates_per_instance: Optional[int] = None) -> torch.Tensor:
        """update_prediction for a batch of (instance, oracle, prediction) + the consensus rounds.

        fast: one coalesced round per touched instance.  exact: per-instance sequential
        transactions (a reverted round restores that update's previous row).
        ``updates_per_instance=K`` (exact): the batch is laid out as K updates of every instance in
        instance order (update b * K + k is instance b's k-th; SyntheticUpdateStream's layout), so
        the transaction waves are strided views: no host synchronisation at all (graph-capturable).
        That layout is trusted, as in :meth:`step_pipelined` (an instance twice in one wave breaks the
        sequential order); any other batch goes through the general device-side grouping."""
        self.pipeline_join()
        if self.mode == "fast":
            st = self.apply_updates(inst, oracle, vals)
            self.run_round()
            return st
        return self._exact_transactions(inst, oracle, vals, updates_per_instance)

    def _transaction_waves(self, inst: torch.Tensor, oracle: torch.Tensor):
        """Device-side grouping of a batch into transaction waves: wave k = the k-th valid update of every
        instance (batch order kept per instance).  Returns (order, bounds): the update indices sorted by
        (wave, batch index) and the host list of wave boundaries -- the one device->host copy (K + 1
        integers), before any wave is issued."""
        U = inst.numel()
        idx = torch.arange(U, device=self.device)
        ok = (inst >= 0) & (inst < self.B) & (oracle >= 0) & (oracle < self.N)
        key = torch.where(ok, inst, torch.full_like(inst, self.B))
        by_inst = torch.sort(key * U + idx).indices                 # grouped by instance, batch order
        sk = key[by_inst]
        first = torch.searchsorted(sk, sk)                          # first position of the own instance
        occ = torch.empty_like(idx)
        occ[by_inst] = torch.arange(U, device=self.device) - first  # rank within the instance
        occ = torch.where(ok, occ, torch.full_like(occ, U))          # invalid updates: after every wave
        order = torch.sort(occ * U + idx).indices
        counts = torch.bincount(occ, minlength=U + 1)[:U].cpu()      # updates per wave (host, once)
        n_waves = int(torch.count_nonzero(counts))
        bounds = [0] + torch.cumsum(counts[:n_waves], 0).tolist()
        return order, bounds

    def _exact_transactions(self, inst, oracle, vals, updates_per_instance: Optional[int] = None) -> torch.Tensor:
        """Sequential per-update transactions (contract.cairo:588-603: update_prediction stores the row,
        then the full consensus round; a round that fails reverts the whole transaction), replayed as
        waves: wave k applies the k-th update of every instance at once -- instances are independent,
        so this is the per-instance sequential order.  Everything stays on the device: per wave one
        gather of the old rows, the batched store, the round over the touched instances and a masked
        restore for the transactions whose round failed."""
        inst = torch.as_tensor(inst, dtype=torch.int64, device=self.device).reshape(-1)
        oracle = torch.as_tensor(oracle, dtype=torch.int64, device=self.device).reshape(-1)
        vals = self._as_storage(torch.as_tensor(vals))
        U = inst.numel()
        out = torch.full((U,), int(Status.NOT_ORACLE), dtype=torch.int32, device=self.device)
        if U == 0:
            return out
        K = int(updates_per_instance or 0)
        if K:
            if U % K:
                raise ValueError("_exact_transactions: updates_per_instance must divide the batch")
            if U > self.B * K:
                raise ValueError("_exact_transactions: more than updates_per_instance updates per instance")
            capturing = self.device.type == "cuda" and torch.cuda.is_current_stream_capturing()
            if not capturing:
                # outside graph capture the b * K + k layout is checked (one host sync); a batch that does
                # not follow it (an instance twice in a wave) takes the general device-side grouping
                okl = (inst >= 0) & (inst < self.B) & (oracle >= 0) & (oracle < self.N)
                lay = inst == torch.arange(U, device=self.device) // K
                if not bool((lay | ~okl).all()):
                    K = 0
            if K and self.device.type == "cuda":
                return self._exact_transactions_k(inst, oracle, vals, K, out)
            waves = [torch.arange(k, U, K, device=self.device) for k in range(K)]
        else:
            order, bounds = self._transaction_waves(inst, oracle)
            waves = [order[bounds[k]:bounds[k + 1]] for k in range(len(bounds) - 1)]
            if bounds[-1] < U:   # unknown instance / oracle: status only (interval check first), no store
                bad = order[bounds[-1]:]
                out[bad] = self.apply_updates(inst[bad], oracle[bad], vals[bad])
        for sel in waves:
            bi, oi = inst[sel], oracle[sel]
            if K:
                # out-of-range entries (status NOT_ORACLE, never applied) point their no-op gathers and
                # write-backs at their own layout slot (instance sel // K): with one entry per instance
                # per wave they cannot collide with another entry's restore.  (The general path drops
                # them in _transaction_waves.)
                okw = (bi >= 0) & (bi < self.B) & (oi >= 0) & (oi < self.N)
                bi_c = torch.where(okw, bi, sel // K)
                oi_c = torch.where(okw, oi, torch.zeros_like(oi))
            else:
                okw, bi_c, oi_c = None, bi, oi
            old_rows = self.values[bi_c, oi_c].clone()
            old_en = self.enabled[bi_c, oi_c].clone()
            old_na = self.n_active[bi_c].clone()
            self.touched.zero_()
            st_u = self.apply_updates(bi, oi, vals[sel])
            self.run_round(only_touched=True)        # outputs are only written when a round succeeds
            st_b = self.status[bi_c]
            full = self.n_active[bi_c] == self.N
            tx = torch.where(st_u != 0, st_u,
                             torch.where(full, st_b, torch.full_like(st_b, int(Status.NOT_ACTIVE))))
            revert = (st_u == 0) & full & (st_b != int(Status.OK))
            if okw is not None:
                revert = revert & okw
            # roll back reverted transactions (contract semantics: the whole tx disappears)
            self.values[bi_c, oi_c] = torch.where(revert[:, None], old_rows, self.values[bi_c, oi_c])
            self.enabled[bi_c, oi_c] = torch.where(revert, old_en, self.enabled[bi_c, oi_c])
            self.n_active[bi_c] = torch.where(revert, old_na, self.n_active[bi_c])
            out[sel] = tx
        return out

    def _exact_transactions_k(self, inst, oracle, vals, K: int, out: torch.Tensor) -> torch.Tensor:
        """_exact_transactions for the b * K + k layout on the GPU, with the transaction bookkeeping in the update
        and restore kernels: per wave the update kernel validates, saves the overwritten row / ``enabled`` flag
        and stores (one launch), the round runs, and the restore kernel rolls back the transactions whose round
        reverted and gives every applied update its transaction status -- the round's code, NOT_ACTIVE where the
        instance is not fully active (the update stays stored), OK otherwise.  The per-wave gathers, compares,
        ``where`` selects and scatters of the general path (~20 small kernels, ~10 % of a c3 wave) go away; the
        batch is reordered wave-major once."""
        n = inst.numel() // K
        iw = inst.view(n, K).t().contiguous()                 # [K, n]: wave k = the k-th update of every instance
        ow = oracle.view(n, K).t().contiguous()
        vw = vals.reshape(n, K, -1).transpose(0, 1).contiguous()
        sw = torch.empty(K, n, dtype=torch.int32, device=self.device)
        sv, sen, _ = self._save_buffer(("exact_tx",), n)
        for k in range(K):
            self.touched.zero_()
            self.apply_updates(iw[k], ow[k], vw[k], unique=True, save=(sv, sen, sw[k]))
            self.run_round(only_touched=True)                 # outputs are only written when a round succeeds
            self._ops.restore_updates(self.values, self.enabled, self.n_active, iw[k], ow[k], sw[k], sv, sen,
                                      self.status, self._active, int(Status.NOT_ACTIVE))
        out.copy_(sw.t().reshape(-1))
        return out

    # ------------------------------------------------------------------ synthetic data
    def randomize(self, seed: int = 0, a: float = 20.0, failing_low: float = 0.0) -> None:
        """Fill every oracle of every instance (Beta(a,a) honest, U(0,1) failing), all enabled.  The
        [B, N] failing set is kept in :attr:`failing_mask` (a synthetic update stream that keeps the same
        oracles failing: SyntheticUpdateStream(failing=...))."""
        self.pipeline_join()
        from .models.oracle_gen import beta_failing_oracles
        g = torch.Generator(device=self.device).manual_seed(seed)
        x, self.failing_mask = beta_failing_oracles(self.B, self.N, self.D, self.cfg.n_failing_oracles, a, g,
                                                    self.device, return_mask=True)
        if self.mode == "exact":
            self.values[:, :, : self.D] = (x.double() * WSAD).to(torch.int64).to(self.vdtype)
        else:
            self.values[:, :, : self.D] = x.to(self.vdtype)
        self.enabled.fill_(1)
        self.n_active.fill_(self.N)
        self.touched.fill_(1)
        self._all_active = True

    # ------------------------------------------------------------------ getters (contract ABI names)
    def get_consensus_value(self, i: Optional[int] = None) -> torch.Tensor:
        self.pipeline_join()
        return self.consensus if i is None else self.consensus[i]

    def get_first_pass_consensus_reliability(self, i: Optional[int] = None):
        self.pipeline_join()
        return self.rel[:, 0] if i is None else self.rel[i, 0]

    def get_second_pass_consensus_reliability(self, i: Optional[int] = None):
        self.pipeline_join()
        return self.rel[:, 1] if i is None else self.rel[i, 1]

    def get_skewness(self, i: Optional[int] = None):
        self.pipeline_join()
        return self.skew if i is None else self.skew[i]

    def get_kurtosis(self, i: Optional[int] = None):
        self.pipeline_join()
        return self.kurt if i is None else self.kurt[i]

    def get_reliability(self) -> torch.Tensor:
        """North-star alias: [B, 2] (first pass, second pass)."""
        self.pipeline_join()
        return self.rel

    get_consensus = get_consensus_value

    def get_predictions_dimension(self) -> int:
        self.pipeline_join()
        return self.D

    def get_oracle_value_list(self, i: int):
        self.pipeline_join()
        return (self.values[i, :, : self.D], self.enabled[i].bool(), self.reliable[i].bool())
