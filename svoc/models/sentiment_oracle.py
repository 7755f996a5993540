"""Sentiment-oracle path: comments -> encoder -> go_emotions scores -> stochastic oracles -> consensus.

One *window* of C = 30 comments feeds one consensus instance (the reference's fetch:
client/oracle_scheduler.py:155-161 = read window -> classify -> gen_oracles_predictions).  The
encoder runs as one batched bf16 forward over all windows; the oracle bootstrap (failing oracles
U(0,1)^6, honest ones = mean of 10-of-30 comment vectors, shuffled) is one fused HIP kernel
(csrc/kernels/oracle_gen.hip) writing straight into the engine's update batch.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from .. import ops as svops
from .corpus import BOOTSTRAPING_SUBSET, WINDOW_SIZE
from .encoder import ORACLE_LABEL_IDX, EncoderConfig, SentimentEncoder, build


class SentimentOraclePipeline:
    def __init__(self, engine, encoder: Optional[SentimentEncoder] = None, enc_cfg: EncoderConfig = EncoderConfig(),
                 window: int = WINDOW_SIZE, subset: int = BOOTSTRAPING_SUBSET, seed: int = 0):
        self.engine = engine
        dev = engine.device
        self.encoder = encoder if encoder is not None else build(dev, torch.bfloat16 if dev.type == "cuda"
                                                                 else torch.float32, seed, enc_cfg)
        self.window, self.subset = window, subset
        self.label_idx = torch.tensor(ORACLE_LABEL_IDX, dtype=torch.int32, device=dev)
        self.seed = seed
        self.fetches = 0
        W, N = engine.B, engine.N
        self._pred = torch.zeros(W, N, len(ORACLE_LABEL_IDX), dtype=torch.float32, device=dev)
        self._inst = torch.arange(W, device=dev).repeat_interleave(N)
        self._orc = torch.arange(N, device=dev).repeat(W)
        if engine.D != len(ORACLE_LABEL_IDX):
            raise ValueError("the sentiment path produces 6-D predictions (client/common.py:19-31)")

    @torch.no_grad()
    def classify(self, ids: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        """[W*C, S] token ids -> [W, C, 28] sigmoid scores."""
        s = self.encoder(ids, mask)
        return s.view(-1, self.window, s.shape[-1]).float().contiguous()

    @torch.no_grad()
    def oracles(self, scores: torch.Tensor, seed: Optional[int] = None) -> torch.Tensor:
        """[W, C, 28] -> [W, N, 6] bootstrapped oracle predictions (fused kernel)."""
        s = self.seed * 1_000_003 + self.fetches if seed is None else seed
        svops.ops().bootstrap_oracles(scores, self.label_idx, self._pred, self.engine.cfg.n_failing_oracles,
                                      self.subset, int(s))
        return self._pred

    @torch.no_grad()
    def fetch(self, ids: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        """One simulation fetch for every window + one consensus round per instance."""
        pred = self.oracles(self.classify(ids, mask))
        self.fetches += 1
        st = self.engine.apply_updates(self._inst, self._orc, pred.view(-1, pred.shape[-1]), unique=True)
        self.engine.run_round()
        return st
