"""RoBERTa/BERT-base style encoder + go_emotions multi-label head (the oracle's sentiment model).

The reference client runs HF ``pipeline("text-classification", "SamLowe/roberta-base-go_emotions",
top_k=None)`` (client/oracle_scheduler.py:23-25): a RoBERTa-base encoder, a 28-way classification
head, sigmoid scores for all 28 go_emotions labels; the client keeps 6 labels
(client/common.py:19-31) and normalises them to sum 1 (oracle_scheduler.py:20-21, 36-40).

There is no network on the GPU boxes, so the weights are random-initialised with a fixed seed and
the architecture is BERT-base sized (12 layers, hidden 768, 12 heads, FFN 3072, vocab 50265,
512 positions).  The implementation is plain PyTorch-ROCm: bf16 (or fp32, the reference's precision)
weights, fused QKV projection (one hipBLASLt GEMM), hand-written MFMA attention kernels for the short
windows (S <= 128: mfma_f32_32x32x16_bf16 / mfma_f32_32x32x2_f32) that read the QKV projection in place
over the packed (unpadded) tokens, erf GELU after the FC1 GEMM, fused residual-add + LayerNorm, fused
embeddings + LayerNorm and segment pooling (encoder_ops.hip, bf16 and fp32); pre-sized buffers so the
forward can be captured in a HIP graph.  ``load_hf_roberta`` maps a HF RobertaForSequenceClassification
checkpoint (e.g. SamLowe/roberta-base-go_emotions, if present locally) onto it.
"""
from __future__ import annotations

import dataclasses
import math
import os
from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

GO_EMOTIONS = [
    "admiration", "amusement", "anger", "annoyance", "approval", "caring", "confusion", "curiosity",
    "desire", "disappointment", "disapproval", "disgust", "embarrassment", "excitement", "fear",
    "gratitude", "grief", "joy", "love", "nervousness", "optimism", "pride", "realization", "relief",
    "remorse", "sadness", "surprise", "neutral",
]
# client/common.py:19-26 (order matters: it is the consensus vector's component order)
ORACLE_LABELS = ["optimism", "anger", "annoyance", "excitement", "nervousness", "remorse"]
ORACLE_LABEL_IDX = [GO_EMOTIONS.index(x) for x in ORACLE_LABELS]


@dataclasses.dataclass
class EncoderConfig:
    vocab_size: int = 50265
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    ffn: int = 3072
    max_positions: int = 514
    n_labels: int = 28
    layer_norm_eps: float = 1e-5
    pad_id: int = 1
    # "cls" = RoBERTa's <s> head; "mean" = masked mean pooling.  With random weights the layers
    # barely mix tokens, so the <s> state is ~input independent: mean pooling keeps the synthetic
    # oracle scores content dependent (the default here, since no trained checkpoint is available).
    pool: str = "mean"

    @classmethod
    def tiny(cls) -> "EncoderConfig":
        return cls(vocab_size=1000, hidden=64, layers=2, heads=4, ffn=128, max_positions=130)


class Layer(nn.Module):
    def __init__(self, c: EncoderConfig):
        super().__init__()
        self.heads = c.heads
        self.qkv = nn.Linear(c.hidden, 3 * c.hidden)
        self.out = nn.Linear(c.hidden, c.hidden)
        self.ln1 = nn.LayerNorm(c.hidden, eps=c.layer_norm_eps)
        self.fc1 = nn.Linear(c.hidden, c.ffn)
        self.fc2 = nn.Linear(c.ffn, c.hidden)
        self.ln2 = nn.LayerNorm(c.hidden, eps=c.layer_norm_eps)

    def forward(self, x: torch.Tensor, key_mask: Optional[torch.Tensor]) -> torch.Tensor:
        B, S, H = x.shape
        from .. import ops as svops
        # attention straight from the fused QKV projection [B, S, 3, heads, 64] into [B, S, H]
        # (MFMA kernel for S <= 128 on the GPU, encoder_ops.hip; ATen otherwise)
        a = svops.ops().attention_qkv(self.qkv(x), key_mask, self.heads)
        # post-LN (BERT/RoBERTa): residual add + LayerNorm fused in one HIP kernel (encoder_ops.hip)
        x = _add_ln(x, self.out(a), self.ln1)
        return _add_ln(x, self.fc2(_linear_gelu(x, self.fc1)), self.ln2)

    def forward_packed(self, x: torch.Tensor, plan: "PackPlan") -> torch.Tensor:
        """x: [T, H] real tokens only (sequence b = rows [cu[b], cu[b+1]))."""
        from .. import ops as svops
        o = svops.ops()
        if _use_emul(x, self.qkv):   # fp32: every GEMM on the bf16 matrix cores (_emul_linear)
            a = o.attention_varlen(_emul_linear(o.split3(x, False), self.qkv), plan.cu, plan.max_len, self.heads)
            x = _add_ln(x, _emul_linear(o.split3(a, False), self.out), self.ln1)
            h = _emul_linear(o.split3(x, False), self.fc1)
            return _add_ln(x, _emul_linear(o.split3(h, True), self.fc2), self.ln2)   # (split3 applies the GELU)
        a = o.attention_varlen(self.qkv(x), plan.cu, plan.max_len, self.heads)
        x = _add_ln(x, self.out(a), self.ln1)
        return _add_ln(x, _ffn(x, self.fc1, self.fc2), self.ln2)


@dataclasses.dataclass
class PackPlan:
    """Unpadded token layout of a right-padded batch (the reference pipeline classifies each comment
    on its own, i.e. never computes padding tokens)."""
    idx: torch.Tensor      # [T] flat positions b * S + s of the real tokens, in order
    pos: torch.Tensor      # [T] position ids
    cu: torch.Tensor       # [B + 1] int32 sequence offsets
    lens: torch.Tensor     # [B] float lengths
    T: int
    B: int
    S: int
    max_len: int


# RoBERTa's FFN activation is the erf GELU (HF hidden_act "gelu").  The hipBLASLt GELU epilogue of
# torch._addmm_activation computes the tanh approximation (tools/probe_gelu_kind.py on the MI355X: fp32
# epilogue - tanh GELU 4.8e-7, - erf GELU 4.7e-4), so the default is the GEMM (bias epilogue) followed by
# an in-place erf GELU over the [tokens, 3072] activation; SVOC_GELU_EPILOGUE=1 selects the tanh epilogue.
GELU_EPILOGUE = os.environ.get("SVOC_GELU_EPILOGUE", "0") == "1"


def _linear_gelu(x: torch.Tensor, fc: nn.Linear) -> torch.Tensor:
    """fc1 + erf GELU (the GPU: hipBLASLt GEMM with the bias epilogue, then the GELU in place)."""
    if x.is_cuda:
        x2 = x.reshape(-1, x.shape[-1])
        if GELU_EPILOGUE:
            y = torch._addmm_activation(fc.bias, x2, fc.weight.t(), use_gelu=True)
        else:
            y = torch.ops.aten.gelu_(torch.addmm(fc.bias, x2, fc.weight.t()))
        return y.view(*x.shape[:-1], -1)
    return F.gelu(fc(x))


# The FFN in row chunks on the GPU (SVOC_FFN_CHUNK rows; default: 32768 rows at fp32, whole at bf16): with a
# chunk's [rows, 3072] FC1 activation small enough to stay in the 256 MB Infinity Cache, the erf GELU pass and
# FC2's read of it are served from there instead of HBM.  Same-box A/B (tools/ab_ffn_chunk.sh, 2 reps): fp32
# c4 295.5 -> 302.3 windows/s; bf16 1,888-1,895 whole vs 1,846-1,886 chunked (the smaller GEMMs lose more than the
# GELU pass saves), so bf16 stays whole.
FFN_CHUNK = os.environ.get("SVOC_FFN_CHUNK")


def _ffn(x: torch.Tensor, fc1: nn.Linear, fc2: nn.Linear) -> torch.Tensor:
    """fc2(gelu(fc1(x))) over [T, H] tokens, in row chunks on the GPU (the same GEMMs per row)."""
    T = x.shape[0]
    chunk = int(FFN_CHUNK) if FFN_CHUNK is not None else (32768 if x.dtype == torch.float32 else 0)
    if not (x.is_cuda and chunk > 0 and T > chunk):
        return fc2(_linear_gelu(x, fc1))
    y = torch.empty(T, fc2.weight.shape[0], dtype=x.dtype, device=x.device)
    for r0 in range(0, T, chunk):
        r1 = min(T, r0 + chunk)
        torch.addmm(fc2.bias, _linear_gelu(x[r0:r1], fc1), fc2.weight.t(), out=y[r0:r1])
    return y


# fp32 weights on the GPU: SVOC_FP32_GEMM=bf16x6 runs the four per-layer linears as fp32 GEMMs emulated on
# the bf16 matrix cores.  Both operands are split three ways into bf16 (encoder_ops.hip split3: x = x0 + x1 +
# x2, 24 significant bits) and the six partial products above 2^-24 run as three bf16 GEMMs with fp32
# accumulation and output: [x0|x1|x2] [w0|w0|w0]^T + [x0|x1] [w1|w1]^T + x0 w2^T -- the error of an fp32 GEMM
# (tests/test_encoder_ops_gpu.py pins it against an fp64 reference next to the native fp32 GEMM's).  Not the
# default: hipBLASLt runs these shapes at ~88 % of the fp32 matrix peak but the bf16 ones at 30-47 % of the
# bf16 peak, so six bf16 products plus the splits measured slower (c4 fp32 262 vs 297 windows/s,
# tools/probe_emul_gemm.py, docs/PERF.md).  "native" (default) = hipBLASLt fp32 GEMMs.
FP32_GEMM = os.environ.get("SVOC_FP32_GEMM", "native")


def _weight_planes(fc: nn.Linear):
    """[w0|w0|w0], [w1|w1], w2 (bf16, [N, 3K] / [N, 2K] / [N, K]) of an fp32 Linear, cached on the module."""
    w = fc.weight
    key = (w.data_ptr(), w._version, w.device)
    cached = getattr(fc, "_emul_planes", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    from .. import ops as svops
    K = w.shape[1]
    p = svops.ops().split3(w.detach(), False)
    w0, w1, w2 = p[:, :K], p[:, K:2 * K], p[:, 2 * K:]
    planes = (torch.cat([w0, w0, w0], 1).contiguous(), torch.cat([w1, w1], 1).contiguous(), w2.contiguous())
    fc._emul_planes = (key, planes)
    return planes


def _emul_linear(xp: torch.Tensor, fc: nn.Linear) -> torch.Tensor:
    """fc(x) in fp32 from x's split planes xp = split3(x) ([M, 3K] bf16): three bf16 GEMMs, fp32 accumulate."""
    b1, b2, b3 = _weight_planes(fc)
    K = fc.weight.shape[1]
    y = torch.mm(xp[:, :K], b3.t(), out_dtype=torch.float32)              # x0 w2
    y = torch.addmm(y, xp[:, :2 * K], b2.t(), out_dtype=torch.float32)    # + x0 w1 + x1 w1
    y = torch.addmm(y, xp, b1.t(), out_dtype=torch.float32)               # + x0 w0 + x1 w0 + x2 w0
    if fc.bias is not None:
        y.add_(fc.bias)
    return y


def _use_emul(x: torch.Tensor, fc: nn.Linear) -> bool:
    return (FP32_GEMM == "bf16x6" and x.is_cuda and x.dtype == torch.float32 and fc.weight.dtype == torch.float32
            and x.dim() == 2 and x.shape[1] % 4 == 0)


def _add_ln(x: torch.Tensor, y: torch.Tensor, ln: nn.LayerNorm) -> torch.Tensor:
    from .. import ops as svops
    return svops.ops().add_layernorm(x, y, ln.weight, ln.bias, ln.eps)


class SentimentEncoder(nn.Module):
    def __init__(self, c: EncoderConfig = EncoderConfig()):
        super().__init__()
        self.cfg = c
        self.tok = nn.Embedding(c.vocab_size, c.hidden, padding_idx=c.pad_id)
        self.pos = nn.Embedding(c.max_positions, c.hidden)
        self.typ = nn.Embedding(1, c.hidden)
        self.ln = nn.LayerNorm(c.hidden, eps=c.layer_norm_eps)
        self.layers = nn.ModuleList([Layer(c) for _ in range(c.layers)])
        self.dense = nn.Linear(c.hidden, c.hidden)      # RobertaClassificationHead: dense-tanh-out
        self.head = nn.Linear(c.hidden, c.n_labels)
        self.apply(self._init)
        self.packed = True                 # unpadded token path on the GPU (see plan())
        # (a two-stream variant that overlapped one sequence range's attention / LayerNorm with the
        # next range's GEMMs measured 1918 vs 2053 windows/s single-stream and is gone: docs/PERF.md)
        self._plan_cache = []              # [(mask tensor, version, plan)], most recent last
        # random-init head scaled so the synthetic scores spread like a trained multi-label head's
        # (larger logits than the default init): keeps honest bootstrap oracles distinguishable at wsad
        # resolution, otherwise every column has ~zero variance and the contract reverts (§2.8-5)
        nn.init.normal_(self.head.weight, std=6.0 / math.sqrt(c.hidden))
        nn.init.normal_(self.dense.weight, std=3.0 / math.sqrt(c.hidden))

    @staticmethod
    def _init(m):
        if isinstance(m, (nn.Linear, nn.Embedding)):
            nn.init.normal_(m.weight, std=0.02)
        if isinstance(m, nn.Linear) and m.bias is not None:
            nn.init.zeros_(m.bias)

    def plan(self, attention_mask: torch.Tensor) -> Optional[PackPlan]:
        """Packing plan of a right-padded mask (None if some row is not of the form 1..1 0..0).
        Cached per mask tensor (identity + version; the cache holds a reference, so the storage
        cannot be recycled under a stale entry) for the last few masks, so a captured HIP graph that
        alternates between batches replays without the host synchronisation this needs the first time."""
        for m_ref, ver, cached in self._plan_cache:
            if m_ref is attention_mask and ver == attention_mask._version:
                return cached
        B, S = attention_mask.shape
        m = attention_mask.bool()
        lens = m.sum(1)
        plan = None
        if torch.equal(m, torch.arange(S, device=m.device)[None] < lens[:, None]):
            idx = m.flatten().nonzero().squeeze(1)
            cu = torch.zeros(B + 1, dtype=torch.int32, device=m.device)
            cu[1:] = lens.cumsum(0).to(torch.int32)
            plan = PackPlan(idx=idx, pos=idx % S + 2, cu=cu, lens=lens.to(torch.float32).clamp(min=1), T=int(idx.numel()),
                            B=B, S=S, max_len=int(lens.max()) if B else 0)
        self._plan_cache = self._plan_cache[-3:] + [(attention_mask, attention_mask._version, plan)]
        return plan

    def _forward_packed(self, ids: torch.Tensor, p: PackPlan) -> torch.Tensor:
        from .. import ops as svops
        o = svops.ops()
        # embeddings + LayerNorm in one HIP kernel (gather, two adds, LN), [T, H]
        x = o.embed_layernorm(ids.reshape(-1)[p.idx], p.pos, self.tok.weight, self.pos.weight, self.typ.weight,
                              self.ln.weight, self.ln.bias, self.ln.eps)
        for layer in self.layers:
            x = layer.forward_packed(x, p)
        if self.cfg.pool == "cls":
            pooled = x[p.cu[:-1].long()]
        else:   # masked mean over each sequence's real tokens (fp32 sums, one HIP kernel)
            pooled = o.segment_mean(x, p.cu)
        h = torch.tanh(self.dense(pooled))
        return torch.sigmoid(self.head(h).float())

    def forward(self, ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        """ids [B, S] -> 28 sigmoid scores [B, 28] (float32)."""
        B, S = ids.shape
        if self.packed and attention_mask is not None and ids.is_cuda and S <= 128:
            p = self.plan(attention_mask)
            if p is not None and p.T > 0:
                return self._forward_packed(ids, p)
        pos = torch.arange(2, S + 2, device=ids.device)           # RoBERTa positions start at pad+1
        x = self.ln(self.tok(ids) + self.pos(pos)[None] + self.typ.weight[0])
        kmask = attention_mask.to(torch.uint8) if attention_mask is not None else None
        for layer in self.layers:
            x = layer(x, kmask)
        if self.cfg.pool == "cls" or attention_mask is None:
            pooled = x[:, 0] if self.cfg.pool == "cls" else x.mean(1)
        else:
            m = attention_mask.to(x.dtype)[:, :, None]
            pooled = (x * m).sum(1) / m.sum(1).clamp(min=1)
        h = torch.tanh(self.dense(pooled))
        return torch.sigmoid(self.head(h).float())


def config_from_hf(hf_cfg) -> EncoderConfig:
    """EncoderConfig of a HF ``RobertaConfig`` (e.g. SamLowe/roberta-base-go_emotions's), ``<s>`` pooling."""
    if getattr(hf_cfg, "hidden_act", "gelu") != "gelu":
        raise ValueError(f"only erf GELU encoders map onto SentimentEncoder (got {hf_cfg.hidden_act})")
    if getattr(hf_cfg, "type_vocab_size", 1) != 1:
        raise ValueError("RoBERTa has one token type")
    return EncoderConfig(vocab_size=hf_cfg.vocab_size, hidden=hf_cfg.hidden_size, layers=hf_cfg.num_hidden_layers,
                         heads=hf_cfg.num_attention_heads, ffn=hf_cfg.intermediate_size,
                         max_positions=hf_cfg.max_position_embeddings, n_labels=hf_cfg.num_labels,
                         layer_norm_eps=hf_cfg.layer_norm_eps, pad_id=hf_cfg.pad_token_id, pool="cls")


@torch.no_grad()
def load_hf_roberta(model: SentimentEncoder, sd) -> SentimentEncoder:
    """Copy a HF ``RobertaForSequenceClassification`` state dict into ``model`` (same sizes): separate
    query / key / value projections -> the fused QKV projection ([q; k; v] rows, the layout
    attention_qkv reads), the classification head (dense-tanh-out_proj on the <s> state) -> dense / head.
    With such weights the encoder computes the reference's classifier (client/oracle_scheduler.py:23-40:
    sigmoid over the 28 go_emotions logits) -- tests/test_sentiment.py pins it against transformers."""
    p = "roberta."
    g = lambda k: sd[k]  # noqa: E731
    model.tok.weight.copy_(g(p + "embeddings.word_embeddings.weight"))
    model.pos.weight.copy_(g(p + "embeddings.position_embeddings.weight"))
    model.typ.weight.copy_(g(p + "embeddings.token_type_embeddings.weight"))
    model.ln.weight.copy_(g(p + "embeddings.LayerNorm.weight"))
    model.ln.bias.copy_(g(p + "embeddings.LayerNorm.bias"))
    for i, L in enumerate(model.layers):
        q = f"{p}encoder.layer.{i}."
        L.qkv.weight.copy_(torch.cat([g(q + f"attention.self.{n}.weight") for n in ("query", "key", "value")]))
        L.qkv.bias.copy_(torch.cat([g(q + f"attention.self.{n}.bias") for n in ("query", "key", "value")]))
        for dst, src in ((L.out, "attention.output.dense"), (L.fc1, "intermediate.dense"), (L.fc2, "output.dense")):
            dst.weight.copy_(g(q + src + ".weight"))
            dst.bias.copy_(g(q + src + ".bias"))
        for dst, src in ((L.ln1, "attention.output.LayerNorm"), (L.ln2, "output.LayerNorm")):
            dst.weight.copy_(g(q + src + ".weight"))
            dst.bias.copy_(g(q + src + ".bias"))
    model.dense.weight.copy_(g("classifier.dense.weight"))
    model.dense.bias.copy_(g("classifier.dense.bias"))
    model.head.weight.copy_(g("classifier.out_proj.weight"))
    model.head.bias.copy_(g("classifier.out_proj.bias"))
    return model


def scores_to_oracle_vectors(scores: torch.Tensor) -> torch.Tensor:
    """prediction_to_vector + normalize (oracle_scheduler.py:20-34): [..., 28] -> [..., 6], sum 1."""
    v = scores[..., ORACLE_LABEL_IDX]
    return v / v.sum(-1, keepdim=True)


def build(device="cuda", dtype=torch.bfloat16, seed: int = 0, cfg: EncoderConfig = EncoderConfig()) -> SentimentEncoder:
    state = torch.random.get_rng_state()   # deterministic weights without disturbing the caller's RNG
    torch.manual_seed(seed)
    m = SentimentEncoder(cfg)
    torch.random.set_rng_state(state)
    return m.to(device=device, dtype=dtype).eval()


def flops_for_lengths(c: EncoderConfig, lens) -> float:
    """Forward FLOPs of a batch of unpadded sequences (lengths ``lens``)."""
    return float(sum(flops_per_sequence(c, int(n)) for n in lens))


def flops_per_sequence(c: EncoderConfig, S: int) -> float:
    """Forward FLOPs for one sequence (GEMMs + attention), for throughput reporting."""
    per_layer = 2 * S * c.hidden * (3 * c.hidden + c.hidden + 2 * c.ffn) + 4 * S * S * c.hidden
    return c.layers * per_layer + 2 * c.hidden * (c.hidden + c.n_labels)
