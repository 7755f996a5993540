"""Fused encoder kernels (csrc/kernels/encoder_ops.hip) vs plain PyTorch fp32."""
import pytest
import torch
import torch.nn.functional as F

from svoc import ops as svops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,H", [(1, 768), (1023, 768), (257, 256), (64, 1024), (5, 512)])
def test_add_layernorm_bf16(rows, H):
    g = torch.Generator(device="cuda").manual_seed(rows + H)
    x = torch.randn(rows, H, device="cuda", generator=g).to(torch.bfloat16)
    y = (0.5 * torch.randn(rows, H, device="cuda", generator=g) + 0.1).to(torch.bfloat16)
    w = (1 + 0.1 * torch.randn(H, device="cuda", generator=g)).to(torch.bfloat16)
    b = (0.1 * torch.randn(H, device="cuda", generator=g)).to(torch.bfloat16)
    out = svops.ops().add_layernorm(x, y, w, b, 1e-5)
    ref = F.layer_norm(x.float() + y.float(), (H,), w.float(), b.float(), 1e-5)
    assert out.dtype == torch.bfloat16 and out.shape == x.shape
    torch.testing.assert_close(out.float(), ref, rtol=1e-2, atol=2e-2)
    # bf16 rounding of the output is the only error source: compare against the rounded reference
    assert (out.float() - ref.to(torch.bfloat16).float()).abs().max().item() <= 0.0625


@pytest.mark.parametrize("H", [768, 256])
def test_add_layernorm_broadcast_row(H):
    """y as one [H] row (the GEMM bias when the residual was accumulated into the GEMM output)."""
    g = torch.Generator(device="cuda").manual_seed(H)
    x = torch.randn(333, H, device="cuda", generator=g).to(torch.bfloat16)
    y = (0.3 * torch.randn(H, device="cuda", generator=g)).to(torch.bfloat16)
    w = (1 + 0.1 * torch.randn(H, device="cuda", generator=g)).to(torch.bfloat16)
    b = (0.1 * torch.randn(H, device="cuda", generator=g)).to(torch.bfloat16)
    out = svops.ops().add_layernorm(x, y, w, b, 1e-5)
    ref = F.layer_norm(x.float() + y.float()[None], (H,), w.float(), b.float(), 1e-5)
    assert (out.float() - ref.to(torch.bfloat16).float()).abs().max().item() <= 0.0625


def test_add_layernorm_3d_and_fallback_width():
    x = torch.randn(2, 7, 64, device="cuda", dtype=torch.bfloat16)
    y = torch.randn(2, 7, 64, device="cuda", dtype=torch.bfloat16)
    w = torch.ones(64, device="cuda", dtype=torch.bfloat16)
    b = torch.zeros(64, device="cuda", dtype=torch.bfloat16)
    out = svops.ops().add_layernorm(x, y, w, b, 1e-5)   # H = 64: ATen path
    torch.testing.assert_close(out.float(), F.layer_norm((x + y).float(), (64,), w.float(), b.float(), 1e-5),
                               rtol=2e-2, atol=3e-2)


def _attn_ref(qkv, mask, heads):
    B, S, H3 = qkv.shape
    HD = H3 // 3
    DH = HD // heads
    t = qkv.float().view(B, S, 3, heads, DH).permute(2, 0, 3, 1, 4)
    s = t[0] @ t[1].transpose(-1, -2) / DH ** 0.5
    if mask is not None:
        s = s.masked_fill(~mask.bool()[:, None, None, :], float("-inf"))
    return (torch.softmax(s, -1) @ t[2]).transpose(1, 2).reshape(B, S, HD)


@pytest.mark.parametrize("S", [32, 64, 96, 128])
def test_attention_qkv_mfma(S):
    B, heads = 5, 12
    g = torch.Generator(device="cuda").manual_seed(S)
    qkv = torch.randn(B, S, 3 * heads * 64, device="cuda", generator=g).to(torch.bfloat16)
    lens = torch.randint(1, S + 1, (B,), device="cuda", generator=g)
    mask = (torch.arange(S, device="cuda")[None] < lens[:, None]).to(torch.uint8)
    out = svops.ops().attention_qkv(qkv, mask, heads)
    ref = _attn_ref(qkv, mask, heads)
    assert out.shape == (B, S, heads * 64) and out.dtype == torch.bfloat16
    torch.testing.assert_close(out.float(), ref, rtol=3e-2, atol=3e-2)
    out2 = svops.ops().attention_qkv(qkv, None, heads)
    torch.testing.assert_close(out2.float(), _attn_ref(qkv, None, heads), rtol=3e-2, atol=3e-2)


def test_encoder_fused_matches_cpu_fp32():
    from svoc.models.encoder import EncoderConfig, build
    cfg = EncoderConfig(vocab_size=500, hidden=768, layers=2, heads=12, ffn=3072, max_positions=130)
    enc_g = build("cuda", torch.bfloat16, seed=3, cfg=cfg)
    enc_c = build("cpu", torch.float32, seed=3, cfg=cfg)
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(3, 500, (6, 128), generator=g)
    mask = (torch.arange(128)[None] < torch.tensor([128, 40, 77, 128, 9, 100])[:, None]).to(torch.int64)
    with torch.no_grad():
        sg = enc_g(ids.cuda(), mask.cuda()).float().cpu()
        sc = enc_c(ids, mask)
    torch.testing.assert_close(sg, sc, rtol=0, atol=0.05)


@pytest.mark.parametrize("packed", [True, False])
def test_encoder_oracle_vectors_match_cpu_fp32_bert_base(packed):
    """The full BERT-base encoder (12 x 768, bf16 on the GPU: MFMA attention, fused embed / add + LN,
    hipBLASLt GEMMs) against the fp32 CPU encoder of the same weights, on what the reference consumes:
    the normalised 6-label oracle vectors (oracle_scheduler.py:20-40).  max |delta| <= 0.01."""
    from svoc.models.encoder import build, scores_to_oracle_vectors
    enc_g = build("cuda", torch.bfloat16, seed=11)
    enc_g.packed = packed
    enc_c = build("cpu", torch.float32, seed=11)
    g = torch.Generator().manual_seed(5)
    lens = torch.tensor([128, 40, 77, 128, 9, 100, 64, 1])
    ids = torch.randint(3, enc_c.cfg.vocab_size, (8, 128), generator=g)
    mask = (torch.arange(128)[None] < lens[:, None]).to(torch.int64)
    with torch.no_grad():
        vg = scores_to_oracle_vectors(enc_g(ids.cuda(), mask.cuda()).float().cpu())
        vc = scores_to_oracle_vectors(enc_c(ids, mask))
    err = (vg - vc).abs().max().item()
    assert err <= 0.005, err


@pytest.mark.parametrize("packed", [True, False])
def test_encoder_fp32_gpu_matches_cpu(packed):
    """The fp32 GPU encoder (bench.py's reference-precision c4 field: packed tokens, the fp32 MFMA attention and
    LayerNorm kernels; or the padded path) equals the CPU fp32 encoder to fp32 rounding: the GEMMs sum in a
    different order (hipBLASLt vs the CPU BLAS) through 12 layers; round 4 measured max |delta| of the
    normalised 6-vectors 0.8e-4 - 1.13e-4 across boxes."""
    from svoc.models.encoder import build, scores_to_oracle_vectors
    enc_g = build("cuda", torch.float32, seed=12)
    enc_g.packed = packed
    enc_c = build("cpu", torch.float32, seed=12)
    g = torch.Generator().manual_seed(6)
    ids = torch.randint(3, enc_c.cfg.vocab_size, (4, 128), generator=g)
    mask = (torch.arange(128)[None] < torch.tensor([128, 50, 3, 90])[:, None]).to(torch.int64)
    with torch.no_grad():
        vg = scores_to_oracle_vectors(enc_g(ids.cuda(), mask.cuda()).cpu())
        vc = scores_to_oracle_vectors(enc_c(ids, mask))
    assert (vg - vc).abs().max().item() <= 5e-4


def test_attention_varlen_mfma():
    heads = 12
    lens = [128, 1, 33, 64, 95, 7, 128, 32]
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device="cuda")
    T = int(cu[-1])
    g = torch.Generator(device="cuda").manual_seed(1)
    qkv = torch.randn(T, 3 * heads * 64, device="cuda", generator=g).to(torch.bfloat16)
    out = svops.ops().attention_varlen(qkv, cu, max(lens), heads)
    ref = svops.ops().attention_varlen(qkv.cpu().float(), cu.cpu(), max(lens), heads)   # CPU reference path
    torch.testing.assert_close(out.float().cpu(), ref.float(), rtol=3e-2, atol=3e-2)


def test_encoder_packed_equals_padded():
    from svoc.models.encoder import EncoderConfig, build
    cfg = EncoderConfig(vocab_size=500, hidden=768, layers=2, heads=12, ffn=3072, max_positions=130)
    enc = build("cuda", torch.bfloat16, seed=4, cfg=cfg)
    g = torch.Generator().manual_seed(2)
    ids = torch.randint(3, 500, (7, 128), generator=g).cuda()
    mask = (torch.arange(128)[None] < torch.tensor([128, 40, 77, 1, 9, 100, 64])[:, None]).to(torch.int64).cuda()
    with torch.no_grad():
        a = enc(ids, mask)
        assert enc.plan(mask) is not None and enc.plan(mask).T == 419
        enc.packed = False
        b = enc(ids, mask)
    torch.testing.assert_close(a, b, rtol=0, atol=0.03)


@pytest.mark.parametrize("H", [768, 256])
def test_embed_layernorm_bf16(H):
    """Fused embedding gather + adds + LayerNorm vs the same PyTorch expression (bf16 adds, fp32 LN)."""
    V, P, T = 300, 130, 1000
    g = torch.Generator(device="cuda").manual_seed(H)
    tok = (0.02 * torch.randn(V, H, device="cuda", generator=g)).to(torch.bfloat16)
    pos = (0.02 * torch.randn(P, H, device="cuda", generator=g)).to(torch.bfloat16)
    typ = (0.02 * torch.randn(1, H, device="cuda", generator=g)).to(torch.bfloat16)
    w = (1 + 0.1 * torch.randn(H, device="cuda", generator=g)).to(torch.bfloat16)
    b = (0.1 * torch.randn(H, device="cuda", generator=g)).to(torch.bfloat16)
    ids = torch.randint(0, V, (T,), device="cuda", generator=g)
    pid = torch.randint(0, P, (T,), device="cuda", generator=g)
    out = svops.ops().embed_layernorm(ids, pid, tok, pos, typ, w, b, 1e-5)
    e = (tok[ids] + pos[pid] + typ[0]).float()
    ref = F.layer_norm(e, (H,), w.float(), b.float(), 1e-5)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)
    cpu = svops.ops().embed_layernorm(ids.cpu(), pid.cpu(), tok.cpu(), pos.cpu(), typ.cpu(), w.cpu(), b.cpu(), 1e-5)
    torch.testing.assert_close(out.cpu().float(), cpu.float(), rtol=2e-2, atol=2e-2)


def test_segment_mean_bf16():
    """Masked mean pooling over packed segments (empty and 1-token segments included) vs fp32."""
    lens = [5, 0, 1, 128, 77, 3]
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device="cuda")
    T, H = int(cu[-1]), 768
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(T, H, device="cuda", generator=g).to(torch.bfloat16)
    out = svops.ops().segment_mean(x, cu)
    ref = torch.stack([x[int(cu[i]):int(cu[i + 1])].float().sum(0) / max(lens[i], 1) for i in range(len(lens))])
    torch.testing.assert_close(out.float(), ref, rtol=1e-2, atol=1e-2)
    assert torch.equal(out[1].float(), torch.zeros(H, device="cuda"))
    cpu = svops.ops().segment_mean(x.cpu(), cu.cpu())
    torch.testing.assert_close(out.cpu().float(), cpu.float(), rtol=1e-2, atol=1e-2)


# ---------------------------------------------------------------- fp32 kernels (the reference's precision)
@pytest.mark.parametrize("rows,H", [(1, 768), (1023, 768), (257, 256), (64, 1024)])
def test_add_layernorm_f32(rows, H):
    g = torch.Generator(device="cuda").manual_seed(rows + H + 1)
    x = torch.randn(rows, H, device="cuda", generator=g)
    y = 0.5 * torch.randn(rows, H, device="cuda", generator=g) + 0.1
    w = 1 + 0.1 * torch.randn(H, device="cuda", generator=g)
    b = 0.1 * torch.randn(H, device="cuda", generator=g)
    out = svops.ops().add_layernorm(x, y, w, b, 1e-5)
    ref = F.layer_norm((x + y).double(), (H,), w.double(), b.double(), 1e-5)
    assert out.dtype == torch.float32
    torch.testing.assert_close(out.double(), ref, rtol=0, atol=2e-5)
    row = svops.ops().add_layernorm(x, y[0], w, b, 1e-5)                      # broadcast [H] row
    torch.testing.assert_close(row.double(), F.layer_norm((x + y[0]).double(), (H,), w.double(), b.double(), 1e-5),
                               rtol=0, atol=2e-5)


def test_embed_layernorm_f32():
    V, P, T, H = 300, 130, 999, 768
    g = torch.Generator(device="cuda").manual_seed(11)
    tok = 0.02 * torch.randn(V, H, device="cuda", generator=g)
    pos = 0.02 * torch.randn(P, H, device="cuda", generator=g)
    typ = 0.02 * torch.randn(1, H, device="cuda", generator=g)
    w = 1 + 0.1 * torch.randn(H, device="cuda", generator=g)
    b = 0.1 * torch.randn(H, device="cuda", generator=g)
    ids = torch.randint(0, V, (T,), device="cuda", generator=g)
    pid = torch.randint(0, P, (T,), device="cuda", generator=g)
    out = svops.ops().embed_layernorm(ids, pid, tok, pos, typ, w, b, 1e-5)
    ref = F.layer_norm((tok[ids] + pos[pid] + typ[0]).double(), (H,), w.double(), b.double(), 1e-5)
    torch.testing.assert_close(out.double(), ref, rtol=0, atol=2e-5)


def test_segment_mean_f32():
    lens = [5, 0, 1, 128, 77, 3]
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device="cuda")
    T, H = int(cu[-1]), 768
    x = torch.randn(T, H, device="cuda", generator=torch.Generator(device="cuda").manual_seed(8))
    out = svops.ops().segment_mean(x, cu)
    ref = torch.stack([x[int(cu[i]):int(cu[i + 1])].double().sum(0) / max(lens[i], 1) for i in range(len(lens))])
    torch.testing.assert_close(out.double(), ref, rtol=0, atol=1e-5)
    assert torch.equal(out[1], torch.zeros(H, device="cuda"))


def _attn_ref64(qkv, mask, heads):
    B, S, H3 = qkv.shape
    DH = H3 // 3 // heads
    t = qkv.double().view(B, S, 3, heads, DH).permute(2, 0, 3, 1, 4)
    s = t[0] @ t[1].transpose(-1, -2) / DH ** 0.5
    if mask is not None:
        s = s.masked_fill(~mask.bool()[:, None, None, :], float("-inf"))
    return (torch.softmax(s, -1) @ t[2]).transpose(1, 2).reshape(B, S, H3 // 3)


@pytest.mark.parametrize("S", [32, 64, 96, 128])
def test_attention_qkv_f32_mfma(S):
    """fp32 attention on mfma_f32_32x32x2_f32 vs an fp64 reference (fp32 products, fp32 sums)."""
    B, heads = 5, 12
    g = torch.Generator(device="cuda").manual_seed(S + 7)
    qkv = torch.randn(B, S, 3 * heads * 64, device="cuda", generator=g)
    lens = torch.randint(1, S + 1, (B,), device="cuda", generator=g)
    mask = (torch.arange(S, device="cuda")[None] < lens[:, None]).to(torch.uint8)
    out = svops.ops().attention_qkv(qkv, mask, heads)
    assert out.dtype == torch.float32 and out.shape == (B, S, heads * 64)
    torch.testing.assert_close(out.double(), _attn_ref64(qkv, mask, heads), rtol=0, atol=2e-5)
    out2 = svops.ops().attention_qkv(qkv, None, heads)
    torch.testing.assert_close(out2.double(), _attn_ref64(qkv, None, heads), rtol=0, atol=2e-5)


def test_attention_varlen_f32_mfma():
    heads = 12
    lens = [128, 1, 33, 64, 95, 7, 128, 32]
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device="cuda")
    T = int(cu[-1])
    qkv = torch.randn(T, 3 * heads * 64, device="cuda", generator=torch.Generator(device="cuda").manual_seed(3))
    out = svops.ops().attention_varlen(qkv, cu, max(lens), heads)
    ref = svops.ops().attention_varlen(qkv.cpu().double(), cu.cpu(), max(lens), heads)
    torch.testing.assert_close(out.double().cpu(), ref, rtol=0, atol=2e-5)


# ---------------------------------------------------------------- fp32 GEMMs on the bf16 matrix cores
@pytest.mark.parametrize("gelu", [False, True])
def test_split3_matches_cpu(gelu):
    """The three-way bf16 split kernel vs its CPU reference: x0 + x1 + x2 reproduces x (or GELU(x)) to 2^-24."""
    g = torch.Generator(device="cuda").manual_seed(3 + gelu)
    x = 3 * torch.randn(1000, 768, device="cuda", generator=g)
    p = svops.ops().split3(x, gelu)
    assert p.shape == (1000, 3 * 768) and p.dtype == torch.bfloat16
    pc = svops.ops().split3(x.cpu(), gelu)
    rec = p[:, :768].double() + p[:, 768:1536].double() + p[:, 1536:].double()
    if gelu:   # (the kernel's fp32 erf GELU vs aten's fp32 one; 1 + erf cancels for negative x: absolute bound)
        torch.testing.assert_close(rec, F.gelu(x).double(), rtol=1e-6, atol=2e-7)
    else:
        assert ((rec - x.double()).abs() <= 2 ** -22 * x.double().abs()).all()
    if not gelu:
        assert torch.equal(p.cpu(), pc)
    else:   # (device erff vs the CPU's: the leading plane may differ by one bf16 ulp on ties)
        recc = pc[:, :768].double() + pc[:, 768:1536].double() + pc[:, 1536:].double()
        torch.testing.assert_close(rec.cpu(), recc, rtol=1e-5, atol=2e-6)


@pytest.mark.parametrize("M,K,N", [(2000, 768, 2304), (1500, 3072, 768), (333, 768, 3072)])
def test_emul_linear_error_is_fp32_like(M, K, N):
    """encoder._emul_linear (fp32 GEMM as six bf16 products, three bf16 GEMMs with fp32 accumulation) against an
    fp64 reference, next to hipBLASLt's native fp32 GEMM: the same error scale."""
    from svoc.models.encoder import _emul_linear
    g = torch.Generator(device="cuda").manual_seed(M + K)
    fc = torch.nn.Linear(K, N).cuda()
    with torch.no_grad():
        fc.weight.copy_(0.05 * torch.randn(N, K, device="cuda", generator=g))
        fc.bias.copy_(0.1 * torch.randn(N, device="cuda", generator=g))
    x = torch.randn(M, K, device="cuda", generator=g)
    with torch.no_grad():
        ref = torch.addmm(fc.bias.double(), x.double(), fc.weight.double().t())
        native = torch.addmm(fc.bias, x, fc.weight.t())
        emul = _emul_linear(svops.ops().split3(x, False), fc)
    en = (native.double() - ref).abs().max().item()
    ee = (emul.double() - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert ee <= 2.0 * en + 1e-6 * scale, (ee, en, scale)
    assert ee <= 1e-5 * scale, (ee, scale)


def test_encoder_fp32_emul_matches_native():
    """The fp32 encoder with every layer GEMM emulated on the bf16 matrix cores equals the native fp32 GEMM
    encoder to fp32 rounding (oracle 6-vectors)."""
    import svoc.models.encoder as enc_mod
    from svoc.models.encoder import build, scores_to_oracle_vectors
    enc = build("cuda", torch.float32, seed=21)
    g = torch.Generator().manual_seed(9)
    ids = torch.randint(3, enc.cfg.vocab_size, (6, 128), generator=g).cuda()
    mask = (torch.arange(128)[None] < torch.tensor([128, 64, 7, 90, 33, 128])[:, None]).to(torch.int64).cuda()
    old = enc_mod.FP32_GEMM
    try:
        with torch.no_grad():
            enc_mod.FP32_GEMM = "native"
            vn = scores_to_oracle_vectors(enc(ids, mask).cpu())
            enc_mod.FP32_GEMM = "bf16x6"
            ve = scores_to_oracle_vectors(enc(ids, mask).cpu())
    finally:
        enc_mod.FP32_GEMM = old
    assert (vn - ve).abs().max().item() <= 2e-4
