"""Sentiment-oracle path: encoder, corpus / SQLite window, fused bootstrap kernel (CPU twin)."""
import pytest
import torch

from svoc import ops as svops
from svoc.config import ConsensusConfig
from svoc.engine import ConsensusEngine
from svoc.models import corpus
from svoc.models.encoder import ORACLE_LABELS, EncoderConfig, build, scores_to_oracle_vectors
from svoc.models.sentiment_oracle import SentimentOraclePipeline

pytestmark = pytest.mark.skipif(not svops.available(), reason="svoc/_C.so not built")


def test_encoder_and_labels():
    m = build("cpu", torch.float32, 0, EncoderConfig.tiny())
    ids, mask = corpus.tokenize(corpus.synthetic_comments(5), seq_len=32, vocab=1000)
    s = m(ids, mask)
    assert s.shape == (5, 28) and (s > 0).all() and (s < 1).all()
    v = scores_to_oracle_vectors(s)
    assert v.shape == (5, 6) and torch.allclose(v.sum(-1), torch.ones(5))
    assert ORACLE_LABELS[0] == "optimism"


def test_sqlite_window_semantics(tmp_path):
    conn = corpus.init_db(str(tmp_path / "db.sqlite"))
    corpus.save_to_db(conn, corpus.synthetic_comments(200, seed=1), "2024-10-08 10:00:00")
    c, ts, pos = corpus.read_window_from_db(conn, 0)
    assert pos == 50 and len(c) == 30 and ts[0] == "2024-10-08 10:00:00"
    c, ts, pos = corpus.read_window_from_db(conn, 100)     # 150 + 50 >= 200 -> wrap to 0
    assert pos == 0
    assert corpus.get_last_comment_time(conn) == "2024-10-08 10:00:00"


def test_bootstrap_semantics():
    W, C, N, D, f = 3, 30, 7, 6, 2
    scores = torch.rand(W, C, 28)
    idx = torch.tensor([20, 2, 3, 13, 19, 24], dtype=torch.int32)
    out = torch.zeros(W, N, D)
    svops.ops().bootstrap_oracles(scores, idx, out, f, 10, 42)
    vecs = scores[:, :, idx.long()]
    vecs = vecs / vecs.sum(-1, keepdim=True)
    for w in range(W):
        honest = 0
        for o in range(N):
            v = out[w, o]
            # an honest oracle is a mean of 10 normalised comment vectors: it sums to 1
            if abs(float(v.sum()) - 1.0) < 1e-5:
                honest += 1
                lo, hi = vecs[w].min(0).values, vecs[w].max(0).values
                assert (v >= lo - 1e-6).all() and (v <= hi + 1e-6).all()
        assert honest == N - f
    out2 = torch.zeros_like(out)
    svops.ops().bootstrap_oracles(scores, idx, out2, f, 10, 42)
    assert torch.equal(out, out2)                          # counter-based RNG: reproducible


def test_pipeline_end_to_end_cpu():
    cfg = ConsensusConfig(n_oracles=7, dimension=6, n_failing_oracles=2)
    eng = ConsensusEngine(cfg, 4, device="cpu", mode="fast", storage="fp32")
    pipe = SentimentOraclePipeline(eng, enc_cfg=EncoderConfig.tiny())
    ids, mask = corpus.tokenize(corpus.synthetic_comments(4 * 30, seed=3), seq_len=32, vocab=1000)
    st = pipe.fetch(ids, mask)
    assert (st == 0).all()
    assert (eng.n_active == 7).all()
    assert eng.consensus_active.any()


@pytest.mark.gpu
def test_bootstrap_gpu_bitwise_equals_cpu():
    W, C, N, D = 50, 30, 64, 6
    scores = torch.rand(W, C, 28)
    idx = torch.tensor([20, 2, 3, 13, 19, 24], dtype=torch.int32)
    oc = torch.zeros(W, N, D)
    og = torch.zeros(W, N, D, device="cuda")
    svops.ops().bootstrap_oracles(scores, idx, oc, 8, 10, 7)
    svops.ops().bootstrap_oracles(scores.cuda(), idx.cuda(), og, 8, 10, 7)
    assert torch.equal(oc, og.cpu())


@pytest.mark.gpu
def test_pipeline_gpu_bert_base():
    cfg = ConsensusConfig(n_oracles=7, dimension=6, n_failing_oracles=2)
    eng = ConsensusEngine(cfg, 8, device="cuda", mode="fast")
    pipe = SentimentOraclePipeline(eng)                     # full BERT-base size, bf16
    g = torch.Generator(device="cuda").manual_seed(0)
    ids, mask = corpus.synthetic_token_batch(8 * 30, 128, 50265, g, "cuda")
    st = pipe.fetch(ids, mask)
    torch.cuda.synchronize()
    assert (st == 0).all()
    assert eng.consensus_active.all()
    assert torch.isfinite(eng.consensus).all()


def test_encoder_matches_hf_roberta_classifier():
    """SentimentEncoder(pool="cls") loaded with a HF RobertaForSequenceClassification's weights computes that
    classifier's 28 sigmoid scores (the reference's pipeline: client/oracle_scheduler.py:23-40 runs
    SamLowe/roberta-base-go_emotions, a multi-label RoBERTa-base) -- random-init weights at full RoBERTa-base
    size (no download), right-padded batches, fp32 on the CPU."""
    transformers = pytest.importorskip("transformers")
    from svoc.models.encoder import SentimentEncoder, config_from_hf, load_hf_roberta
    torch.manual_seed(0)
    hc = transformers.RobertaConfig(vocab_size=50265, num_labels=28, problem_type="multi_label_classification",
                                    max_position_embeddings=514, type_vocab_size=1, layer_norm_eps=1e-5,
                                    pad_token_id=1)
    hf = transformers.RobertaForSequenceClassification(hc).eval()
    with torch.no_grad():   # spread the scores (the default init leaves every logit near 0)
        for n, p in hf.named_parameters():
            if n.endswith("LayerNorm.weight"):
                p.uniform_(0.8, 1.2)
            elif n.endswith("bias"):
                p.normal_(0.0, 0.02)
            elif "classifier" in n:
                p.normal_(0.0, 0.2)
    ours = load_hf_roberta(SentimentEncoder(config_from_hf(hc)), hf.state_dict()).eval()
    g = torch.Generator().manual_seed(1)
    B, S = 6, 40
    lens = torch.tensor([40, 7, 23, 2, 31, 12])
    ids = torch.randint(3, 50265, (B, S), generator=g)
    mask = (torch.arange(S)[None] < lens[:, None]).long()
    ids[:, 0] = 0                                                    # <s>
    ids[torch.arange(B), lens - 1] = 2                               # </s>
    ids = torch.where(mask.bool(), ids, torch.ones_like(ids))        # <pad> = 1
    with torch.no_grad():
        ref = torch.sigmoid(hf(input_ids=ids, attention_mask=mask).logits)
        got = ours(ids, mask)
    assert got.shape == (B, 28)
    assert float(ref.std()) > 0.05                                   # the comparison is not between constants
    torch.testing.assert_close(got, ref, rtol=0, atol=1e-5)
