"""The reference's classifier on the GPU path.

The reference classifies each comment with the ``<s>`` head of SamLowe/roberta-base-go_emotions
(client/oracle_scheduler.py:23-40; six labels, client/common.py:19-31).  ``tests/test_sentiment.py`` pins the
CPU encoder to a random-init HF ``RobertaForSequenceClassification``; here the same HF weights are loaded
into ``SentimentEncoder(pool="cls")`` on the GPU and its packed (unpadded-token) path -- the fused embedding
+ LayerNorm kernel, the MFMA varlen attention kernel, hipBLASLt GEMMs, the add + LayerNorm kernel and the
``<s>`` gather -- is compared with the HF classifier computed on the CPU in fp32.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _hf_pair(dtype):
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
    ours = load_hf_roberta(SentimentEncoder(config_from_hf(hc)), hf.state_dict())
    return hf, ours.to("cuda", dtype).eval()


def _batch(B, S, seed):
    g = torch.Generator().manual_seed(seed)
    lens = torch.randint(2, S + 1, (B,), generator=g)
    lens[0] = S
    ids = torch.randint(3, 50265, (B, S), generator=g)
    mask = (torch.arange(S)[None] < lens[:, None]).long()
    ids[:, 0] = 0                                                    # <s>
    ids[torch.arange(B), lens - 1] = 2                               # </s>
    ids = torch.where(mask.bool(), ids, torch.ones_like(ids))        # <pad> = 1
    return ids, mask


@pytest.mark.parametrize("B,S", [(12, 40), (30, 128)])
def test_cls_head_gpu_packed_matches_hf_fp32(B, S):
    hf, ours = _hf_pair(torch.float32)
    ids, mask = _batch(B, S, seed=B + S)
    with torch.no_grad():
        ref = torch.sigmoid(hf(input_ids=ids, attention_mask=mask).logits)
        p = ours.plan(mask.cuda())
        assert p is not None and p.T == int(mask.sum())               # the packed path runs
        got = ours(ids.cuda(), mask.cuda()).cpu()
    assert got.shape == (B, 28)
    assert float(ref.std()) > 0.05                                   # the comparison is not between constants
    torch.testing.assert_close(got, ref, rtol=0, atol=1e-4)


def test_cls_head_gpu_bf16_close_to_hf():
    """bf16 weights / activations (the c4 bench's precision): the six oracle labels stay within bf16 noise of the
    fp32 HF classifier."""
    from svoc.models.encoder import scores_to_oracle_vectors
    hf, ours = _hf_pair(torch.bfloat16)
    ids, mask = _batch(16, 64, seed=3)
    with torch.no_grad():
        ref = torch.sigmoid(hf(input_ids=ids, attention_mask=mask).logits)
        got = ours(ids.cuda(), mask.cuda()).float().cpu()
    # (12 bf16 layers: a few scores move by a few hundredths; on average well under one)
    torch.testing.assert_close(got, ref, rtol=0, atol=0.08)
    assert float((got - ref).abs().mean()) < 0.01
    torch.testing.assert_close(scores_to_oracle_vectors(got), scores_to_oracle_vectors(ref), rtol=0, atol=0.05)
