"""BERT encoder on the kernel path vs a plain PyTorch fp32 BERT."""
import numpy as np
import pytest
import torch

from flink_tensorflow_amd.models.zoo.bert import (BertClassifierModel, BertConfig, BertDeviceWeights,
                                                  BertEncoderPlan, HashingTokenizer, init_bert_weights,
                                                  reference_forward)


def _ids(B, S, vocab, seed=0):
    rng = np.random.default_rng(seed)
    ids = rng.integers(1000, vocab, (B, S)).astype(np.int32)
    lens = rng.integers(S // 2, S + 1, B)
    for b, n in enumerate(lens):
        ids[b, n:] = 0  # padding masked in attention
    ids[:, 0] = 101
    return torch.from_numpy(ids)


def test_bert_plan_host_matches_reference():
    cfg = BertConfig.tiny(vocab_size=2000)
    host = init_bert_weights(cfg, seed=1)
    plan = BertEncoderPlan(BertDeviceWeights(host, cfg, "cpu"), batch=3, seq=24)
    ids = _ids(3, 24, cfg.vocab_size)
    got = plan(ids)
    ref = torch.softmax(reference_forward(host, cfg, ids), -1)
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-5)


def test_tokenizer_and_model_host():
    tok = HashingTokenizer(30522, 16)
    a = tok("Hello, world!")
    assert a[0] == 101 and a[5] == 102 and (a[6:] == 0).all() and a.dtype == np.int32  # hello , world !
    m = BertClassifierModel(BertConfig.tiny(), seq_len=16, buckets=(4,), device="cpu")
    m.open()
    p = m.predict(["good movie", "bad movie", "meh"])
    assert p.shape == (3, 2)
    torch.testing.assert_close(p.sum(-1), torch.ones(3))
    m.close()


@pytest.mark.gpu
@pytest.mark.parametrize("S", [128, 77])
def test_bert_base_gpu_vs_fp32_reference(S):
    cfg = BertConfig.base()
    host = init_bert_weights(cfg, seed=2)
    dev = torch.device("cuda", 0)
    plan = BertEncoderPlan(BertDeviceWeights(host, cfg, dev), batch=4, seq=S)
    ids = _ids(4, S, cfg.vocab_size, seed=S)
    got = plan(ids.to(dev)).cpu()
    logits, hidden = reference_forward(host, cfg, ids, return_hidden=True)
    torch.testing.assert_close(got, torch.softmax(logits, -1), rtol=0, atol=3e-2)
    # the class probabilities of a random-init model are insensitive: also check the final
    # hidden states (12 layers of bf16 rounding: compare direction, per token)
    hid = plan.x.view(4, S, -1).float().cpu()
    cos = torch.nn.functional.cosine_similarity(hid, hidden, dim=-1)
    assert cos.min() > 0.98, cos.min()
    assert plan.graph is not None


@pytest.mark.gpu
@pytest.mark.parametrize("S", [100, 50, 128, 200])
def test_attention_kernel_vs_reference(S):
    from flink_tensorflow_amd.ops import kernels as K

    B, H = 3, 12
    g = torch.Generator().manual_seed(0)
    qkv = torch.randn(B * S, 3 * H * 64, generator=g).to(torch.bfloat16)
    ids = _ids(B, S, 30000).reshape(-1)
    ref = K.attention(qkv, ids, B, S, H)
    got = K.attention(qkv.cuda(), ids.cuda(), B, S, H)
    torch.testing.assert_close(got.float().cpu(), ref.float(), rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
def test_embed_ln_kernel():
    from flink_tensorflow_amd.ops import kernels as K

    V, D, S = 500, 768, 32
    word, pos, typ = (torch.randn(V, D) * 0.02).to(torch.bfloat16), (torch.randn(64, D) * 0.02).to(torch.bfloat16), \
        (torch.randn(2, D) * 0.02).to(torch.bfloat16)
    gm, bt = torch.randn(D), torch.randn(D)
    ids = torch.randint(0, V, (4 * S,), dtype=torch.int32)
    ref = K.embed_layernorm(ids, None, word, pos, typ, gm, bt, S)
    got = K.embed_layernorm(ids.cuda(), None, word.cuda(), pos.cuda(), typ.cuda(), gm.cuda(), bt.cuda(), S)
    torch.testing.assert_close(got.float().cpu(), ref.float(), rtol=2e-2, atol=5e-2)


def test_pack_tokens_host():
    from flink_tensorflow_amd.ops import kernels as K

    ids = _ids(5, 24, 2000, seed=3).reshape(5, 24)
    T = int((ids != 0).sum())
    packed, pos = torch.empty(T + 7, dtype=torch.int32), torch.empty(T + 7, dtype=torch.int32)
    cu, cls = torch.empty(6, dtype=torch.int32), torch.empty(5, dtype=torch.int32)
    assert K.pack_tokens(ids, 0, T + 7, packed, pos, cu, cls) == T
    for b in range(5):
        n = int((ids[b] != 0).sum())
        assert cu[b + 1] - cu[b] == n and cls[b] == cu[b]
        assert torch.equal(packed[cu[b]:cu[b + 1]], ids[b, :n]) and torch.equal(pos[cu[b]:cu[b + 1]], torch.arange(n, dtype=torch.int32))
    assert (packed[T:] == 0).all()


def test_packed_encoder_host_matches_padded():
    """Padding-free execution changes nothing for the real tokens: same class
    probabilities as the padded plan and as the fp32 reference."""
    from flink_tensorflow_amd.models.zoo.bert import PackedBertEncoder

    cfg = BertConfig.tiny(vocab_size=2000)
    host = init_bert_weights(cfg, seed=4)
    w = BertDeviceWeights(host, cfg, "cpu")
    ids = _ids(6, 32, cfg.vocab_size, seed=5)
    packed = PackedBertEncoder(w, 6, 32, granule=16)
    got = packed(ids)
    assert packed.current.T == packed.capacity_for(int((ids != 0).sum())) < 6 * 32
    ref = torch.softmax(reference_forward(host, cfg, ids), -1)
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(got, BertEncoderPlan(w, 6, 32)(ids), rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
def test_packed_encoder_gpu_matches_padded():
    from flink_tensorflow_amd.models.zoo.bert import PackedBertEncoder

    cfg = BertConfig.base()
    host = init_bert_weights(cfg, seed=6)
    dev = torch.device("cuda", 0)
    w = BertDeviceWeights(host, cfg, dev)
    B, S = 16, 128
    ids = _ids(B, S, cfg.vocab_size, seed=7)
    padded = BertEncoderPlan(w, B, S)
    packed = PackedBertEncoder(w, B, S, granule=256)
    p_pad = padded(ids.to(dev)).cpu()
    p_pack = packed(ids.to(dev)).cpu()
    n = int((ids != 0).sum())
    assert packed.current.T == packed.capacity_for(n) < B * S and packed.current.graph is not None
    torch.testing.assert_close(p_pack, p_pad, rtol=0, atol=2e-2)
    # the final layer only computes the first-token rows: compare them with the padded
    # plan's final hidden state at position 0
    hp = padded.x.view(B, S, -1)[:, 0].float().cpu()
    hk = packed.current.cls_in.float().cpu()
    cos = torch.nn.functional.cosine_similarity(hk, hp, dim=-1)
    assert cos.min() > 0.99, cos.min()


@pytest.mark.gpu
@pytest.mark.parametrize("S", [128, 77])
def test_packed_attention_and_pack_kernel_gpu(S):
    from flink_tensorflow_amd.ops import kernels as K

    B, H = 5, 12
    ids = _ids(B, S, 30000, seed=S).reshape(B, S)
    T = int((ids != 0).sum())
    cap = T + 100
    outs = [torch.empty(cap, dtype=torch.int32) for _ in range(2)] + [torch.empty(B + 1, dtype=torch.int32),
                                                                      torch.empty(B, dtype=torch.int32)]
    K.pack_tokens(ids, 0, cap, *outs)
    douts = [torch.full_like(t, -7).cuda() for t in outs]
    K.pack_tokens(ids.cuda(), 0, cap, *douts)
    torch.cuda.synchronize()
    for a, b in zip(outs, douts):
        assert torch.equal(a, b.cpu())
    g = torch.Generator().manual_seed(1)
    qkv = torch.randn(cap, 3 * H * 64, generator=g).to(torch.bfloat16)
    ref = K.attention(qkv, None, B, S, H, out=torch.zeros(cap, H * 64, dtype=torch.bfloat16), cu_seqlens=outs[2])
    got = K.attention(qkv.cuda(), None, B, S, H, out=torch.zeros(cap, H * 64, dtype=torch.bfloat16, device="cuda"),
                      cu_seqlens=douts[2])
    torch.testing.assert_close(got.float().cpu(), ref.float(), rtol=2e-2, atol=2e-2)
    # first-token-only attention == those rows of the full packed attention
    cls_ref = K.cls_attention(qkv, outs[2], B, H)
    cls_got = K.cls_attention(qkv.cuda(), douts[2], B, H)
    torch.testing.assert_close(cls_ref.float(), ref[outs[3].long()].float(), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(cls_got.float().cpu(), cls_ref.float(), rtol=2e-2, atol=2e-2)
