"""Native models vs the stock HF classes (same weights -> same loss/grads),
checkpoint interop, fused-loss semantics, LoRA."""
import tempfile

import pytest
import torch
import transformers

from distributed_lion_pytorch_amd.models import lora
from distributed_lion_pytorch_amd.models.gpt2 import GPT2LMHeadModel, gpt2_config
from distributed_lion_pytorch_amd.models.llama import LlamaForCausalLM, llama_config
from distributed_lion_pytorch_amd.ops import fused


def _grads_close(a, b, tol=1e-5):
    for (na, pa), (nb, pb) in zip(a.named_parameters(), b.named_parameters()):
        assert na == nb
        if pa.grad is None and pb.grad is None:
            continue
        assert (pa.grad - pb.grad).abs().max().item() < tol, na


def test_gpt2_matches_hf_and_roundtrips():
    cfg = gpt2_config("gpt2-tiny", resid_pdrop=0.0, embd_pdrop=0.0, attn_pdrop=0.0)
    torch.manual_seed(0)
    ours = GPT2LMHeadModel(cfg)
    assert ours.lm_head.weight is ours.transformer.wte.weight
    with tempfile.TemporaryDirectory() as d:
        ours.save_pretrained(d)
        hf = transformers.GPT2LMHeadModel.from_pretrained(d)
        back = GPT2LMHeadModel.from_pretrained(d)
    ids = torch.randint(0, cfg.vocab_size, (2, 40))
    la, lb = ours(ids, labels=ids).loss, hf(ids, labels=ids).loss
    assert abs(la.item() - lb.item()) < 1e-5
    assert abs(back(ids, labels=ids).loss.item() - la.item()) < 1e-6
    la.backward()
    lb.backward()
    _grads_close(ours, hf)


def test_llama_gqa_matches_hf():
    cfg = llama_config("llama-tiny")
    torch.manual_seed(0)
    ours = LlamaForCausalLM(cfg)
    with tempfile.TemporaryDirectory() as d:
        ours.save_pretrained(d)
        hf = transformers.LlamaForCausalLM.from_pretrained(d)
    ids = torch.randint(0, cfg.vocab_size, (2, 33))
    la, lb = ours(ids, labels=ids).loss, hf(ids, labels=ids).loss
    assert abs(la.item() - lb.item()) < 1e-5
    la.backward()
    lb.backward()
    _grads_close(ours, hf)


def _small(cls, **kw):
    return cls(vocab_size=97, hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
               num_key_value_heads=2, max_position_embeddings=128, **kw)


@pytest.mark.parametrize("family", ["mistral", "qwen2", "qwen2-sliding"])
def test_mistral_qwen2_match_hf(family):
    """Loss / grads / checkpoint round trip against the HF classes.  The
    sequence (40) is longer than the sliding windows (mistral: every layer 16;
    qwen2-sliding: layer 1 of 2, window 12), so the windowed masks are covered."""
    from distributed_lion_pytorch_amd.models import llama as L
    from distributed_lion_pytorch_amd.models.registry import NATIVE
    if family == "mistral":
        cfg, ours_cls, hf_cls = _small(transformers.MistralConfig, sliding_window=16), L.MistralForCausalLM, \
            transformers.MistralForCausalLM
    elif family == "qwen2":
        cfg, ours_cls, hf_cls = _small(transformers.Qwen2Config, tie_word_embeddings=True), L.Qwen2ForCausalLM, \
            transformers.Qwen2ForCausalLM
    else:
        cfg = _small(transformers.Qwen2Config, tie_word_embeddings=True, use_sliding_window=True, sliding_window=12,
                     max_window_layers=1)
        ours_cls, hf_cls = L.Qwen2ForCausalLM, transformers.Qwen2ForCausalLM
    expect_windows = {"mistral": [16, 16], "qwen2": [0, 0], "qwen2-sliding": [0, 12]}[family]
    family = family.split("-")[0]
    assert NATIVE[family] is ours_cls
    torch.manual_seed(0)
    ours = ours_cls(cfg)
    if family == "qwen2":  # q/k/v biases, none on o_proj; tied head
        at = ours.model.layers[0].self_attn
        assert at.q_proj.bias is not None and at.o_proj.bias is None
        assert ours.lm_head.weight is ours.model.embed_tokens.weight
        with torch.no_grad():
            for layer in ours.model.layers:  # non-zero biases so the parity covers them
                for p in (layer.self_attn.q_proj, layer.self_attn.k_proj, layer.self_attn.v_proj):
                    p.bias.normal_(0, 0.1)
    with tempfile.TemporaryDirectory() as d:
        ours.save_pretrained(d)
        hf = hf_cls.from_pretrained(d)
        back = ours_cls.from_pretrained(d)
    ids = torch.randint(0, cfg.vocab_size, (2, 40))
    la, lb = ours(ids, labels=ids).loss, hf(ids, labels=ids).loss
    assert abs(la.item() - lb.item()) < 1e-5
    assert abs(back(ids, labels=ids).loss.item() - la.item()) < 1e-6
    la.backward()
    lb.backward()
    _grads_close(ours, hf)
    assert [layer.self_attn.window for layer in ours.model.layers] == expect_windows


def test_sliding_window_attention_reference():
    """The masked SDPA path (CPU / head_dims without a kernel): query q sees
    keys q - window < k <= q, and a window covering T is plain causal."""
    torch.manual_seed(0)
    q, k, v = (torch.randn(2, 37, 4, 16) for _ in range(3))
    w = 8
    out = fused.causal_attention_gqa(q, k, v, 0.0, window=w).view(2, 37, 4, 16)
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) / 4.0
    i = torch.arange(37)
    ok = (i[:, None] >= i[None, :]) & (i[:, None] - i[None, :] < w)
    ref = torch.einsum("bhqk,bkhd->bqhd", s.masked_fill(~ok, float("-inf")).softmax(-1), v)
    assert torch.allclose(out, ref, atol=1e-5)
    full = fused.causal_attention_gqa(q, k, v, 0.0)
    assert torch.equal(fused.causal_attention_gqa(q, k, v, 0.0, window=37), full)


def test_fused_ce_matches_reference_and_normalizer():
    torch.manual_seed(0)
    h = torch.randn(3, 17, 16, requires_grad=True)
    w = torch.randn(37, 16, requires_grad=True)
    labels = torch.randint(0, 37, (3, 17))
    labels[0, :5] = -100
    loss = fused.lm_head_cross_entropy(h, w, labels)
    ref = fused.reference_lm_loss(h, w, labels)
    assert abs(loss.item() - ref.item()) < 1e-5
    gh, gw = torch.autograd.grad(loss, (h, w))
    rh, rw = torch.autograd.grad(ref, (h, w))
    assert torch.allclose(gh, rh, atol=1e-5) and torch.allclose(gw, rw, atol=1e-5)
    n_valid = int((labels != -100).sum())
    s = fused.lm_head_cross_entropy(h, w, labels, normalizer=2 * n_valid)
    assert abs(s.item() - loss.item() / 2) < 1e-5


def test_lora_inject_merge_and_adapter_io():
    cfg = llama_config("llama-tiny")
    torch.manual_seed(0)
    m = LlamaForCausalLM(cfg)
    ids = torch.randint(0, cfg.vocab_size, (2, 16))
    base_loss = m(ids, labels=ids).loss.item()
    lora.inject_lora(m, lora.LoraConfig(r=4, lora_alpha=8, lora_dropout=0.0))
    trainable = lora.trainable_parameters(m)
    assert trainable and all("lora_" in n for n, p in m.named_parameters() if p.requires_grad)
    assert abs(m(ids, labels=ids).loss.item() - base_loss) < 1e-6  # B = 0 at init
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "lora_B" in n:
                p.normal_(0, 0.02)
    adapted = m(ids, labels=ids).loss.item()
    with tempfile.TemporaryDirectory() as d:
        lora.save_adapter(m, d)
        m2 = LlamaForCausalLM(cfg)
        m2.load_state_dict({k: v for k, v in m.state_dict().items() if "lora_" not in k}, strict=False)
        # base weights of m2 must equal m's base weights: copy via name mapping
        base = {n.replace(".base_layer", ""): p for n, p in m.named_parameters() if "lora_" not in n}
        with torch.no_grad():
            for n, p in m2.named_parameters():
                p.copy_(base[n])
        lora.load_adapter(m2, d)
        assert abs(m2(ids, labels=ids).loss.item() - adapted) < 1e-5
    lora.merge_and_unload(m)
    assert not any(isinstance(x, lora.LoraLinear) for x in m.modules())
    assert abs(m(ids, labels=ids).loss.item() - adapted) < 1e-4


@pytest.mark.parametrize("T,H,Hkv,D", [(64, 2, 1, 64), (16, 4, 4, 8)])
def test_attention_fallback_matches_reference(T, H, Hkv, D):
    torch.manual_seed(0)
    q = torch.randn(2, T, H, D)
    k = torch.randn(2, T, Hkv, D)
    v = torch.randn(2, T, Hkv, D)
    out = fused.causal_attention_gqa(q, k, v, 0.0)
    ref = fused.reference_attention(q, k, v, 0.0)
    assert torch.allclose(out, ref, atol=1e-5)


def test_token_logps_matches_log_softmax_cpu():
    import torch

    from distributed_lion_pytorch_amd.ops import fused

    torch.manual_seed(0)
    h = torch.randn(3, 7, 16, requires_grad=True)
    w = torch.randn(50, 16, requires_grad=True)
    labels = torch.randint(0, 50, (3, 7))
    labels[0, :3] = -100
    lp = fused.token_logps(h, w, labels)
    ref = torch.log_softmax(h @ w.t(), -1).gather(-1, labels.clamp_min(0)[..., None])[..., 0] * (labels != -100)
    assert torch.allclose(lp, ref, atol=1e-4)
    g = torch.randn(3)
    lp.sum(-1).mul(g).sum().backward()
    gh, gw = h.grad.clone(), w.grad.clone()
    h.grad = w.grad = None
    ref.sum(-1).mul(g).sum().backward()
    assert torch.allclose(gh, h.grad, atol=1e-4) and torch.allclose(gw, w.grad, atol=1e-4)


def test_rope_frequencies_stay_fp32_under_bf16_cast():
    """model.to(bfloat16) must not round the RoPE inverse frequencies (they were
    a module buffer: at position ~1000 the bf16 rounding is an angle error of
    radians).  The tables equal HF LlamaRotaryEmbedding's fp32 ones exactly."""
    from transformers.models.llama.modeling_llama import LlamaRotaryEmbedding

    from distributed_lion_pytorch_amd.models.llama import LlamaForCausalLM, llama_config

    cfg = llama_config("llama-tiny", max_position_embeddings=4096)
    m = LlamaForCausalLM(cfg).to(torch.bfloat16)
    cos, sin = m.model.rotary.tables(2048, torch.device("cpu"), torch.float32)
    hf = LlamaRotaryEmbedding(config=cfg)
    hc, hs = hf(torch.zeros(1, dtype=torch.float32), torch.arange(2048)[None])
    assert torch.equal(cos, hc[0]) and torch.equal(sin, hs[0])


def test_registry_builds_native_families_from_local_dirs(tmp_path):
    """A local HF config directory of each Llama-architecture family builds the
    native class (registry.NATIVE); an unknown type falls back to the HF class."""
    from distributed_lion_pytorch_amd.models import llama as L
    from distributed_lion_pytorch_amd.models.registry import build_model, load_config

    for name, cfg, cls in (("mistral", _small(transformers.MistralConfig, sliding_window=16), L.MistralForCausalLM),
                           ("qwen2", _small(transformers.Qwen2Config), L.Qwen2ForCausalLM),
                           ("llama", _small(transformers.LlamaConfig), L.LlamaForCausalLM)):
        d = tmp_path / name
        cfg.save_pretrained(d)
        m = build_model(load_config(str(d)))
        assert type(m) is cls, (name, type(m))
    gpt_neox = transformers.GPTNeoXConfig(vocab_size=97, hidden_size=64, num_hidden_layers=1, num_attention_heads=4,
                                          intermediate_size=128)
    gpt_neox.save_pretrained(tmp_path / "neox")
    assert type(build_model(load_config(str(tmp_path / "neox")))).__name__ == "GPTNeoXForCausalLM"
    for key in ("mistral-7b", "qwen2-0.5b", "qwen2-7b"):
        assert load_config(key).model_type == key.split("-")[0]


def test_config_overrides_rebuild_per_layer_types(tmp_path):
    """--config_overrides on a Qwen2 size: the derived per-layer attention
    types follow the overridden depth (HF refuses to save a mismatch)."""
    from distributed_lion_pytorch_amd.models.registry import load_config

    cfg = load_config("qwen2-0.5b", "num_hidden_layers=3,hidden_size=64")
    assert cfg.layer_types == ["full_attention"] * 3 and cfg.hidden_size == 64
    cfg.save_pretrained(tmp_path)
