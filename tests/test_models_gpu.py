"""Native models on MI355X (HIP attention / xent / Lion kernels) vs the stock
HF classes with the same weights, plus a short training run on the GPU."""
import pytest
import torch
import transformers

from distributed_lion_pytorch_amd import Lion
from distributed_lion_pytorch_amd.models.gpt2 import GPT2LMHeadModel, gpt2_config
from distributed_lion_pytorch_amd.models.llama import LlamaForCausalLM, llama_config
from distributed_lion_pytorch_amd.ops import hip

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return (a - b).abs().max().item() / (b.abs().max().item() + 1e-8)


@pytest.mark.parametrize("kind", ["gpt2", "llama", "mistral", "qwen2"])
def test_native_matches_hf_on_gpu(kind, cuda, tmp_path):
    hip.require()
    torch.manual_seed(0)
    if kind == "gpt2":
        cfg = gpt2_config("gpt2-tiny", resid_pdrop=0.0, embd_pdrop=0.0, attn_pdrop=0.0)
        ours = GPT2LMHeadModel(cfg)
        ours.save_pretrained(tmp_path)
        hf = transformers.GPT2LMHeadModel.from_pretrained(tmp_path)
    elif kind == "llama":
        cfg = llama_config("llama-tiny")
        ours = LlamaForCausalLM(cfg)
        ours.save_pretrained(tmp_path)
        hf = transformers.LlamaForCausalLM.from_pretrained(tmp_path)
    else:  # Llama-architecture families: GQA + sliding window (mistral), q/k/v biases + tied head (qwen2)
        from distributed_lion_pytorch_amd.models import llama as L
        kw = dict(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
                  num_key_value_heads=2, max_position_embeddings=512)
        if kind == "mistral":
            cfg, cls, hf_cls = transformers.MistralConfig(sliding_window=256, **kw), L.MistralForCausalLM, \
                transformers.MistralForCausalLM
        else:
            cfg, cls, hf_cls = transformers.Qwen2Config(tie_word_embeddings=True, **kw), L.Qwen2ForCausalLM, \
                transformers.Qwen2ForCausalLM
        ours = cls(cfg)
        with torch.no_grad():
            for n, p in ours.named_parameters():
                if n.endswith("proj.bias"):
                    p.normal_(0, 0.1)
        ours.save_pretrained(tmp_path)
        hf = hf_cls.from_pretrained(tmp_path)
    ours, hf = ours.to(cuda, torch.bfloat16), hf.to(cuda, torch.bfloat16)
    ids = torch.randint(0, cfg.vocab_size, (4, 128), device=cuda)
    la = ours(ids, labels=ids).loss
    lb = hf(ids, labels=ids).loss
    assert abs(la.item() - lb.item()) < 2e-2
    la.backward()
    lb.backward()
    for (n, p), (_, q) in zip(ours.named_parameters(), hf.named_parameters()):
        if p.grad is not None and q.grad is not None and q.grad.abs().max() > 0:
            assert _rel(p.grad.float(), q.grad.float()) < 0.1, n


def test_gpt2_trains_with_lion_on_gpu(cuda):
    hip.require()
    torch.manual_seed(0)
    cfg = gpt2_config("gpt2-tiny")
    m = GPT2LMHeadModel(cfg).to(cuda, torch.bfloat16)
    opt = Lion(m.parameters(), lr=3e-3, weight_decay=0.0)
    ids = torch.randint(0, 64, (8, 128), device=cuda)  # learnable: small token range
    first = None
    for _ in range(30):
        loss = m(ids, labels=ids).loss
        first = loss.item() if first is None else first
        opt.zero_grad()
        loss.backward()
        opt.step()
    assert loss.item() < first - 1.0
