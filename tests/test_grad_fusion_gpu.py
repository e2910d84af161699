"""Gradient-accumulation fusion (weight grads deposited straight into
param.grad by the split-K reduction / beta=1 GEMM) vs autograd's own
accumulation over several micro-batches."""
import pytest
import torch

from distributed_lion_pytorch_amd.models.gpt2 import GPT2LMHeadModel, gpt2_config
from distributed_lion_pytorch_amd.models.llama import LlamaForCausalLM, llama_config
from distributed_lion_pytorch_amd.ops import hip
from distributed_lion_pytorch_amd.ops.linear import grad_accumulation_fusion

pytestmark = pytest.mark.gpu


def _grads(model, batches, fuse):
    model.zero_grad(set_to_none=True)
    with grad_accumulation_fusion(fuse):
        for ids in batches:
            model(input_ids=ids, labels=ids).loss.backward()
    return {n: p.grad.detach().float().clone() for n, p in model.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("family", ["gpt2", "llama"])
def test_fused_accumulation_matches_autograd(family, cuda):
    hip.require()
    torch.manual_seed(0)
    if family == "gpt2":
        cfg = gpt2_config("gpt2-tiny", n_embd=256, n_head=4, resid_pdrop=0.0, embd_pdrop=0.0, attn_pdrop=0.0)
        model = GPT2LMHeadModel(cfg)
    else:
        cfg = llama_config("llama-tiny")
        model = LlamaForCausalLM(cfg)
    model = model.to(device=cuda, dtype=torch.bfloat16).train()
    batches = [torch.randint(0, cfg.vocab_size, (2, 64), device=cuda) for _ in range(3)]
    ref = _grads(model, batches, False)
    fused = _grads(model, batches, True)
    assert ref.keys() == fused.keys()
    for n in ref:
        err = (ref[n] - fused[n]).abs().max().item() / (ref[n].abs().max().item() + 1e-8)
        assert err < 2e-2, (n, err)
