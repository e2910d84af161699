"""LoRA adapter kernels (csrc/lora.hip, ops/fused.lora_add) against a plain
PyTorch fp32 reference of the same op, with the kernels' own dropout mask
(ops/fused.norm_dropout_keep draws the same stateless hash on the host)."""
import pytest
import torch

from distributed_lion_pytorch_amd.models.lora import LoraConfig, inject_lora
from distributed_lion_pytorch_amd.ops import fused, hip
from distributed_lion_pytorch_amd.ops import linear as L

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return (a.float() - b.float()).abs().max().item() / max(b.float().abs().max().item(), 1e-6)


@pytest.mark.parametrize("r", [8, 16])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_lora_add_matches_fp32(cuda, r, p):
    hip.require()
    torch.manual_seed(0)
    M, K, N, s = 1027, 512, 768, 2.0
    x = torch.randn(M, K, device=cuda, dtype=torch.bfloat16).requires_grad_()
    wide = torch.randn(M, 3 * N, device=cuda, dtype=torch.bfloat16)
    o = wide[:, N:2 * N].detach().requires_grad_()  # a strided column view, like a fused projection's slice
    a = (torch.randn(r, K, device=cuda) * 0.05).to(torch.bfloat16).requires_grad_()
    b = (torch.randn(N, r, device=cuda) * 0.05).to(torch.bfloat16).requires_grad_()
    seed = 1234
    out = fused._LoraAdd.apply(o, x, a, b, s, p, seed)
    dout = torch.randn(M, N, device=cuda, dtype=torch.bfloat16)
    out.backward(dout)

    keep = fused.norm_dropout_keep(M, K, p, seed, device=cuda).float() if p > 0 else torch.ones(M, K, device=cuda)
    inv = 65536.0 / (65536.0 - min(65535, int(round(p * 65536))))
    xr, orf, ar, br = (t.detach().float().requires_grad_() for t in (x, o, a, b))
    ref = orf + ((xr * keep * inv) @ ar.t()) @ br.t() * s
    ref.backward(dout.float())
    assert _rel(out, ref) < 1e-2
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(a.grad, ar.grad) < 2e-2
    assert _rel(b.grad, br.grad) < 2e-2
    assert torch.equal(o.grad, dout)


def test_lora_dropout_mask_is_fresh_per_call(cuda):
    hip.require()
    x = torch.ones(64, 256, device=cuda, dtype=torch.bfloat16)
    a = torch.ones(8, 256, device=cuda, dtype=torch.bfloat16)
    u1 = hip.ops().lora_rows(x, a, 1.0, 0.5, 1)
    u2 = hip.ops().lora_rows(x, a, 1.0, 0.5, 2)
    assert not torch.equal(u1, u2)
    # E[sum of kept * 2] == 256 per row
    assert abs(u1.float().mean().item() - 256.0) < 16.0


def _tiny_llama(cuda):
    from distributed_lion_pytorch_amd.models.llama import LlamaForCausalLM, llama_config

    torch.manual_seed(0)
    cfg = llama_config(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                       num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=128)
    model = LlamaForCausalLM(cfg).to(device=cuda, dtype=torch.bfloat16)
    inject_lora(model, LoraConfig(r=8, lora_alpha=16, lora_dropout=0.0))
    for n, prm in model.named_parameters():
        if "lora_B" in n:
            torch.nn.init.normal_(prm, std=0.02)  # non-zero B so every adapter gradient is exercised
    return model


def test_lora_llama_fused_matches_unfused(cuda, monkeypatch):
    hip.require()
    model = _tiny_llama(cuda)
    ids = torch.randint(0, 512, (2, 128), device=cuda)

    def grads(flag):
        monkeypatch.setattr(fused, "_LORA_FUSED", flag)
        model.zero_grad(set_to_none=True)
        loss = model(input_ids=ids, labels=ids).loss
        loss.backward()
        return loss.item(), {n: prm.grad.float().clone() for n, prm in model.named_parameters() if prm.grad is not None}

    l0, g0 = grads(False)
    l1, g1 = grads(True)
    assert abs(l0 - l1) < 1e-2
    assert set(g0) == set(g1) and any("lora_A" in n for n in g1)
    for n in g0:
        assert _rel(g1[n], g0[n]) < 3e-2, n


def test_lora_fusion_window_deposits(cuda):
    hip.require()
    model = _tiny_llama(cuda)
    batches = [torch.randint(0, 512, (2, 128), device=cuda) for _ in range(3)]

    def run(fuse):
        model.zero_grad(set_to_none=True)
        with L.grad_accumulation_fusion(fuse, micro_batches=len(batches)):
            for ids in batches:
                model(input_ids=ids, labels=ids).loss.backward()
        return {n: prm.grad.float().clone() for n, prm in model.named_parameters() if prm.grad is not None}

    g_plain, g_fused = run(False), run(True)
    assert set(g_plain) == set(g_fused)
    for n in g_plain:
        assert _rel(g_fused[n], g_plain[n]) < 3e-2, n


def test_lora_grads_reach_parameters_under_checkpointing(cuda):
    """Activation checkpointing (the DPO preset) + a fusion window: the adapter
    gradients must land on the Parameter objects, not on the recomputed
    aliases that ctx.saved_tensors returns under non-reentrant checkpointing."""
    hip.require()
    model = _tiny_llama(cuda)
    batches = [torch.randint(0, 512, (2, 128), device=cuda) for _ in range(2)]

    def run(ckpt):
        if ckpt:
            model.gradient_checkpointing_enable()
        else:
            model.gradient_checkpointing_disable()
        model.zero_grad(set_to_none=True)
        with L.grad_accumulation_fusion(True, micro_batches=len(batches)):
            for ids in batches:
                model(input_ids=ids, labels=ids).loss.backward()
        return {n: p.grad.float().clone() for n, p in model.named_parameters() if p.grad is not None}

    g_plain, g_ckpt = run(False), run(True)
    assert set(g_plain) == set(g_ckpt) and any("lora_A" in n for n in g_ckpt)
    for n in g_plain:
        assert _rel(g_ckpt[n], g_plain[n]) < 3e-2, n
