"""4-bit frozen bases (models/quant.py, ops/quant.py) on the CPU: the
quantization contract (64-element blocks, fp32 absmax, nearest codebook
entry, first element in the high nibble), Linear4bit == nn.Linear over the
dequantized weight, QLoRA training through the fused Llama projections, LoRA
merge into a 4-bit base, and the ``--load_in_4bit`` entrypoints.

Reference: bitsandbytes 4-bit NF4 bases of /root/reference/sft_llama2.py:141-154
and dpo_llama2.py:133-152.  bitsandbytes is not installed, so byte-level parity
with its checkpoints is unpinned; the codebooks are its published tables."""
import os

import pytest
import torch
import torch.nn as nn

from distributed_lion_pytorch_amd.models.llama import LlamaForCausalLM, llama_config
from distributed_lion_pytorch_amd.models.lora import LoraConfig, LoraLinear, inject_lora, merge_and_unload
from distributed_lion_pytorch_amd.models.quant import (Linear4bit, QuantConfig, dequantize_model, quantize_model,
                                                       quantized_bytes)
from distributed_lion_pytorch_amd.ops.quant import (NF4_CODE, code_tensor, dequantize_4bit, dequantize_4bit_ref,
                                                    quantize_4bit, quantize_4bit_ref)


@pytest.mark.parametrize("qt", ["nf4", "fp4"])
def test_quantize_contract(qt):
    torch.manual_seed(0)
    w = torch.randn(96, 128)
    code = code_tensor(qt)
    q, absmax = quantize_4bit(w, code)
    assert q.dtype == torch.uint8 and q.numel() == w.numel() // 2
    assert torch.equal(absmax, w.reshape(-1, 64).abs().amax(1))
    idx = torch.stack([q >> 4, q & 15], 1).reshape(-1, 64).long()  # high nibble first
    x = w.reshape(-1, 64) / absmax[:, None]
    # every element maps to a nearest codebook entry
    err = (x - code[idx]).abs()
    best = (x.unsqueeze(-1) - code).abs().amin(-1)
    assert torch.equal(err, best)
    d = dequantize_4bit(q, absmax, code, w.shape, torch.float32)
    assert torch.equal(d, (code[idx] * absmax[:, None]).reshape(w.shape))
    rel = ((d - w).norm() / w.norm()).item()
    assert rel < (0.11 if qt == "nf4" else 0.14)
    # the block max is represented exactly (code has +-1)
    assert torch.allclose(d.reshape(-1, 64).abs().amax(1), absmax)


def test_zero_block_and_nf4_table():
    assert len(NF4_CODE) == 16 and NF4_CODE[7] == 0.0 and NF4_CODE[0] == -1.0 and NF4_CODE[15] == 1.0
    w = torch.zeros(2, 64)
    w[1, 5] = 3.0
    q, a = quantize_4bit_ref(w, code_tensor("nf4"))
    assert a[0] == 0 and a[1] == 3.0
    d = dequantize_4bit_ref(q, a, code_tensor("nf4"), torch.float32).view(2, 64)
    assert torch.equal(d, w)


def test_linear4bit_matches_dequantized_linear():
    torch.manual_seed(0)
    lin = nn.Linear(128, 192, bias=True)
    q4 = Linear4bit.from_linear(lin, "nf4")
    ref = nn.Linear(128, 192, bias=True)
    with torch.no_grad():
        ref.weight.copy_(q4.dequantize(torch.float32))
        ref.bias.copy_(lin.bias)
    x = torch.randn(5, 7, 128, requires_grad=True)
    xr = x.detach().clone().requires_grad_()
    y = q4(x)
    yr = ref(xr)
    assert torch.allclose(y, yr, atol=1e-5)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    assert torch.allclose(x.grad, xr.grad, atol=1e-5)
    assert all(not p.requires_grad for p in q4.parameters())
    # state_dict round trip
    q4b = Linear4bit(128, 192, bias=True, compute_dtype=torch.float32)
    q4b.load_state_dict(q4.state_dict())
    assert torch.equal(q4b.dequantize(), q4.dequantize())


def _tiny(seed=0):
    torch.manual_seed(seed)
    return LlamaForCausalLM(llama_config("llama-tiny"))


def test_qlora_equals_lora_on_dequantized_base():
    """A 4-bit base + LoRA computes the same loss and adapter gradients as
    bf16/fp32 LoRA on the dequantized weights (fused q/k/v, gate/up path)."""
    m4 = quantize_model(_tiny(), QuantConfig())
    assert isinstance(m4.model.layers[0].mlp.gate_proj, Linear4bit)
    assert type(m4.lm_head) is nn.Linear  # skipped like bitsandbytes
    mr = dequantize_model(quantize_model(_tiny(), QuantConfig()))
    assert type(mr.model.layers[0].mlp.gate_proj) is nn.Linear
    cfg = LoraConfig(r=8, lora_alpha=16, lora_dropout=0.0, target_modules=["q_proj", "v_proj", "up_proj"])
    torch.manual_seed(1)
    inject_lora(m4, cfg)
    torch.manual_seed(1)
    inject_lora(mr, cfg)
    pr_by_name = dict(mr.named_parameters())
    for n, p in m4.named_parameters():
        if "lora_" in n:
            with torch.no_grad():
                if "lora_B" in n:
                    p.normal_(0, 0.02)
                pr_by_name[n].copy_(p)
    ids = torch.randint(0, 512, (2, 64))
    l4 = m4(input_ids=ids, labels=ids).loss
    lr = mr(input_ids=ids, labels=ids).loss
    assert torch.allclose(l4, lr, atol=1e-5)
    l4.backward()
    lr.backward()
    g4 = {n: p.grad for n, p in m4.named_parameters() if p.requires_grad}
    gr = {n: p.grad for n, p in mr.named_parameters() if p.requires_grad}
    assert set(g4) == set(gr) and len(g4) == 12
    for n in g4:
        assert torch.allclose(g4[n], gr[n], atol=1e-5, rtol=1e-4), n


def test_qlora_merge_and_memory():
    m = quantize_model(_tiny(), QuantConfig())
    n_lin = sum(l.in_features * l.out_features for l in m.modules() if isinstance(l, Linear4bit))
    assert quantized_bytes(m) < 0.6 * n_lin  # ~0.5625 B/param
    inject_lora(m, LoraConfig(r=8, lora_alpha=16, lora_dropout=0.0))
    lora = m.model.layers[0].self_attn.q_proj
    assert isinstance(lora, LoraLinear) and isinstance(lora.base_layer, Linear4bit)
    with torch.no_grad():
        lora.lora_B.weight.normal_(0, 0.05)
    ids = torch.randint(0, 512, (1, 64))
    before = m(input_ids=ids, labels=ids).loss
    merged = merge_and_unload(dequantize_model(m))
    assert type(merged.model.layers[0].self_attn.q_proj) is nn.Linear
    after = merged(input_ids=ids, labels=ids).loss
    assert torch.allclose(before, after, atol=1e-4)


def test_sft_dpo_entrypoints_load_in_4bit(tmp_path):
    import dpo_llama2
    import sft_llama2

    sft_out = str(tmp_path / "sft")
    sft_llama2.main(["--model_name", "llama-tiny", "--synthetic_data", "--synthetic_samples", "100", "--seq_length", "64",
                     "--output_dir", sft_out, "--max_steps", "2", "--per_device_train_batch_size", "2",
                     "--learning_rate", "1e-3", "--lion", "--async_grad", "--report_to", "none", "--use_cpu",
                     "--torch_dtype", "float32", "--load_in_4bit", "--save_strategy", "no"])
    merged = os.path.join(sft_out, "final_merged_checkpoint")
    assert os.path.isfile(os.path.join(sft_out, "final_checkpoint", "adapter_model.safetensors"))
    from safetensors.torch import load_file

    sd = load_file(os.path.join(merged, "model.safetensors"))
    assert "model.layers.0.self_attn.q_proj.weight" in sd and not any("qweight" in k for k in sd)
    tr = dpo_llama2.main(["--model_name_or_path", merged, "--synthetic_data", "--synthetic_samples", "60", "--max_length", "1024",
                          "--max_prompt_length", "256", "--output_dir", str(tmp_path / "dpo"), "--max_steps", "1",
                          "--per_device_train_batch_size", "2", "--gradient_accumulation_steps", "1", "--lion",
                          "--async_grad", "--use_cpu", "--torch_dtype", "float32", "--eval_steps", "0",
                          "--warmup_steps", "1", "--logging_steps", "1", "--load_in_4bit"])
    assert tr.state.global_step == 1
    assert isinstance(tr.model.model.layers[0].mlp.down_proj, Linear4bit)


def test_linear4bit_survives_model_dtype_cast():
    m = quantize_model(_tiny(), QuantConfig())
    l4 = m.model.layers[0].self_attn.k_proj
    before = l4.dequantize(torch.float32)
    m.to(dtype=torch.bfloat16)
    assert l4.absmax.dtype == torch.float32 and l4.quant_map.dtype == torch.float32
    assert l4.qweight.dtype == torch.uint8
    assert torch.equal(l4.dequantize(torch.float32), before)


def test_quantize_after_lora_keeps_adapters_trainable():
    m = _tiny()
    inject_lora(m, LoraConfig(r=8, lora_alpha=16, lora_dropout=0.0))
    quantize_model(m, QuantConfig())
    q = m.model.layers[0].self_attn.q_proj
    assert isinstance(q.base_layer, Linear4bit)
    assert type(q.lora_A) is nn.Linear and q.lora_A.weight.requires_grad
    ids = torch.randint(0, 512, (1, 64))
    m(input_ids=ids, labels=ids).loss.backward()
    assert q.lora_B.weight.grad is not None
