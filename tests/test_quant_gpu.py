"""4-bit quantization kernels (csrc/quant.hip) against the PyTorch oracle of
ops/quant.py (identical indices / absmax, bit-identical expansion), and the
Linear4bit / QLoRA path on the GPU against fp32 PyTorch references."""
import pytest
import torch
import torch.nn as nn

from distributed_lion_pytorch_amd.models.llama import LlamaForCausalLM, llama_config
from distributed_lion_pytorch_amd.models.lora import LoraConfig, inject_lora
from distributed_lion_pytorch_amd.models.quant import Linear4bit, QuantConfig, dequantize_model, quantize_model
from distributed_lion_pytorch_amd.ops import hip
from distributed_lion_pytorch_amd.ops.quant import (code_tensor, dequantize_4bit, dequantize_4bit_ref, quantize_4bit,
                                                    quantize_4bit_ref)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("qt", ["nf4", "fp4"])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
def test_quant4_kernel_matches_oracle(cuda, qt, dt):
    hip.require()
    torch.manual_seed(0)
    w = (torch.randn(384, 1024, device=cuda) * 0.02).to(dt)
    w[3, :64] = 0  # an all-zero block
    code = code_tensor(qt, cuda)
    q, a = quantize_4bit(w, code)
    qr, ar = quantize_4bit_ref(w, code)
    assert torch.equal(a, ar)
    assert torch.equal(q, qr)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
def test_dequant4_kernel_bit_exact(cuda, dt):
    hip.require()
    torch.manual_seed(0)
    # 20000 x 4096: 2.56M work items > one grid (exercises the grid-stride loop)
    w = torch.randn(20000, 4096, device=cuda, dtype=torch.bfloat16)
    code = code_tensor("nf4", cuda)
    q, a = quantize_4bit(w, code)
    d = dequantize_4bit(q, a, code, w.shape, dt)
    assert torch.equal(d.view(-1), dequantize_4bit_ref(q, a, code, dt))
    # into a row block of a bigger buffer (the fused projection layout)
    big = torch.full((20000 + 128, 4096), 7.0, device=cuda, dtype=dt)
    dequantize_4bit(q, a, code, w.shape, dt, out=big[64:64 + 20000])
    assert torch.equal(big[64:64 + 20000], d)
    assert (big[:64] == 7).all() and (big[-64:] == 7).all()


def test_linear4bit_fwd_bwd_vs_fp32(cuda):
    hip.require()
    torch.manual_seed(0)
    lin = nn.Linear(1024, 768, bias=False, device=cuda, dtype=torch.bfloat16)
    q4 = Linear4bit.from_linear(lin)
    wref = q4.dequantize(torch.float32)
    x = torch.randn(4, 256, 1024, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    y = q4(x)
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().float().requires_grad_()
    yr = xr @ wref.t()
    yr.backward(g.float())
    assert (y.float() - yr).abs().max().item() < 2e-2 * yr.abs().max().item()
    assert (x.grad.float() - xr.grad).abs().max().item() < 2e-2 * xr.grad.abs().max().item()


def test_qlora_llama_gpu_matches_dequantized(cuda):
    """QLoRA step on the GPU (fused q/k/v + gate/up 4-bit GEMMs, LoRA kernels)
    equals LoRA over the dequantized bf16 weights."""
    hip.require()
    cfg = llama_config("llama-tiny", hidden_size=256, intermediate_size=768, num_attention_heads=4,
                       num_key_value_heads=2)

    def make():
        torch.manual_seed(0)
        with torch.device(cuda):
            return LlamaForCausalLM(cfg).to(torch.bfloat16)

    m4 = quantize_model(make(), QuantConfig(bnb_4bit_compute_dtype=torch.bfloat16))
    mr = dequantize_model(quantize_model(make(), QuantConfig(bnb_4bit_compute_dtype=torch.bfloat16)))
    lc = LoraConfig(r=8, lora_alpha=16, lora_dropout=0.0, target_modules=["q_proj", "v_proj"])
    torch.manual_seed(1)
    inject_lora(m4, lc)
    torch.manual_seed(1)
    inject_lora(mr, lc)
    byname = dict(mr.named_parameters())
    with torch.no_grad():
        for n, p in m4.named_parameters():
            if "lora_" in n:
                if "lora_B" in n:
                    p.normal_(0, 0.02)
                byname[n].copy_(p)
    ids = torch.randint(0, cfg.vocab_size, (2, 128), device=cuda)
    l4 = m4(input_ids=ids, labels=ids).loss
    lr = mr(input_ids=ids, labels=ids).loss
    assert abs(l4.item() - lr.item()) < 1e-2
    l4.backward()
    lr.backward()
    for n, p in m4.named_parameters():
        if p.requires_grad:
            gr = byname[n].grad.float()
            assert (p.grad.float() - gr).abs().max().item() <= 5e-2 * gr.abs().max().item() + 1e-6, n


def test_dequant4_transposed_into_column_blocks(cuda):
    """The transposed expansion (input-gradient GEMM layout) equals the plain
    one transposed, written into a column block of a concatenated W^T."""
    hip.require()
    torch.manual_seed(1)
    code = code_tensor("nf4", cuda)
    w = torch.randn(1024, 768, device=cuda, dtype=torch.bfloat16)
    q, a = quantize_4bit(w, code)
    full = dequantize_4bit(q, a, code, w.shape, torch.bfloat16)
    big = torch.full((768, 3 * 1024), 5.0, device=cuda, dtype=torch.bfloat16)
    hip.ops().dequant4_t_(q, a, code, big[:, 1024:2048])
    assert torch.equal(big[:, 1024:2048], full.t())
    assert (big[:, :1024] == 5).all() and (big[:, 2048:] == 5).all()
