"""Stage-by-stage native Llama attention sub-block vs fp32 math at 7B width
(each stage fed the same bf16 inputs): fused q|k|v GEMM, RoPE, flash attention
(with and without RoPE), o_proj, and the full self_attn module."""
import sys

import torch

sys.path.insert(0, ".")
from distributed_lion_pytorch_amd.models.llama import LlamaForCausalLM, llama_config  # noqa: E402
from distributed_lion_pytorch_amd.ops import fused  # noqa: E402

dev = torch.device("cuda")


def rel(a, b):
    return round(float((a.float() - b.float()).norm() / b.float().norm()), 5)


def attn_ref(q, k, v):  # q [B,T,H,D] fp32, causal
    B, T, H, D = q.shape
    rep = H // k.shape[2]
    qh, kh, vh = q.transpose(1, 2), k.transpose(1, 2).repeat_interleave(rep, 1), v.transpose(1, 2).repeat_interleave(rep, 1)
    s = (qh @ kh.transpose(-1, -2)) / D ** 0.5
    s = s.masked_fill(~torch.ones(T, T, dtype=torch.bool, device=q.device).tril(), float("-inf"))
    return (torch.softmax(s, -1) @ vh).transpose(1, 2).reshape(B, T, H * D)


for hidden, heads in ((4096, 32), (4096, 64), (1024, 8)):
    torch.manual_seed(0)
    cfg = llama_config("llama-2-7b", num_hidden_layers=1, hidden_size=hidden, num_attention_heads=heads,
                       num_key_value_heads=heads, intermediate_size=2 * hidden)
    m = LlamaForCausalLM(cfg).to(dev, torch.bfloat16).eval()
    ids = torch.randint(0, 32000, (2, 1024), device=dev, generator=torch.Generator(device=dev).manual_seed(1))
    D = hidden // heads
    att = m.model.layers[0].self_attn
    with torch.no_grad():
        x = m.model.embed_tokens(ids)
        hn = m.model.layers[0].input_layernorm(x)
        cos, sin = m.model.rotary.tables(1024, dev, torch.bfloat16)
        from distributed_lion_pytorch_amd.models.llama import _proj
        q, k, v = _proj(hn, (att.q_proj, att.k_proj, att.v_proj))
        qf = hn.float() @ att.q_proj.weight.float().t()
        line = {"qproj": rel(q, qf)}
        B, T = 2, 1024
        q4, k4, v4 = q.view(B, T, heads, D), k.view(B, T, heads, D), v.view(B, T, heads, D)
        qr = fused.rope(q4.contiguous(), cos, sin)
        qr_ref = fused.rope_reference(q4.float(), cos.float(), sin.float())
        line["rope"] = rel(qr, qr_ref)
        kr = fused.rope(k4.contiguous(), cos, sin)
        o_flash = fused.causal_attention_gqa(qr.contiguous(), kr.contiguous(), v4.contiguous())
        o_ref = attn_ref(qr.float(), kr.float(), v4.float())
        line["flash"] = rel(o_flash, o_ref)
        o_ra = fused.rope_attention(q4, k4, v4, cos, sin, 0.0)
        o_ra_ref = attn_ref(qr_ref, fused.rope_reference(k4.float(), cos.float(), sin.float()), v4.float())
        line["rope_attention"] = rel(o_ra, o_ra_ref)
        full = att(hn, cos, sin)
        full_ref = o_ra_ref.view(B, T, -1) @ att.o_proj.weight.float().t()
        line["self_attn"] = rel(full, full_ref)
        # score scale: how peaked is the attention?
        s = (qr_ref[0, :, 0].float() @ fused.rope_reference(k4.float(), cos.float(), sin.float())[0, :, 0].t()) / D ** 0.5
        line["score_std"] = round(float(s.std()), 3)
    print(f"hidden={hidden} D={D}: {line}", flush=True)
