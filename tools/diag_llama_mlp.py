"""Native Llama MLP / norm stages vs fp32 math at 7B width (same bf16 inputs)."""
import sys

import torch

sys.path.insert(0, ".")
from distributed_lion_pytorch_amd.models.llama import LlamaForCausalLM, llama_config  # noqa: E402
from distributed_lion_pytorch_amd.ops import fused  # noqa: E402

dev = torch.device("cuda")


def rel(a, b):
    return round(float((a.float() - b.float()).norm() / b.float().norm()), 5)


def rms(x, w, eps):
    x = x.float()
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w.float()


for hidden, heads, inter in ((4096, 32, 11008), (1024, 8, 2816)):
    torch.manual_seed(0)
    cfg = llama_config("llama-2-7b", num_hidden_layers=1, hidden_size=hidden, num_attention_heads=heads,
                       num_key_value_heads=heads, intermediate_size=inter)
    m = LlamaForCausalLM(cfg).to(dev, torch.bfloat16).eval()
    ids = torch.randint(0, 32000, (2, 1024), device=dev, generator=torch.Generator(device=dev).manual_seed(1))
    lay = m.model.layers[0]
    line = {}
    with torch.no_grad():
        x = m.model.embed_tokens(ids)
        line["embed_std"] = round(float(x.float().std()), 4)
        h0 = fused.norm(x, lay.input_layernorm.weight, None, lay.input_layernorm.eps, rms=True)
        line["norm0"] = rel(h0, rms(x, lay.input_layernorm.weight, lay.input_layernorm.eps))
        cos, sin = m.model.rotary.tables(1024, dev, torch.bfloat16)
        a = lay.self_attn(h0, cos, sin)
        line["attn_std"] = round(float(a.float().std()), 4)
        x1, h1 = fused.dropout_add_norm(a, x, lay.post_attention_layernorm.weight, None, 1e-5, 0.0, rms=True)
        x1r = x.float() + a.float()
        line["add"] = rel(x1, x1r)
        line["addnorm"] = rel(h1, rms(x1r, lay.post_attention_layernorm.weight, 1e-5))
        mo = lay.mlp(h1)
        g = h1.float() @ lay.mlp.gate_proj.weight.float().t()
        u = h1.float() @ lay.mlp.up_proj.weight.float().t()
        mr = (torch.nn.functional.silu(g) * u) @ lay.mlp.down_proj.weight.float().t()
        line["mlp"] = rel(mo, mr)
        line["mlp_std"] = round(float(mo.float().std()), 4)
        x2, h2 = fused.dropout_add_norm(mo, x1, m.model.norm.weight, None, 1e-5, 0.0, rms=True)
        x2r = x1.float() + mo.float()
        line["final_norm"] = rel(h2, rms(x2r, m.model.norm.weight, 1e-5))
        line["model_vs_stages"] = rel(m.model(ids), h2)
    print(f"hidden={hidden}: {line}", flush=True)
