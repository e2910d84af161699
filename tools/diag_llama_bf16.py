"""Is the native Llama's deviation from HF fp32 at 7B width just bf16?  On one
GPU, 1 decoder layer, T=1024: HF bf16 vs HF fp32 and native vs HF fp32, at the
embedding+input norm, attention sub-block, full layer and final hidden state."""
import sys
import tempfile

import torch
import transformers

sys.path.insert(0, ".")
from distributed_lion_pytorch_amd.models.llama import LlamaForCausalLM, llama_config  # noqa: E402

dev = torch.device("cuda")


def rel(a, b):
    return round(float((a.float() - b.float()).norm() / b.float().norm()), 5)


for hidden, heads, inter in ((4096, 32, 11008), (4096, 64, 11008), (1024, 8, 2816)):
    torch.manual_seed(0)
    cfg = llama_config("llama-2-7b", num_hidden_layers=1, hidden_size=hidden, num_attention_heads=heads,
                       num_key_value_heads=heads, intermediate_size=inter)
    ours = LlamaForCausalLM(cfg).to(torch.bfloat16)
    with tempfile.TemporaryDirectory() as d:
        ours.save_pretrained(d)
        hf32 = transformers.LlamaForCausalLM.from_pretrained(d, torch_dtype=torch.float32,
                                                             attn_implementation="eager").to(dev)
        hf16 = transformers.LlamaForCausalLM.from_pretrained(d, torch_dtype=torch.bfloat16,
                                                             attn_implementation="eager").to(dev)
    ours = ours.to(dev).eval()
    ids = torch.randint(0, 32000, (2, 1024), device=dev, generator=torch.Generator(device=dev).manual_seed(1))
    res = {}
    with torch.no_grad():
        for name, m in (("hf32", hf32), ("hf16", hf16)):
            x = m.model.embed_tokens(ids)
            pos = torch.arange(1024, device=dev)[None]
            ce = m.model.rotary_emb(x, pos)
            lay = m.model.layers[0]
            hn = lay.input_layernorm(x)
            a = lay.self_attn(hn, position_embeddings=ce, attention_mask=None)[0]
            x1 = x + a
            m1 = lay.mlp(lay.post_attention_layernorm(x1))
            res[name] = dict(norm_in=hn, attn=a, layer=x1 + m1, final=m.model(input_ids=ids).last_hidden_state)
        x = ours.model.embed_tokens(ids)
        cos, sin = ours.model.rotary.tables(1024, dev, x.dtype)
        lay = ours.model.layers[0]
        hn = lay.input_layernorm(x)
        a = lay.self_attn(hn, cos, sin)
        x1 = x + a
        res["ours"] = dict(norm_in=hn, attn=a, layer=x1 + lay.mlp(lay.post_attention_layernorm(x1)),
                           final=ours.model(ids))
    print(f"hidden={hidden} D={hidden // heads}:", flush=True)
    for k in ("norm_in", "attn", "layer", "final"):
        print(f"   {k:8s} hf_bf16 {rel(res['hf16'][k], res['hf32'][k]):8.5f}   ours {rel(res['ours'][k], res['hf32'][k]):8.5f}"
              f"   ours-vs-hf_bf16 {rel(res['ours'][k], res['hf16'][k]):8.5f}", flush=True)
