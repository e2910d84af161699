"""Native Llama (bf16, GPU) vs HF fp32 on GPU and on CPU vs a hand-written
fp32 pipeline: which reference is off?  1 layer, 7B width, T = 1024."""
import sys
import tempfile

import torch
import transformers

sys.path.insert(0, ".")
from distributed_lion_pytorch_amd.models.llama import LlamaForCausalLM, llama_config  # noqa: E402
from distributed_lion_pytorch_amd.ops import fused  # noqa: E402

dev = torch.device("cuda")


def rel(a, b):
    return round(float((a.float().cpu() - b.float().cpu()).norm() / b.float().cpu().norm()), 6)


def rms(x, w, eps=1e-5):
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w


def manual(sd, ids, heads, cos, sin):
    g = {k: v.float() for k, v in sd.items()}
    p = "model.layers.0."
    x = g["model.embed_tokens.weight"][ids]
    h = rms(x, g[p + "input_layernorm.weight"])
    B, T, C = h.shape
    D = C // heads
    q = (h @ g[p + "self_attn.q_proj.weight"].t()).view(B, T, heads, D)
    k = (h @ g[p + "self_attn.k_proj.weight"].t()).view(B, T, heads, D)
    v = (h @ g[p + "self_attn.v_proj.weight"].t()).view(B, T, heads, D)
    q, k = fused.rope_reference(q, cos, sin), fused.rope_reference(k, cos, sin)
    s = (q.transpose(1, 2) @ k.transpose(1, 2).transpose(-1, -2)) / D ** 0.5
    s = s.masked_fill(~torch.ones(T, T, dtype=torch.bool, device=s.device).tril(), float("-inf"))
    o = (torch.softmax(s, -1) @ v.transpose(1, 2)).transpose(1, 2).reshape(B, T, C)
    x1 = x + o @ g[p + "self_attn.o_proj.weight"].t()
    h1 = rms(x1, g[p + "post_attention_layernorm.weight"])
    m = (torch.nn.functional.silu(h1 @ g[p + "mlp.gate_proj.weight"].t()) * (h1 @ g[p + "mlp.up_proj.weight"].t())) \
        @ g[p + "mlp.down_proj.weight"].t()
    return rms(x1 + m, g["model.norm.weight"])


torch.manual_seed(0)
heads = 32
cfg = llama_config("llama-2-7b", num_hidden_layers=1)
ours = LlamaForCausalLM(cfg).to(torch.bfloat16)
sd = {k: v.clone() for k, v in ours.state_dict().items()}
with tempfile.TemporaryDirectory() as d:
    ours.save_pretrained(d)
    hf_gpu = transformers.LlamaForCausalLM.from_pretrained(d, torch_dtype=torch.float32,
                                                           attn_implementation="eager").to(dev)
    hf_cpu = transformers.LlamaForCausalLM.from_pretrained(d, torch_dtype=torch.float32, attn_implementation="eager")
print("hf config rope:", getattr(hf_gpu.config, "rope_parameters", None), getattr(hf_gpu.config, "rope_theta", None),
      "eps", hf_gpu.config.rms_norm_eps, flush=True)
ours = ours.to(dev).eval()
ids = torch.randint(0, 32000, (1, 1024), generator=torch.Generator().manual_seed(1))
cos, sin = ours.model.rotary.tables(1024, torch.device("cpu"), torch.float32)
with torch.no_grad():
    o = ours.model(ids.to(dev))
    a = hf_gpu.model(input_ids=ids.to(dev)).last_hidden_state
    b = hf_cpu.model(input_ids=ids).last_hidden_state
    man_cpu = manual(sd, ids, heads, cos, sin)
    man_gpu = manual({k: v.to(dev) for k, v in sd.items()}, ids.to(dev), heads, cos.to(dev), sin.to(dev))
print("ours_vs_hfgpu", rel(o, a), "ours_vs_hfcpu", rel(o, b), "hfgpu_vs_hfcpu", rel(a, b), flush=True)
print("manual_cpu_vs_hfcpu", rel(man_cpu, b), "manual_gpu_vs_manual_cpu", rel(man_gpu, man_cpu),
      "ours_vs_manual_cpu", rel(o, man_cpu), "hfgpu_vs_manual_cpu", rel(a, man_cpu), flush=True)
print("tf32 flags", torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32,
      torch.get_float32_matmul_precision(), flush=True)
