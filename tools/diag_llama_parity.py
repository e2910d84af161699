"""Where does the Llama (7B width) gradient differ from HF fp32?  Compares the
final hidden state (forward) and the gradients for head_dim 128 vs 64, GA 1
unfused vs GA 2 in the fusion window."""
import sys
import tempfile

import torch
import transformers

sys.path.insert(0, ".")
from distributed_lion_pytorch_amd.models.llama import LlamaForCausalLM, llama_config  # noqa: E402
from distributed_lion_pytorch_amd.ops.linear import grad_accumulation_fusion  # noqa: E402

dev = torch.device("cuda")


def rel(a, b):
    return round(float((a.float() - b.float()).norm() / b.float().norm()), 5)


def run(layers, ga, fused, hidden=4096, vocab=32000, inter=11008, heads=32, kv=None, T=1024, mb=2):
    torch.manual_seed(0)
    cfg = llama_config("llama-2-7b", num_hidden_layers=layers, hidden_size=hidden, vocab_size=vocab,
                       intermediate_size=inter, num_attention_heads=heads, num_key_value_heads=kv or heads)
    ours = LlamaForCausalLM(cfg).to(torch.bfloat16)
    with tempfile.TemporaryDirectory() as d:
        ours.save_pretrained(d)
        hf = transformers.LlamaForCausalLM.from_pretrained(d, torch_dtype=torch.float32,
                                                           attn_implementation="eager").to(dev)
    ours = ours.to(dev)
    g = torch.Generator(device=dev).manual_seed(7)
    batches = [torch.randint(0, vocab, (mb, T), device=dev, generator=g) for _ in range(ga)]
    with torch.no_grad():
        h_ours = ours.model(batches[0])
        h_hf = hf.model(input_ids=batches[0]).last_hidden_state
    losses = []
    for m, f in ((ours, fused), (hf, False)):
        ctx = grad_accumulation_fusion(True, micro_batches=ga) if f else torch.enable_grad()
        ls = []
        with ctx:
            for ids in batches:
                loss = m(input_ids=ids, labels=ids).loss
                (loss / ga).backward()
                ls.append(round(float(loss), 5))
        losses.append(ls)
    hp = dict(hf.named_parameters())
    out = {n: (rel(p.grad, hp[n].grad), round(float(p.grad.float().norm() / hp[n].grad.float().norm()), 4))
           for n, p in ours.named_parameters() if p.grad is not None}
    keys = ["lm_head.weight", "model.norm.weight", "model.embed_tokens.weight",
            "model.layers.0.self_attn.q_proj.weight", "model.layers.0.self_attn.v_proj.weight",
            "model.layers.0.mlp.down_proj.weight", "model.layers.0.input_layernorm.weight"]
    print(f"L={layers} ga={ga} fused={fused} hidden={hidden} heads={heads} kv={kv or heads} vocab={vocab}: "
          f"h_rel={rel(h_ours, h_hf)} loss ours/hf={losses} grads(rel, norm ratio)={ {k: out.get(k) for k in keys} }",
          flush=True)


run(1, 1, False)                      # D = 128
run(1, 1, False, heads=64)            # D = 64, same width
run(1, 1, False, vocab=512)
run(1, 2, True)
run(1, 1, False, hidden=1024, inter=2816, heads=8)  # D = 128, narrow
run(1, 1, False, hidden=1024, inter=2816, heads=8, kv=2)
