"""Find the copies / concatenations / adds in a LoRA Llama training step:
reports ops/linear._adjacent_views misses (fused-projection backward falling
back to torch.cat) and a torch.profiler table of the copy-like ATen ops with
their input shapes."""
import torch
from torch.profiler import ProfilerActivity, profile

from distributed_lion_pytorch_amd.models.llama import LlamaForCausalLM, llama_config
from distributed_lion_pytorch_amd.models.lora import LoraConfig, inject_lora
from distributed_lion_pytorch_amd.ops import linear as L

orig = L._adjacent_views


def traced(ts):
    out = orig(ts)
    if out is None:
        print("cat fallback:", [(tuple(t.shape), t.stride(), t.data_ptr() % 4096, t.untyped_storage().data_ptr())
                                for t in ts if t is not None])
    return out


L._adjacent_views = traced
import sys

if len(sys.argv) > 1 and sys.argv[1] == "7b":  # Llama-2-7B layer shapes, 2 layers, the SFT micro-batch
    cfg = llama_config("llama-2-7b", num_hidden_layers=2)
    B, T = 4, 1024
else:
    cfg = llama_config("llama-tiny", hidden_size=512, intermediate_size=1024, num_attention_heads=4,
                       num_key_value_heads=4)
    B, T = 2, 256
model = LlamaForCausalLM(cfg).to("cuda", torch.bfloat16)
inject_lora(model, LoraConfig(r=8, lora_alpha=16, lora_dropout=0.05))
model.train()
ids = torch.randint(0, 512, (B, T), device="cuda")
model(input_ids=ids, labels=ids).loss.backward()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU], record_shapes=True) as prof:
    model(input_ids=ids, labels=ids).loss.backward()
    torch.cuda.synchronize()
keys = ("copy", "cat", "add", "contiguous", "clone", "to")
for e in prof.key_averages(group_by_input_shape=True):
    if any(k in e.key for k in keys) and e.key.startswith("aten::"):
        print(f"{e.count:4d} {e.key:28s} {str(e.input_shapes)[:150]}")
print("done")
