import torch
from distributed_lion_pytorch_amd.models.gpt2 import GPT2LMHeadModel, gpt2_config
from distributed_lion_pytorch_amd.ops import linear as L
torch.manual_seed(5)
cfg = gpt2_config("gpt2-tiny")
cfg.resid_pdrop = cfg.embd_pdrop = cfg.attn_pdrop = 0.0
model = GPT2LMHeadModel(cfg).to("cuda", torch.bfloat16)
ids = torch.randint(0, cfg.vocab_size, (2, 128), device="cuda")
for ckpt in (False, True):
    for fuse in (False, True):
        if ckpt: model.gradient_checkpointing_enable()
        else: model.gradient_checkpointing_disable()
        model.zero_grad(set_to_none=True)
        with L.grad_accumulation_fusion(fuse, micro_batches=2):
            for _ in range(2):
                model(input_ids=ids, labels=ids).loss.backward()
        missing = [n for n, p in model.named_parameters() if p.grad is None]
        print("ckpt", ckpt, "fuse", fuse, "missing", missing)
