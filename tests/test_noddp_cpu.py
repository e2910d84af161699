"""the async trainers no longer let accelerate wrap the
model in DDP (whose reducer allocates a never-used flat copy of every trainable
gradient; the reference wraps only to switch DDP off,
/root/reference/async_trainer.py:15).  Replicas are initialised by one
coalesced broadcast instead of DDP's constructor broadcast; ``--lion_ddp_wrap``
restores the wrap."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from dist_utils import run_world  # noqa: E402


class _Tiny(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.l1 = torch.nn.Linear(16, 32)
        self.l2 = torch.nn.Linear(32, 16)
        self.register_buffer("scale", torch.ones(16))

    def forward(self, x, labels=None):
        y = self.l2(torch.tanh(self.l1(x))) * self.scale
        return {"loss": ((y - labels) ** 2).mean()}


def _rank(rank, world, out_dir, wrap):
    from torch.nn.parallel import DistributedDataParallel as DDP

    from distributed_lion_pytorch_amd.trainer.async_trainer import AsyncTrainer, AsyncTrainingArguments

    torch.manual_seed(100 + rank)  # a different initialisation on every rank: only the broadcast aligns them
    model = _Tiny()
    with torch.no_grad():
        model.scale.fill_(1.0 + rank)
    g = torch.Generator().manual_seed(7 + rank)
    data = [{"x": torch.randn(16, generator=g), "labels": torch.randn(16, generator=g)} for _ in range(32)]
    args = AsyncTrainingArguments(output_dir=os.path.join(out_dir, f"r{rank}"), use_cpu=True, max_steps=3,
                                  per_device_train_batch_size=4, learning_rate=1e-2, lion=True, async_grad=True,
                                  report_to="none", save_strategy="no", ddp_backend="gloo", logging_steps=1,
                                  lion_ddp_wrap=wrap, dataloader_num_workers=0)
    tr = AsyncTrainer(model=model, args=args, train_dataset=data)
    tr.train()
    end = [h for h in tr.state.log_history if "replicas_identical" in h][-1]
    return {"ddp": float(isinstance(tr.model_wrapped, DDP)), "identical": end["replicas_identical"],
            "logged_ddp": end["ddp_wrapped"], "w": model.l1.weight.detach().clone(),
            "scale": model.scale.detach().clone()}


@pytest.mark.parametrize("wrap", [False, True])
def test_async_trainer_without_ddp_wrap(tmp_path, wrap):
    r0, r1 = run_world(_rank, 2, str(tmp_path), wrap)
    assert r0["ddp"] == r1["ddp"] == float(wrap) == r0["logged_ddp"]
    assert r0["identical"] == 1.0
    assert torch.equal(r0["w"], r1["w"])  # rank 1's different init was replaced by rank 0's, then voted
    assert torch.equal(r0["scale"], r1["scale"]) and r0["scale"][0] == 1.0  # buffers too
