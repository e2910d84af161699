"""HBM-aware checkpointing policy (trainer/memory.py): the DPO preset's
activations fit a 288 GB MI355X, a tiny-memory device still checkpoints, and
'reference' honours the flag as given."""
import types

import torch

from distributed_lion_pytorch_amd.models.registry import load_config
from distributed_lion_pytorch_amd.trainer import memory


def _fake_device(monkeypatch, total):
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 0)
    monkeypatch.setattr(torch.cuda, "get_device_properties", lambda d: types.SimpleNamespace(total_memory=total))


def test_policy(monkeypatch):
    cfg = load_config("llama-2-7b")
    tokens = 2 * 4 * 1024  # DPO preset: 4 pairs x 1024
    assert 25e9 < memory.activation_bytes(cfg, tokens) < 40e9
    m = torch.nn.Linear(8, 8)
    assert memory.should_checkpoint(False, "auto", cfg, tokens, m) is False
    assert memory.should_checkpoint(True, "reference", cfg, tokens, m) is True
    _fake_device(monkeypatch, 288 << 30)
    assert memory.should_checkpoint(True, "auto", cfg, tokens, m) is False
    _fake_device(monkeypatch, 40 << 30)
    assert memory.should_checkpoint(True, "auto", cfg, tokens, m) is True
