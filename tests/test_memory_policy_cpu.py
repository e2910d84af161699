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


def test_policy_counts_the_fusion_window_reserve(monkeypatch):
    """Keeping activations turns on deferred weight gradients: their operand
    budget (a quarter of HBM by default) and the 8 GB split-K accumulators are
    part of the fit check (they were invisible to it)."""
    cfg = load_config("llama-2-7b")
    tokens = 2 * 4 * 1024
    m = torch.nn.Linear(8, 8)
    _fake_device(monkeypatch, 288 << 30)
    assert memory.engine_reserve_bytes() == (8 << 30) + (72 << 30)
    # 96 GB: activations alone (~30 GB) fit 0.6 x 96 = 58 GB, with the 8 + 24 GB reserve they do not
    _fake_device(monkeypatch, 96 << 30)
    assert memory.should_checkpoint(True, "auto", cfg, tokens, m) is True
    monkeypatch.setenv("DLION_WGRAD_DEFER_GB", "1")
    assert memory.should_checkpoint(True, "auto", cfg, tokens, m) is False
