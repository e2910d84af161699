"""Deferred weight-gradient bookkeeping (ops/linear.py _defer_wgrad /
_run_deferred) on the CPU with a stub TN GEMM: the in-place guard compares
each kept operand with its own version -- operands whose versions differ
(the LM head's logits were rewritten in place by the softmax before being
kept, its s * h operand is fresh) must not trip it, a real in-place change
after the deferral must."""
import types

import pytest
import torch

from distributed_lion_pytorch_amd.ops import hip, linear


@pytest.fixture
def stub(monkeypatch):
    calls = []
    ops = types.SimpleNamespace(gemm_tn_=lambda a, b, out, acc: calls.append((len(a), acc)))
    monkeypatch.setattr(hip, "ops", lambda: ops)
    monkeypatch.setattr(linear, "_WDEFER_ON", True)
    monkeypatch.setattr(linear, "_wdefer_budget", lambda: 1 << 30)
    monkeypatch.setattr(linear, "_ensure_acc", lambda params, cols, shape, dev: linear._ST.acc.setdefault(
        tuple(id(p) for p in params), [None, torch.zeros(shape)]) is not None)
    linear.begin_fusion_window(4)
    yield calls
    linear._ST.pending.clear()
    linear._drop_deferred()
    linear._ST.acc.clear()
    linear._ST.fuse["on"], linear._ST.fuse["multi"] = False, True


def _operands():
    logits = torch.randn(16, 8)
    logits.mul_(1.0)  # version 1, like the softmax rewrite of the logits
    return logits, torch.randn(16, 4)  # version 0


def test_differing_operand_versions_do_not_trip_the_guard(stub):
    w = torch.nn.Parameter(torch.zeros(8, 4))
    for _ in range(3):
        a, b = _operands()
        assert linear._defer_wgrad([w], [(0, 32)], a, b, 1)
    linear._run_all_deferred()
    assert stub == [(3, False)]


def test_in_place_change_after_deferral_is_caught(stub):
    w = torch.nn.Parameter(torch.zeros(8, 4))
    kept = []
    for _ in range(2):
        a, b = _operands()
        kept.append(b)
        assert linear._defer_wgrad([w], [(0, 32)], a, b, 1)
    kept[1].add_(1.0)
    with pytest.raises(RuntimeError, match=r"micro-batch 1, operand b"):
        linear._run_all_deferred()
