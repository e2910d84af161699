"""PhaseTimer on the GPU: the bounded-pending fold never synchronises the
device and still accounts every completed phase."""
import pytest
import torch

from distributed_lion_pytorch_amd.utils.timing import PhaseTimer


@pytest.mark.gpu
def test_fold_moves_completed_pairs_without_sync(cuda, monkeypatch):
    t = PhaseTimer(cuda)
    t.MAX_PENDING = 8
    x = torch.randn(1 << 20, device=cuda)
    for _ in range(12):
        with t.phase("work"):
            x = x * 1.0001
    torch.cuda.synchronize()
    calls = []
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: calls.append(1))
    t.step()  # 12 > 8 pending: fold, no device sync
    assert not calls
    assert sum(len(v) for v in t._events.values()) == 0 and t._wall["work"] > 0
    # pairs still in flight stay pending instead of being waited for
    big = torch.randn(4096, 4096, device=cuda)
    for _ in range(10):
        with t.phase("busy"):
            big = big @ big / 4096.0
    t.step()
    assert not calls
    monkeypatch.undo()
    tot = t.totals_ms()
    assert tot["busy"] > 0 and tot["work"] > 0
