"""The per-shape GEMM choice (ops/linear.gemm_fwd / gemm_dgrad) is a pure
dispatch: off the GPU (or below the size threshold) it is ATen's product."""
import torch

from distributed_lion_pytorch_amd.ops import linear as L


def test_cpu_fallbacks_are_aten():
    torch.manual_seed(0)
    x = torch.randn(64, 32)
    w = torch.randn(48, 32)
    b = torch.randn(48)
    assert torch.equal(L.gemm_fwd(x, w), torch.nn.functional.linear(x, w))
    assert torch.equal(L.gemm_fwd(x, w, b), torch.nn.functional.linear(x, w, b))
    dy = torch.randn(64, 48)
    assert torch.equal(L.gemm_dgrad(dy, w, True), dy @ w)
    assert torch.equal(L.gemm_dgrad(dy, w, False), dy @ w)
    assert not L._GEMM_PICK  # nothing was timed on the CPU
    t = torch.randn(40, 24)
    assert torch.equal(L.fast_transpose(t), t.t().contiguous())
    padded = L.fast_transpose(t, 48)
    assert padded.shape == (24, 48) and torch.equal(padded[:, :40], t.t()) and (padded[:, 40:] == 0).all()
