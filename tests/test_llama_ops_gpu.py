"""Llama-path kernels vs fp32 PyTorch references: wide-row fused residual +
RMSNorm/LayerNorm (C = 2048..8192, multi-wave rows), SwiGLU and RoPE."""
import pytest
import torch

from distributed_lion_pytorch_amd.ops import fused, hip

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return (a.float() - b.float()).abs().max().item() / (b.float().abs().max().item() + 1e-6)


@pytest.mark.parametrize("C,rms", [(4096, True), (2048, False), (5120, True), (8192, True), (3072, False),
                                   (6144, False)])
def test_wide_add_norm(C, rms, cuda):
    hip.require()
    torch.manual_seed(C)
    rows = 70
    x = torch.randn(rows, C, device=cuda).bfloat16()
    y = torch.randn(rows, C, device=cuda).bfloat16()
    g = (1 + 0.1 * torch.randn(C, device=cuda)).bfloat16()
    b = None if rms else (0.1 * torch.randn(C, device=cuda)).bfloat16()
    ys, xs, gs = (t.clone().requires_grad_() for t in (y, x, g))
    bs = None if b is None else b.clone().requires_grad_()
    xo, h = fused._AddNorm.apply(ys, xs, None, gs, bs, 1e-5, rms, 0.0, 1)
    yr, xr, gr = (t.float().requires_grad_() for t in (y, x, g))
    br = None if b is None else b.float().requires_grad_()
    xo_r = xr + yr
    if rms:
        h_r = xo_r * torch.rsqrt(xo_r.pow(2).mean(-1, keepdim=True) + 1e-5) * gr
    else:
        h_r = torch.nn.functional.layer_norm(xo_r, (C,), gr, br, 1e-5)
    assert _rel(xo, xo_r) < 1e-2 and _rel(h, h_r) < 2e-2
    dxo, dh = torch.randn_like(x), torch.randn_like(x)
    torch.autograd.backward([xo, h], [dxo, dh])
    torch.autograd.backward([xo_r, h_r], [dxo.float(), dh.float()])
    for a, r in ((ys.grad, yr.grad), (xs.grad, xr.grad), (gs.grad, gr.grad)):
        assert _rel(a, r) < 2e-2
    if b is not None:
        assert _rel(bs.grad, br.grad) < 2e-2


def test_wide_plain_rmsnorm_matches_module(cuda):
    hip.require()
    torch.manual_seed(3)
    x = torch.randn(2, 33, 4096, device=cuda).bfloat16().requires_grad_()
    g = (1 + 0.1 * torch.randn(4096, device=cuda)).bfloat16().requires_grad_()
    h = fused.norm(x, g, None, 1e-6, rms=True)
    xr, gr = x.detach().float().requires_grad_(), g.detach().float().requires_grad_()
    hr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6) * gr
    assert _rel(h, hr) < 2e-2
    dh = torch.randn_like(h)
    h.backward(dh)
    hr.backward(dh.float())
    assert _rel(x.grad, xr.grad) < 2e-2 and _rel(g.grad, gr.grad) < 2e-2


def test_swiglu(cuda):
    hip.require()
    torch.manual_seed(4)
    gt = (3 * torch.randn(257, 1376, device=cuda)).bfloat16().requires_grad_()
    up = torch.randn(257, 1376, device=cuda).bfloat16().requires_grad_()
    h = fused.swiglu(gt, up)
    gr, ur = gt.detach().float().requires_grad_(), up.detach().float().requires_grad_()
    hr = torch.nn.functional.silu(gr) * ur
    assert _rel(h, hr) < 1e-2
    dh = torch.randn_like(h)
    h.backward(dh)
    hr.backward(dh.float())
    assert _rel(gt.grad, gr.grad) < 2e-2 and _rel(up.grad, ur.grad) < 2e-2


@pytest.mark.parametrize("D", [64, 128])
def test_rope(D, cuda):
    hip.require()
    from distributed_lion_pytorch_amd.models.llama import Rotary

    torch.manual_seed(5)
    B, T, H = 2, 77, 5
    rot = Rotary(D, 10000.0)
    cos, sin = rot.tables(T + 3, torch.device(cuda), torch.bfloat16)  # tables longer than T are fine
    x = torch.randn(B, T, H, D, device=cuda).bfloat16().requires_grad_()
    y = fused.rope(x, cos, sin)
    xr = x.detach().float().requires_grad_()
    yr = fused.rope_reference(xr, cos.float(), sin.float())
    assert _rel(y, yr) < 1e-2
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy.float())
    assert _rel(x.grad, xr.grad) < 1e-2
