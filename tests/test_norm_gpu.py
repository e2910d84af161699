"""Fused residual + dropout + LayerNorm/RMSNorm kernels vs an fp32 PyTorch
reference using the identical stateless dropout mask."""
import pytest
import torch

from distributed_lion_pytorch_amd.ops import fused, hip

pytestmark = pytest.mark.gpu


def _ref(y, x, g, b, eps, p, seed, rms, bias=None):
    rows, C = x.shape
    if bias is not None:
        y = y + bias
    if p > 0:
        th = min(65535, int(round(p * 65536)))
        keep = fused.norm_dropout_keep(rows, C, p, seed, x.device)
        y = y * keep * (65536.0 / (65536.0 - th))
    xo = x + y
    if rms:
        h = xo * torch.rsqrt(xo.pow(2).mean(-1, keepdim=True) + eps) * g
    else:
        h = torch.nn.functional.layer_norm(xo, (C,), g, b, eps)
    return xo, h


def _rel(a, b):
    return (a.float() - b.float()).abs().max().item() / (b.float().abs().max().item() + 1e-6)


def _close(a, b, tol):
    """Next to the max-normalised _rel: a bound that a wrong value on a
    small-magnitude row (2-D: per-row max error / per-row max) or element
    (1-D: elementwise, atol = tolerance x the MEAN magnitude -- a column sum
    that cancels to near zero keeps the absolute rounding error of its
    summands) cannot hide under the tensor-wide maximum."""
    a, b = a.float(), b.float()
    if b.dim() >= 2:
        err = (a - b).abs().amax(-1)
        scale = b.abs().amax(-1)
        return bool((err <= tol * scale + 1e-6).all())
    return bool(((a - b).abs() <= tol * b.abs() + tol * b.abs().mean() + 1e-6).all())


@pytest.mark.parametrize("C,rms", [(768, False), (1024, True), (512, True), (256, False)])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_add_norm_fwd_bwd(C, rms, p, cuda):
    hip.require()
    torch.manual_seed(0)
    rows = 333
    x = torch.randn(rows, C, device=cuda).bfloat16()
    y = torch.randn(rows, C, device=cuda).bfloat16()
    g = (1 + 0.1 * torch.randn(C, device=cuda)).bfloat16()
    b = None if rms else (0.1 * torch.randn(C, device=cuda)).bfloat16()
    seed = 4242
    bias = (0.1 * torch.randn(C, device=cuda)).bfloat16()
    ys, xs, gs = y.clone().requires_grad_(), x.clone().requires_grad_(), g.clone().requires_grad_()
    bs = None if b is None else b.clone().requires_grad_()
    bias_s = bias.clone().requires_grad_()
    xo, h = fused._AddNorm.apply(ys, xs, bias_s, gs, bs, 1e-5, rms, p, seed)
    yr, xr, gr, bias_r = (t.float().requires_grad_() for t in (y, x, g, bias))
    br = None if b is None else b.float().requires_grad_()
    xo_r, h_r = _ref(yr, xr, gr, br, 1e-5, p, seed, rms, bias_r)
    assert _rel(xo, xo_r) < 1e-2 and _rel(h, h_r) < 2e-2
    assert _close(xo, xo_r, 1e-2) and _close(h, h_r, 2e-2)
    dxo = torch.randn_like(x)
    dh = torch.randn_like(x)
    torch.autograd.backward([xo, h], [dxo, dh])
    torch.autograd.backward([xo_r, h_r], [dxo.float(), dh.float()])
    assert _rel(ys.grad, yr.grad) < 2e-2
    assert _rel(xs.grad, xr.grad) < 2e-2
    assert _rel(gs.grad, gr.grad) < 2e-2
    assert _rel(bias_s.grad, bias_r.grad) < 2e-2
    assert _close(ys.grad, yr.grad, 2e-2) and _close(xs.grad, xr.grad, 2e-2)
    assert _close(gs.grad, gr.grad, 5e-2) and _close(bias_s.grad, bias_r.grad, 5e-2)
    if b is not None:
        assert _rel(bs.grad, br.grad) < 2e-2
        assert _close(bs.grad, br.grad, 5e-2)


def test_plain_norm(cuda):
    hip.require()
    torch.manual_seed(1)
    x = torch.randn(100, 768, device=cuda).bfloat16().requires_grad_()
    g = torch.ones(768, device=cuda).bfloat16().requires_grad_()
    b = torch.zeros(768, device=cuda).bfloat16().requires_grad_()
    h = fused._Norm.apply(x, g, b, 1e-5, False)
    xr = x.detach().float().requires_grad_()
    hr = torch.nn.functional.layer_norm(xr, (768,), None, None, 1e-5)
    assert _rel(h, hr) < 2e-2 and _close(h, hr, 2e-2)
    dh = torch.randn_like(h)
    h.backward(dh)
    hr.backward(dh.float())
    assert _rel(x.grad, xr.grad) < 2e-2 and _close(x.grad, xr.grad, 2e-2)


@pytest.mark.parametrize("exact", [False, True])
def test_bias_gelu(exact, cuda):
    hip.require()
    torch.manual_seed(2)
    z = torch.randn(300, 3072, device=cuda).bfloat16().requires_grad_()
    b = (0.1 * torch.randn(3072, device=cuda)).bfloat16().requires_grad_()
    h = fused._BiasGelu.apply(z, b, exact)
    zr, br = z.detach().float().requires_grad_(), b.detach().float().requires_grad_()
    hr = torch.nn.functional.gelu(zr + br, approximate="none" if exact else "tanh")
    assert _rel(h, hr) < 1e-2
    dh = torch.randn_like(h)
    h.backward(dh)
    hr.backward(dh.float())
    assert _rel(z.grad, zr.grad) < 2e-2 and _rel(b.grad, br.grad) < 2e-2
    assert _close(h, hr, 1e-2) and _close(z.grad, zr.grad, 2e-2) and _close(b.grad, br.grad, 5e-2)


@pytest.mark.parametrize("S,shape", [(7, (3, 256)), (2048, (3, 768)), (1000, (3076,)), (16, (768, 3072))])
def test_sum_partials(S, shape, cuda):
    hip.require()
    part = torch.randn(S, *shape, device=cuda)
    out = hip.ops().sum_partials(part)
    assert out.dtype == torch.bfloat16 and out.shape == shape
    ref = part.double().sum(0)
    assert ((out.double() - ref).abs() <= ref.abs() * 2 ** -7 + 1e-3 * S ** 0.5).all()


def test_colsum_and_strided_partials(cuda):
    hip.require()
    torch.manual_seed(3)
    x = torch.randn(2000, 2304, device=cuda).bfloat16()
    part = hip.ops().colsum_partials(x, 125)
    assert part.shape == (125, 2304)
    assert _rel(hip.ops().sum_partials(part), x.float().sum(0)) < 1e-2
    # row-strided slice of a [S, 3, C] norm partial stack, with in-place accumulation
    stack = torch.randn(64, 3, 768, device=cuda)
    sl = stack.view(64, 3 * 768)[:, 768:1536]
    assert _rel(hip.ops().sum_partials(sl), stack[:, 1].sum(0)) < 1e-2
    acc = torch.randn(768, device=cuda).bfloat16()
    ref = acc.float() + stack[:, 2].sum(0)
    hip.ops().sum_partials_acc_(stack.view(64, 3 * 768)[:, 1536:], acc)
    assert _rel(acc, ref) < 1e-2
