"""Fused GPT-2 MLP: the own NT GEMM with the DGELU epilogue (dz = (dy . W^T) *
gelu'(z + b) plus bias-gradient partials) vs fp32 PyTorch, and the mlp_gelu
autograd op (fused / unfused forward and backward) vs fp32 autograd of
gelu(x @ Wfc + b) @ Wproj."""
import pytest
import torch
import torch.nn.functional as F

from distributed_lion_pytorch_amd.ops import fused, hip

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-6)).item()


def _gelu_grad(u, exact):
    u = u.detach().clone().requires_grad_(True)
    F.gelu(u, approximate="none" if exact else "tanh").backward(torch.ones_like(u))
    return u.grad


@pytest.mark.parametrize("M,N,K", [(512, 1024, 256), (300, 520, 128), (2048, 3072, 768)])
@pytest.mark.parametrize("exact", [False, True])
def test_gemm_nt_dgelu(M, N, K, exact, cuda):
    hip.require()
    torch.manual_seed(M + N)
    dy = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=cuda).to(torch.bfloat16)
    z = torch.randn(M, N, device=cuda).to(torch.bfloat16)
    dz, part = hip.ops().gemm_nt_dgelu(dy, w, b, z, exact)
    g = (dy.float() @ w.float().t()).bfloat16().float()  # the unfused GEMM's bf16 output
    ref = g * _gelu_grad(z.float() + b.float(), exact)
    assert _rel(dz, ref) < 1e-2, _rel(dz, ref)
    assert part.shape == (2 * ((M + 255) // 256), N)
    assert _rel(part.sum(0), ref.sum(0)) < 1e-2


@pytest.mark.parametrize("M,N,K", [(512, 1024, 256), (300, 520, 128)])
@pytest.mark.parametrize("exact", [False, True])
def test_gemm_nt_gelu_derivative_store_and_multiply(M, N, K, exact, cuda):
    """EPI 6/7 (h = gelu(z + b), d = gelu'(z + b) from one tanh/erf) and EPI 8
    (dz = bf16(dy . w^T) * d with bias-gradient partials) against fp32."""
    hip.require()
    torch.manual_seed(M + K)
    x = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=cuda).to(torch.bfloat16)
    h, d = hip.ops().gemm_nt_gelu_d(x, w, b, exact)
    z = (x.float() @ w.float().t()).bfloat16().float() + b.float()  # the GEMM output is rounded to bf16 first
    assert _rel(h, F.gelu(z, approximate="none" if exact else "tanh")) < 1e-2
    assert _rel(d, _gelu_grad(z, exact)) < 1e-2
    dy = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w2 = (torch.randn(N, K, device=cuda) / K ** 0.5).to(torch.bfloat16)
    dz, part = hip.ops().gemm_nt_dmul(dy, w2, d)
    ref = (dy.float() @ w2.float().t()).bfloat16().float() * d.float()
    assert _rel(dz, ref) < 1e-2
    assert _rel(part.sum(0), ref.sum(0)) < 1e-2


@pytest.mark.parametrize("fused_fwd,fused_bwd,dstore", [(True, True, True), (True, True, False), (False, False, True),
                                                         (True, False, True), (False, True, True)])
def test_mlp_gelu_grads(fused_fwd, fused_bwd, dstore, cuda, monkeypatch):
    hip.require()
    monkeypatch.setattr(fused, "_GELU_FUSED", fused_fwd)
    monkeypatch.setattr(fused, "_DGELU_FUSED", fused_bwd)
    monkeypatch.setattr(fused, "_GELU_DSTORE", dstore)
    torch.manual_seed(3)
    M, C, F4 = 512, 256, 1024
    x = torch.randn(M, C, device=cuda).to(torch.bfloat16).requires_grad_(True)
    wf = (torch.randn(C, F4, device=cuda) / C ** 0.5).to(torch.bfloat16).requires_grad_(True)
    b = (0.1 * torch.randn(F4, device=cuda)).to(torch.bfloat16).requires_grad_(True)
    wp = (torch.randn(F4, C, device=cuda) / F4 ** 0.5).to(torch.bfloat16).requires_grad_(True)
    dy = torch.randn(M, C, device=cuda).to(torch.bfloat16)
    y = fused.mlp_gelu(x, wf, b, wp)
    y.backward(dy)
    xr, wfr, br, wpr = (t.detach().float().requires_grad_(True) for t in (x, wf, b, wp))
    yr = F.gelu(xr @ wfr + br, approximate="tanh") @ wpr
    yr.backward(dy.float())
    assert _rel(y, yr) < 1e-2
    for got, ref in ((x.grad, xr.grad), (wf.grad, wfr.grad), (b.grad, br.grad), (wp.grad, wpr.grad)):
        assert _rel(got, ref) < 2e-2, _rel(got, ref)


def test_gpt2_mlp_fused_matches_unfused(cuda, monkeypatch):
    """Whole tiny GPT-2 (dropout off): gradients with the fused DGELU backward
    equal the unfused path's to bf16 rounding."""
    from distributed_lion_pytorch_amd.models.gpt2 import GPT2LMHeadModel, gpt2_config

    hip.require()
    torch.manual_seed(0)
    cfg = gpt2_config("gpt2-tiny", n_embd=256, n_head=4, resid_pdrop=0.0, embd_pdrop=0.0, attn_pdrop=0.0)
    model = GPT2LMHeadModel(cfg).to(device=cuda, dtype=torch.bfloat16).train()
    ids = torch.randint(0, cfg.vocab_size, (2, 128), device=cuda)
    grads = {}
    for flag in (True, False):
        monkeypatch.setattr(fused, "_DGELU_FUSED", flag)
        monkeypatch.setattr(fused, "_GELU_FUSED", flag)
        model.zero_grad(set_to_none=True)
        model(ids, labels=ids)["loss"].backward()
        grads[flag] = {n: p.grad.float().clone() for n, p in model.named_parameters() if p.grad is not None}
    for n in grads[True]:
        assert _rel(grads[True][n], grads[False][n]) < 3e-2, n
