"""Fused softmax cross-entropy kernel (fp32-row, streaming and packed 16-bit
row variants) vs an fp32 PyTorch reference: per-row loss and the in-place
softmax - onehot."""
import pytest
import torch

from distributed_lion_pytorch_amd.ops import fused, hip

pytestmark = pytest.mark.gpu


# variant: 0 auto, 1 fp32 row in registers, 2 streaming, 4 / 5 packed row (512 / 1024 threads)
CASES = [(V, var) for V in (512, 32000, 50257) for var in (0, 1, 2, 4, 5)] + [(128256, 0), (128256, 2)]


@pytest.mark.parametrize("V,variant", CASES)
def test_softmax_xent_kernel(V, variant, cuda):
    hip.require()
    torch.manual_seed(V)
    N = 67
    Vp = (V + 63) // 64 * 64
    x = (2 * torch.randn(N, Vp, device=cuda)).bfloat16()
    labels = torch.randint(0, V, (N,), device=cuda)
    labels[::7] = -100
    ref_in = x[:, :V].float()
    y = x.clone()
    loss = hip.ops().softmax_xent_(y, labels, V, variant)
    valid = labels != -100
    ref_loss = torch.nn.functional.cross_entropy(ref_in, labels.clamp_min(0), reduction="none") * valid
    assert (loss - ref_loss).abs().max().item() < 1e-3
    prob = torch.softmax(ref_in, -1)
    prob[torch.arange(N, device=cuda), labels.clamp_min(0)] -= 1
    prob[~valid] = 0
    assert (y[:, :V].float() - prob).abs().max().item() < 1e-2
    if Vp > V:
        assert y[:, V:].abs().max().item() == 0.0


def test_lm_head_ce_wide_vocab_matches_reference(cuda):
    hip.require()
    torch.manual_seed(0)
    h = torch.randn(2, 33, 64, device=cuda).bfloat16().requires_grad_()
    w = (0.05 * torch.randn(128256, 64, device=cuda)).bfloat16().requires_grad_()
    labels = torch.randint(0, 128256, (2, 33), device=cuda)
    loss = fused.lm_head_cross_entropy(h, w, labels)
    hr, wr = h.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    ref = torch.nn.functional.cross_entropy((hr @ wr.t()).view(-1, 128256), labels.view(-1))
    assert abs(loss.item() - ref.item()) < 1e-2
    loss.backward()
    ref.backward()
    assert (h.grad.float() - hr.grad).abs().max().item() < 2e-2 * hr.grad.abs().max().item() + 1e-4


def test_lm_head_ce_parameter_uses_own_dgrad_gemm(cuda):
    """Parameter weight, GPT-2 vocab (padded 50304 = 393 x 128): the input
    gradient runs on the own NT GEMM against the cached padded W^T."""
    hip.require()
    torch.manual_seed(1)
    V, C = 50257, 128
    h = torch.randn(3, 40, C, device=cuda).bfloat16().requires_grad_()
    w = torch.nn.Parameter((0.05 * torch.randn(V, C, device=cuda)).bfloat16())
    labels = torch.randint(0, V, (3, 40), device=cuda)
    loss = fused.lm_head_cross_entropy(h, w, labels)
    loss.backward()
    hr, wr = h.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    ref = torch.nn.functional.cross_entropy((hr @ wr.t()).view(-1, V), labels.view(-1))
    ref.backward()
    assert abs(loss.item() - ref.item()) < 1e-2
    assert (h.grad.float() - hr.grad).abs().max().item() < 2e-2 * hr.grad.abs().max().item() + 1e-4
    assert (w.grad.float() - wr.grad).abs().max().item() < 2e-2 * wr.grad.abs().max().item() + 1e-4
    from distributed_lion_pytorch_amd.ops.linear import _WT_CACHE

    assert (id(w), "pad_t") in _WT_CACHE


@pytest.mark.parametrize("preexisting_grad", [False, True])
def test_lm_head_ce_weight_grad_on_tn_kernel(cuda, preexisting_grad):
    """Token count % 128 == 0: the LM head's weight gradient comes from the own
    TN kernel as fp32 split partials, reduced + scaled (+ accumulated) in one
    pass (ops/fused._lm_wgrad_partials, sum_partials_scaled_)."""
    hip.require()
    torch.manual_seed(3)
    V, C = 50257, 256
    h = torch.randn(2, 128, C, device=cuda).bfloat16().requires_grad_()
    w = torch.nn.Parameter((0.05 * torch.randn(V, C, device=cuda)).bfloat16())
    g0 = (0.01 * torch.randn(V, C, device=cuda)).bfloat16() if preexisting_grad else None
    if g0 is not None:
        w.grad = g0.clone()
    labels = torch.randint(0, V, (2, 128), device=cuda)
    loss = 3.0 * fused.lm_head_cross_entropy(h, w, labels)  # a non-unit loss gradient
    loss.backward()
    hr, wr = h.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    ref = 3.0 * torch.nn.functional.cross_entropy((hr @ wr.t()).view(-1, V), labels.view(-1))
    ref.backward()
    want = wr.grad + (g0.float() if g0 is not None else 0.0)
    assert (w.grad.float() - want).abs().max().item() < 2e-2 * want.abs().max().item() + 1e-4
    assert (h.grad.float() - hr.grad).abs().max().item() < 2e-2 * hr.grad.abs().max().item() + 1e-4


@pytest.mark.parametrize("preexisting_grad", [False, True])
def test_lm_head_ce_late_unsplit_weight_grad(cuda, preexisting_grad, monkeypatch):
    """Llama-3 vocabulary (128256, % 8 == 0) and a head the split model runs
    unsplit: the weight gradient is computed in the backward by one TN GEMM of
    the padded logits' first v columns against s * h, bf16 straight into (or
    onto) .grad (ops/fused._LMHeadCE._backward_late)."""
    from distributed_lion_pytorch_amd.ops import linear

    hip.require()
    torch.manual_seed(5)
    V, C = 128256, 256
    assert linear.tn_split_factor(256, V, C, direct=True) == 1
    h = torch.randn(2, 128, C, device=cuda).bfloat16().requires_grad_()
    w = torch.nn.Parameter((0.05 * torch.randn(V, C, device=cuda)).bfloat16())
    g0 = (0.01 * torch.randn(V, C, device=cuda)).bfloat16() if preexisting_grad else None
    if g0 is not None:
        w.grad = g0.clone()
    labels = torch.randint(0, V, (2, 128), device=cuda)
    labels[0, :5] = -100
    calls = []
    late = fused._LMHeadCE._backward_late
    monkeypatch.setattr(fused._LMHeadCE, "_backward_late", staticmethod(lambda ctx, g: calls.append(1) or late(ctx, g)))
    loss = 2.5 * fused.lm_head_cross_entropy(h, w, labels)
    loss.backward()
    assert calls == [1]
    hr, wr = h.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    ref = 2.5 * torch.nn.functional.cross_entropy((hr @ wr.t()).view(-1, V), labels.view(-1))
    ref.backward()
    want = wr.grad + (g0.float() if g0 is not None else 0.0)
    assert (w.grad.float() - want).abs().max().item() < 2e-2 * want.abs().max().item() + 1e-4
    assert (h.grad.float() - hr.grad).abs().max().item() < 2e-2 * hr.grad.abs().max().item() + 1e-4
