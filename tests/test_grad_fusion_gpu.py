"""Gradient-accumulation fusion (weight grads deposited straight into
param.grad by the split-K reduction / beta=1 GEMM) vs autograd's own
accumulation over several micro-batches."""
import pytest
import torch

from distributed_lion_pytorch_amd.models.gpt2 import GPT2LMHeadModel, gpt2_config
from distributed_lion_pytorch_amd.models.llama import LlamaForCausalLM, llama_config
from distributed_lion_pytorch_amd.ops import hip
from distributed_lion_pytorch_amd.ops.linear import grad_accumulation_fusion

pytestmark = pytest.mark.gpu


def _grads(model, batches, fuse):
    model.zero_grad(set_to_none=True)
    with grad_accumulation_fusion(fuse):
        for ids in batches:
            model(input_ids=ids, labels=ids).loss.backward()
    return {n: p.grad.detach().float().clone() for n, p in model.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("family", ["gpt2", "llama"])
def test_fused_accumulation_matches_autograd(family, cuda):
    hip.require()
    torch.manual_seed(0)
    if family == "gpt2":
        cfg = gpt2_config("gpt2-tiny", n_embd=256, n_head=4, resid_pdrop=0.0, embd_pdrop=0.0, attn_pdrop=0.0)
        model = GPT2LMHeadModel(cfg)
    else:
        cfg = llama_config("llama-tiny")
        model = LlamaForCausalLM(cfg)
    model = model.to(device=cuda, dtype=torch.bfloat16).train()
    batches = [torch.randint(0, cfg.vocab_size, (2, 64), device=cuda) for _ in range(3)]
    ref = _grads(model, batches, False)
    fused = _grads(model, batches, True)
    assert ref.keys() == fused.keys()
    for n in ref:
        err = (ref[n] - fused[n]).abs().max().item() / (ref[n].abs().max().item() + 1e-8)
        assert err < 2e-2, (n, err)


def test_split_k_accumulator_window(cuda, monkeypatch):
    """Split-K weight gradients stay in fp32 [S, K, N] buffers across the
    micro-batches of one window (GEMM epilogue accumulation) and reach
    param.grad once, when the window closes; the sum is fp32-exact to bf16
    rounding of the final gradient.  (Deferral off: this is the per-micro-batch
    accumulator path; tests/test_gemm_tn_gpu.py covers the deferred one.)"""
    from distributed_lion_pytorch_amd.ops import linear as L

    hip.require()
    monkeypatch.setattr(L, "_WDEFER_ON", False)
    torch.manual_seed(3)
    K, N, M = 256, 768, 2048
    assert L.split_k_factor(M, K, N) > 1
    w = torch.nn.Parameter((torch.randn(N, K, device=cuda) * 0.05).to(torch.bfloat16))
    xs = [torch.randn(M, K, device=cuda, dtype=torch.bfloat16) for _ in range(4)]
    dys = [torch.randn(M, N, device=cuda, dtype=torch.bfloat16) for _ in range(4)]
    with L.grad_accumulation_fusion(True):
        for i, (x, dy) in enumerate(zip(xs, dys)):
            y = L.linear_nk(x, w)
            y.backward(dy)
            assert w.grad is None, "deposit must wait for the end of the window"
            assert len(L._ST.pending) == 1
    assert not L._ST.pending
    ref = sum(dy.float().t() @ x.float() for x, dy in zip(xs, dys))
    err = (w.grad.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 8e-3, err
    # a second window accumulates on top of the existing gradient
    with L.grad_accumulation_fusion(True):
        L.linear_nk(xs[0], w).backward(dys[0])
    ref2 = ref + dys[0].float().t() @ xs[0].float()
    err2 = (w.grad.float() - ref2).abs().max().item() / ref2.abs().max().item()
    assert err2 < 8e-3, err2


def _window_ref(steps):
    """fp32 autograd-free reference: sum of dy^T x over the window."""
    return sum(dy.float().t() @ x.float() for x, dy in steps)


@pytest.mark.parametrize("case", ["varying_m", "tiny_budget", "shared_weight", "single_micro_batch"])
def test_split_k_window_edge_cases(case, cuda, monkeypatch):
    """The branches where the accumulators could lose or corrupt partials:
    a split factor that changes inside a window (different token counts), an
    over-budget buffer, one weight used by two layers (two keys deposit into
    one .grad), and a window declared as one micro-batch (no buffers)."""
    from distributed_lion_pytorch_amd.ops import linear as L

    hip.require()
    torch.manual_seed(7)
    K, N = 256, 768
    if case == "tiny_budget":
        monkeypatch.setattr(L, "_ACC_BUDGET", 1 << 20)
    w = torch.nn.Parameter((torch.randn(N, K, device=cuda) * 0.05).to(torch.bfloat16))
    w2 = torch.nn.Parameter((torch.randn(N, K, device=cuda) * 0.05).to(torch.bfloat16))
    Ms = [2048, 1032, 2048, 1032] if case in ("varying_m", "tiny_budget") else [2048, 2048, 2048]
    if case == "single_micro_batch":
        Ms = [2048]
    if case == "varying_m":
        assert L.split_k_factor(2048, K, N) != L.split_k_factor(1032, K, N)
    steps = [(torch.randn(m, K, device=cuda, dtype=torch.bfloat16),
              torch.randn(m, N, device=cuda, dtype=torch.bfloat16)) for m in Ms]
    L.release_split_k_accumulators()
    with L.grad_accumulation_fusion(True, micro_batches=len(Ms)):
        for x, dy in steps:
            if case == "shared_weight":
                # w alone (single key) and w fused with w2 (multi key)
                L.linear_nk(x, w).backward(dy)
                ya, yb = L.linear_multi_nk(x, [w, w2])
                torch.autograd.backward([ya, yb], [dy, dy])
            else:
                L.linear_nk(x, w).backward(dy)
        if case == "single_micro_batch":
            assert not L._ST.pending and w.grad is not None
    assert not L._ST.pending
    ref = _window_ref(steps)
    if case == "shared_weight":
        ref2 = ref.clone()
        ref = 2 * ref
        err2 = (w2.grad.float() - ref2).abs().max().item() / ref2.abs().max().item()
        assert err2 < 8e-3, err2
    err = (w.grad.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 8e-3, (case, err)
    L.release_split_k_accumulators()
    assert not L._ST.acc


def test_lm_head_weight_gradient_joins_the_window(cuda, monkeypatch):
    """Inside a multi-micro-batch window the LM head's weight gradient is not
    computed per micro-batch: (softmax - onehot, s * h) go to the window's TN
    GEMM and reach w.grad when the window closes -- equal to the per-micro-batch
    path (different loss scales per micro-batch included)."""
    from distributed_lion_pytorch_amd.ops import fused
    from distributed_lion_pytorch_amd.ops import linear as L

    hip.require()
    torch.manual_seed(5)
    N, C, V = 256, 256, 1000
    hs = [torch.randn(N, C, device=cuda).to(torch.bfloat16).requires_grad_(True) for _ in range(3)]
    w = torch.nn.Parameter((torch.randn(V, C, device=cuda) * 0.05).to(torch.bfloat16))
    labels = [torch.randint(0, V, (N,), device=cuda) for _ in range(3)]
    labels[1][::3] = -100  # a different normalizer per micro-batch
    grads = {}
    for defer in (True, False):
        monkeypatch.setattr(fused, "_LM_DEFER", defer)
        w.grad = None
        with L.grad_accumulation_fusion(True, micro_batches=3):
            for i in range(3):
                (fused.lm_head_cross_entropy(hs[i], w, labels[i]) * (i + 1)).backward()
                if defer:
                    assert w.grad is None, "the deferred gradient must wait for the end of the window"
        grads[defer] = w.grad.float().clone()
    ref = grads[False]
    err = (grads[True] - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-2, err
