"""Weight-gradient GEMM (csrc/gemm_tn.hip): sum over its split slices of
P^T Q against a PyTorch fp32 reference, over several segments, strided
operands, edge tiles and split counts."""
import pytest
import torch

from distributed_lion_pytorch_amd.ops import hip

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,rows,nseg,splits,ldp_pad,ldq_pad", [
    (256, 256, 128, 1, 1, 0, 0),
    (768, 2304, 1024, 2, 3, 0, 0),
    (776, 264, 256, 3, 2, 8, 16),   # edge tiles in both dims, row strides > width
    (3072, 768, 512, 4, 7, 0, 0),   # uneven splits of 16 k-tile pairs
])
def test_gemm_tn_matches_fp32(cuda, M, N, rows, nseg, splits, ldp_pad, ldq_pad):
    hip.require()
    torch.manual_seed(0)
    P = [torch.randn(rows, M + ldp_pad, device=cuda, dtype=torch.bfloat16)[:, :M] for _ in range(nseg)]
    Q = [torch.randn(rows, N + ldq_pad, device=cuda, dtype=torch.bfloat16)[:, :N] for _ in range(nseg)]
    out = hip.ops().gemm_tn(P, Q, splits)
    assert out.shape == (splits, M, N) and out.dtype == torch.float32
    ref = torch.cat(P).float().t() @ torch.cat(Q).float()
    err = (out.sum(0) - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-3, err


def test_gemm_tn_split_slices_are_partial_sums(cuda):
    hip.require()
    torch.manual_seed(1)
    P = [torch.randn(512, 256, device=cuda, dtype=torch.bfloat16)]
    Q = [torch.randn(512, 512, device=cuda, dtype=torch.bfloat16)]
    out = hip.ops().gemm_tn(P, Q, 2)  # 2 pairs of 64-row k-tiles: rows 0..255 and 256..511
    for z, (a, b) in enumerate(((0, 256), (256, 512))):
        ref = P[0][a:b].float().t() @ Q[0][a:b].float()
        assert (out[z] - ref).abs().max().item() / ref.abs().max().item() < 1e-3


@pytest.mark.parametrize("defer", [True, False])
def test_window_wgrad_deferral(cuda, monkeypatch, defer):
    """Inside a multi-micro-batch fusion window the weight gradients are kept
    as operand segments and reduced by ONE TN GEMM at the window's exit
    (ops/linear._defer_wgrad); the result equals the per-micro-batch sum."""
    from distributed_lion_pytorch_amd.ops import linear as L

    hip.require()
    monkeypatch.setattr(L, "_WDEFER_ON", defer)
    torch.manual_seed(2)
    T, K, N, mbs = 512, 768, 2304, 3
    w = torch.nn.Parameter(torch.zeros(K, N, device=cuda, dtype=torch.bfloat16))
    xs = [torch.randn(T, K, device=cuda, dtype=torch.bfloat16) for _ in range(mbs)]
    gs = [torch.randn(T, N, device=cuda, dtype=torch.bfloat16) for _ in range(mbs)]
    L.release_split_k_accumulators()
    with L.grad_accumulation_fusion(True, micro_batches=mbs):
        for x, g in zip(xs, gs):
            L.wgrad_into(x, g, w)
        assert bool(L._WDEFER) == defer
        assert w.grad is None  # nothing reduced before the window closes
    assert not L._WDEFER
    ref = sum(x.float().t() @ g.float() for x, g in zip(xs, gs))
    err = (w.grad.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 8e-3, err


@pytest.mark.parametrize("case", ["varying_tokens", "tiny_budget", "many_segments", "shared_weight"])
def test_window_wgrad_deferral_edge_cases(cuda, monkeypatch, case):
    """Deferred weight gradients against the fp32 sum in the branches that
    reshape or bypass the kept segments: a token count change inside the
    window (segments flushed, accumulator re-split), a memory cap below one
    micro-batch (per-micro-batch accumulation), more micro-batches than the
    kernel's 16 segments, and one weight used twice per micro-batch (tied
    layers: both calls land in the same kept segments)."""
    from distributed_lion_pytorch_amd.ops import linear as L

    hip.require()
    torch.manual_seed(4)
    K, N = 256, 768
    Ms = {"varying_tokens": [1024, 1024, 512, 1024], "many_segments": [256] * 18}.get(case, [512, 512, 512])
    if case == "tiny_budget":
        monkeypatch.setattr(L, "_wdefer_budget", lambda: 1)
    w = torch.nn.Parameter(torch.zeros(K, N, device=cuda, dtype=torch.bfloat16))
    reps = 2 if case == "shared_weight" else 1
    xs = [torch.randn(m, K, device=cuda, dtype=torch.bfloat16) for m in Ms for _ in range(reps)]
    gs = [torch.randn(x.shape[0], N, device=cuda, dtype=torch.bfloat16) for x in xs]
    L.release_split_k_accumulators()
    with L.grad_accumulation_fusion(True, micro_batches=len(Ms)):
        for x, g in zip(xs, gs):
            L.wgrad_into(x, g, w)
    assert not L._WDEFER
    ref = sum(x.float().t() @ g.float() for x, g in zip(xs, gs))
    err = (w.grad.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 8e-3, err


def test_checkpointed_model_skips_wgrad_deferral(cuda, monkeypatch):
    """Activation checkpointing + a multi-micro-batch window: the layer inputs
    are not kept for a window-level GEMM (that would undo the checkpointing's
    memory saving); the gradients equal the non-checkpointed deferred run's."""
    from distributed_lion_pytorch_amd.models.gpt2 import GPT2LMHeadModel, gpt2_config
    from distributed_lion_pytorch_amd.ops import linear as L

    hip.require()
    torch.manual_seed(5)
    cfg = gpt2_config("gpt2-tiny")
    cfg.resid_pdrop = cfg.embd_pdrop = cfg.attn_pdrop = 0.0
    model = GPT2LMHeadModel(cfg).to(cuda, torch.bfloat16)
    batches = [torch.randint(0, cfg.vocab_size, (2, 128), device=cuda) for _ in range(3)]
    kept = []
    orig = L._defer_wgrad

    def spy(*args):
        r = orig(*args)
        kept.append(r)
        return r

    monkeypatch.setattr(L, "_defer_wgrad", spy)

    def run(ckpt):
        if ckpt:
            model.gradient_checkpointing_enable()
        else:
            model.gradient_checkpointing_disable()
        model.zero_grad(set_to_none=True)
        kept.clear()
        with L.grad_accumulation_fusion(True, micro_batches=len(batches)):
            for ids in batches:
                model(input_ids=ids, labels=ids).loss.backward()
        return any(kept), {n: p.grad.float().clone() for n, p in model.named_parameters() if p.grad is not None}

    kept_plain, g_plain = run(False)
    kept_ckpt, g_ckpt = run(True)
    assert kept_plain and not kept_ckpt
    assert set(g_plain) == set(g_ckpt)
    for n in g_plain:
        err = (g_ckpt[n] - g_plain[n]).abs().max().item() / max(g_plain[n].abs().max().item(), 1e-6)
        assert err < 3e-2, n
