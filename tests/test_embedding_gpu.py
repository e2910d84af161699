"""Fused token + position embedding with dropout (csrc/embedding.hip) vs the
ATen chain, forward and backward (dense and in-place fused gradients), and the
LM head's device-scaled gradient deposit."""
import pytest
import torch
import torch.nn.functional as F

from distributed_lion_pytorch_amd.ops import fused, hip
from distributed_lion_pytorch_amd.ops.linear import grad_accumulation_fusion

pytestmark = pytest.mark.gpu


def _ref(ids, wte, wpe, p, seed):
    B, T = ids.shape
    C = wte.shape[1]
    x = (F.embedding(ids, wte.float()) + wpe.float()[:T][None]).bfloat16().float()
    if p > 0:
        keep = fused.norm_dropout_keep(B * T, C, p, seed, device=ids.device).view(B, T, C)
        th = min(65535, round(p * 65536))
        x = torch.where(keep, x * (65536.0 / (65536.0 - th)), torch.zeros_like(x))
    return x


@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("fuse", [False, True])
def test_embed_fwd_bwd(p, fuse, cuda):
    hip.require()
    torch.manual_seed(0)
    V, C, P, B, T = 1000, 128, 256, 4, 64
    ids = torch.randint(0, V, (B, T), device=cuda)
    ids[0, :8] = 7  # repeated tokens: one segment with several rows
    wte = torch.nn.Parameter((0.1 * torch.randn(V, C, device=cuda)).bfloat16())
    wpe = torch.nn.Parameter((0.1 * torch.randn(P, C, device=cuda)).bfloat16())
    seed = 1234
    out = fused._Embed.apply(ids, wte, wpe, p, seed) if not fuse else None
    if fuse:
        with grad_accumulation_fusion(True):
            wte.grad = torch.ones_like(wte) * 0.5  # an LM-head gradient already deposited (tied weights)
            out = fused._Embed.apply(ids, wte, wpe, p, seed)
            dy = torch.randn_like(out)
            out.backward(dy)
    else:
        dy = torch.randn_like(out)
        out.backward(dy)
    ref = _ref(ids, wte.detach(), wpe.detach(), p, seed)
    assert (out.float() - ref).abs().max().item() < 2e-2
    wr = wte.detach().float().requires_grad_(True)
    pr = wpe.detach().float().requires_grad_(True)
    x = F.embedding(ids, wr) + pr[:T][None]
    if p > 0:
        keep = fused.norm_dropout_keep(B * T, C, p, seed, device=cuda).view(B, T, C)
        th = min(65535, round(p * 65536))
        x = torch.where(keep, x * (65536.0 / (65536.0 - th)), torch.zeros_like(x))
    x.backward(dy.float())
    g_wte = wr.grad + (0.5 if fuse else 0.0)
    assert (wte.grad.float() - g_wte).abs().max().item() < 3e-2 * g_wte.abs().max().item()
    assert (wpe.grad.float() - pr.grad).abs().max().item() < 3e-2 * pr.grad.abs().max().item()
    assert torch.all(wpe.grad[T:] == 0)


def test_gpt2_fused_embedding_and_lm_head_grads_match_autograd(cuda):
    """Tiny GPT-2 (dropout off): every gradient inside a fusion window (LM-head
    scale deposit + in-place embedding rows into the tied wte) equals the plain
    autograd accumulation to bf16 rounding."""
    from distributed_lion_pytorch_amd.models.gpt2 import GPT2LMHeadModel, gpt2_config

    hip.require()
    torch.manual_seed(0)
    cfg = gpt2_config("gpt2-tiny", n_embd=128, n_head=2, resid_pdrop=0.0, embd_pdrop=0.0, attn_pdrop=0.0)
    model = GPT2LMHeadModel(cfg).to(device=cuda, dtype=torch.bfloat16).train()
    batches = [torch.randint(0, cfg.vocab_size, (2, 64), device=cuda) for _ in range(2)]
    grads = {}
    for f in (False, True):
        model.zero_grad(set_to_none=True)
        with grad_accumulation_fusion(f):
            for ids in batches:
                (model(ids, labels=ids)["loss"] / 2).backward()
        grads[f] = {n: p.grad.float().clone() for n, p in model.named_parameters()}
    for n in grads[False]:
        a, b = grads[True][n], grads[False][n]
        assert (a - b).abs().max().item() < 2e-2 * b.abs().max().item() + 1e-6, n


def test_out_of_range_ids_and_labels_are_errors(cuda):
    """ATen's embedding / cross-entropy raise on an id >= V; the fused kernels
    flag it on the device (no clamp-and-continue) and check_index_errors()
    raises -- a step late in the non-blocking per-step form, at once blocking."""
    hip.require()
    V, C, P = 1000, 128, 256
    wte = torch.randn(V, C, device=cuda, dtype=torch.bfloat16)
    wpe = torch.randn(P, C, device=cuda, dtype=torch.bfloat16)
    ok = torch.randint(0, V, (2, 64), device=cuda)
    fused.embed(ok, wte, wpe, 0.0)
    fused.check_index_errors(blocking=True)  # clean
    bad = ok.clone()
    bad[1, 7] = V  # one id past the table
    fused.embed(bad, wte, wpe, 0.0)
    fused.check_index_errors()  # starts the async copy of the flag
    torch.cuda.synchronize()
    with pytest.raises(ValueError, match="embedding table"):
        fused.check_index_errors()  # the landed copy shows the error
    fused.check_index_errors(blocking=True)  # the flag was reset
    labels = torch.randint(0, V, (128,), device=cuda)
    labels[3] = -100  # the ignore index is fine
    fused.check_labels(labels, V)
    fused.check_index_errors(blocking=True)
    labels[5] = V + 3
    fused.check_labels(labels, V)
    with pytest.raises(ValueError, match="label"):
        fused.check_index_errors(blocking=True)
