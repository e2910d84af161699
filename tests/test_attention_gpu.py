"""gfx950 flash attention (fwd + bwd, dropout, GQA) vs an fp32 PyTorch reference
that uses the identical stateless dropout mask."""
import pytest
import torch

from distributed_lion_pytorch_amd.ops import fused, hip


def test_dropout_mask_statistics_cpu():
    keep = fused.attention_dropout_keep(2, 3, 128, 0.1, seed=7)
    frac = keep.float().mean().item()
    assert abs(frac - 0.9) < 0.01
    keep2 = fused.attention_dropout_keep(2, 3, 128, 0.1, seed=8)
    assert (keep != keep2).float().mean().item() > 0.1
    # no structure between neighbours: adjacent keys (same hash word), adjacent
    # queries and adjacent heads drop independently (P(both dropped) ~ p^2)
    d = (~fused.attention_dropout_keep(1, 4, 512, 0.1, seed=3)).float()
    for a, b in ((d[..., 0::2], d[..., 1::2]), (d[:, :, :-1], d[:, :, 1:]), (d[:, :-1], d[:, 1:])):
        both = (a * b).mean().item()
        assert abs(both - 0.01) < 0.003, both


def test_dropout_masks_of_different_rows_are_not_shifted_copies_cpu():
    """with v2's tile-linear pair hash, every row's mask was a
    window of one fixed 2^24-periodic sequence, so ~15 other rows per row held
    shifted copies of it.  No 256-key window (at any even offset) may repeat
    across the rows of a GPT-2-sized head set (random masks: P ~ 1e-22)."""
    import torch

    B, H, T = 1, 12, 1024
    keep = fused.attention_dropout_keep(B, H, T, 0.1, seed=11).view(B * H * T, T).double()
    g = torch.Generator().manual_seed(0)
    v = torch.randn(1, 1, 256, generator=g, dtype=torch.float64)
    # signature of every 256-key window at an even offset: a random projection
    sig = torch.nn.functional.conv1d(keep.unsqueeze(1), v, stride=2).reshape(-1)
    rows = torch.arange(B * H * T).repeat_interleave((T - 256) // 2 + 1)
    _, inv, counts = torch.unique(sig, return_inverse=True, return_counts=True)
    dup = counts[inv] > 1
    # the only repeats allowed are rows too short to be random (none here)
    assert int(dup.sum()) == 0, f"{int(dup.sum())} repeated windows, e.g. rows {rows[dup][:6].tolist()}"


def _close(a, b, tol, floor=0.0):
    err = (a.float() - b.float()).abs().max().item()
    scale = max(b.float().abs().max().item(), floor) + 1e-6
    assert err <= tol * scale, f"max err {err} vs scale {scale}"


@pytest.mark.gpu
@pytest.mark.parametrize("B,T,H,Hkv,D", [(2, 128, 4, 4, 64), (1, 256, 8, 2, 128), (3, 64, 2, 1, 64)])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_flash_attention_fwd_bwd(B, T, H, Hkv, D, p, cuda):
    hip.require()
    torch.manual_seed(0)
    q = torch.randn(B, T, H, D, device=cuda, dtype=torch.bfloat16)
    k = torch.randn(B, T, Hkv, D, device=cuda, dtype=torch.bfloat16)
    v = torch.randn(B, T, Hkv, D, device=cuda, dtype=torch.bfloat16)
    dout = torch.randn(B, T, H * D, device=cuda, dtype=torch.bfloat16)
    seed = 1234
    qs, ks, vs = (t.clone().requires_grad_() for t in (q, k, v))
    out = fused._FlashAttn.apply(qs, ks, vs, p, seed).view(B, T, H * D)
    out.backward(dout)
    qr, kr, vr = (t.float().requires_grad_() for t in (q, k, v))
    ref = fused.reference_attention(qr, kr, vr, p, seed)
    ref.backward(dout.float())
    _close(out, ref, 2e-2)
    _close(qs.grad, qr.grad, 3e-2)
    _close(ks.grad, kr.grad, 3e-2)
    _close(vs.grad, vr.grad, 3e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_packed_qkv_attention_matches_reference(p, cuda):
    hip.require()
    torch.manual_seed(1)
    B, T, H, D = 2, 192, 3, 64
    qkv = torch.randn(B, T, 3, H, D, device=cuda, dtype=torch.bfloat16)
    dout = torch.randn(B, T, H * D, device=cuda, dtype=torch.bfloat16)
    a = qkv.clone().requires_grad_()
    out = fused._FlashAttnPacked.apply(a, p, 99).view(B, T, H * D)
    out.backward(dout)
    r = qkv.float().requires_grad_()
    ref = fused.reference_attention(r[:, :, 0], r[:, :, 1], r[:, :, 2], p, 99)
    ref.backward(dout.float())
    _close(out, ref, 2e-2)
    _close(a.grad, r.grad, 3e-2)


@pytest.mark.parametrize("fuse", [False, True])
def test_qkv_attention_bias_grad_from_kernels(fuse, cuda):
    """GPT-2 c_attn projection + attention as one op: the c_attn bias gradient
    comes from the dQ/dKV kernels' column partials; all gradients vs fp32."""
    from distributed_lion_pytorch_amd.ops import fused
    from distributed_lion_pytorch_amd.ops.linear import grad_accumulation_fusion

    hip.require()
    torch.manual_seed(5)
    B, T, H, D = 2, 128, 4, 64
    C = H * D
    x = torch.randn(B, T, C, device=cuda).bfloat16().requires_grad_(True)
    w = torch.nn.Parameter((torch.randn(C, 3 * C, device=cuda) / C ** 0.5).bfloat16())
    b = torch.nn.Parameter((0.1 * torch.randn(3 * C, device=cuda)).bfloat16())
    dy = torch.randn(B, T, C, device=cuda).bfloat16()
    with grad_accumulation_fusion(fuse):
        y = fused.qkv_attention(x, w, b, H, 0.0)
        y.backward(dy)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    qkv = (xr @ wr + br).view(B, T, 3, H, D).permute(2, 0, 3, 1, 4)
    yr = torch.nn.functional.scaled_dot_product_attention(qkv[0], qkv[1], qkv[2], is_causal=True)
    yr = yr.transpose(1, 2).reshape(B, T, C)
    yr.backward(dy.float())
    rel = lambda a, r: ((a.float() - r).abs().max() / (r.abs().max() + 1e-6)).item()  # noqa: E731
    assert rel(y, yr) < 2e-2
    for got, ref in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        assert rel(got, ref) < 3e-2, rel(got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("T", [1, 33, 100, 1000, 1023])
@pytest.mark.parametrize("B,H,Hkv,D,p", [(2, 4, 4, 64, 0.1), (1, 4, 2, 128, 0.0)])
def test_flash_attention_tail_tiles(T, B, H, Hkv, D, p, cuda):
    """Any sequence length: the last 32-row tile is partial and masked in-kernel
    (no padding copy, no SDPA fallback); fwd + bwd vs fp32 with the same mask."""
    hip.require()
    torch.manual_seed(T)
    q = torch.randn(B, T, H, D, device=cuda, dtype=torch.bfloat16)
    k = torch.randn(B, T, Hkv, D, device=cuda, dtype=torch.bfloat16)
    v = torch.randn(B, T, Hkv, D, device=cuda, dtype=torch.bfloat16)
    dout = torch.randn(B, T, H * D, device=cuda, dtype=torch.bfloat16)
    assert fused._attn_ok(q, T, D)
    qs, ks, vs = (t.clone().requires_grad_() for t in (q, k, v))
    out = fused._FlashAttn.apply(qs, ks, vs, p, 4321).view(B, T, H * D)
    out.backward(dout)
    qr, kr, vr = (t.float().requires_grad_() for t in (q, k, v))
    ref = fused.reference_attention(qr, kr, vr, p, 4321)
    ref.backward(dout.float())
    _close(out, ref, 2e-2)
    # T = 1: dq and dk are exactly 0 in fp32 (one key, softmax = 1) and bf16
    # rounding noise in the kernels -- judge them on the scale of dv
    floor = vr.grad.abs().max().item() if T == 1 else 0.0
    _close(qs.grad, qr.grad, 3e-2, floor)
    _close(ks.grad, kr.grad, 3e-2, floor)
    _close(vs.grad, vr.grad, 3e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("T,window", [(100, 1), (100, 31), (100, 32), (100, 33), (300, 64), (1000, 200),
                                      (1000, 999), (257, 100)])
@pytest.mark.parametrize("B,H,Hkv,p", [(1, 4, 2, 0.0), (2, 2, 1, 0.1), (1, 2, 2, 0.0)])
def test_flash_attention_sliding_window(T, window, B, H, Hkv, p, cuda):
    """Mistral-style sliding window at head_dim 128 (key k visible to query q iff
    q - window < k <= q): skipped and boundary-masked tiles, tail tiles, GQA and
    dropout, fwd + bwd vs the fp32 reference with the same masks.  H == Hkv
    without dropout runs the K-in-registers dK/dV kernel (its window bounds,
    ADVICE r5), the other cases the LDS one."""
    hip.require()
    D = 128
    torch.manual_seed(T + window)
    q = torch.randn(B, T, H, D, device=cuda, dtype=torch.bfloat16)
    k = torch.randn(B, T, Hkv, D, device=cuda, dtype=torch.bfloat16)
    v = torch.randn(B, T, Hkv, D, device=cuda, dtype=torch.bfloat16)
    dout = torch.randn(B, T, H * D, device=cuda, dtype=torch.bfloat16)
    assert fused._attn_ok(q, T, D, window)
    qs, ks, vs = (t.clone().requires_grad_() for t in (q, k, v))
    out = fused._FlashAttn.apply(qs, ks, vs, p, 77, window).view(B, T, H * D)
    out.backward(dout)
    qr, kr, vr = (t.float().requires_grad_() for t in (q, k, v))
    ref = fused.reference_attention(qr, kr, vr, p, 77, window)
    ref.backward(dout.float())
    # window 1: each query sees only itself -- dq, dk are exactly 0 in fp32
    floor = vr.grad.abs().max().item() if window == 1 else 0.0
    _close(out, ref, 2e-2)
    _close(qs.grad, qr.grad, 3e-2, floor)
    _close(ks.grad, kr.grad, 3e-2, floor)
    _close(vs.grad, vr.grad, 3e-2)


@pytest.mark.gpu
def test_sliding_window_rope_attention_and_mistral_model(cuda):
    """The Llama-path op with a window (RoPE fused into the backward stores) and
    a small Mistral (head_dim 128, window < T) against HF's model on the GPU."""
    import transformers

    from distributed_lion_pytorch_amd.models.llama import MistralForCausalLM

    hip.require()
    torch.manual_seed(3)
    cfg = transformers.MistralConfig(vocab_size=256, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                                     num_attention_heads=2, num_key_value_heads=1, max_position_embeddings=512,
                                     sliding_window=96)
    ours = MistralForCausalLM(cfg)
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        ours.save_pretrained(d)
        hf = transformers.MistralForCausalLM.from_pretrained(d)
    ours, hf = ours.to(cuda, torch.bfloat16), hf.to(cuda, torch.float32)
    ids = torch.randint(0, 256, (2, 300), device=cuda)
    la = ours(ids, labels=ids).loss
    lb = hf(ids, labels=ids).loss
    assert abs(la.item() - lb.item()) < 2e-2, (la.item(), lb.item())
    la.backward()
    lb.backward()
    for (n, p_), (_, r) in zip(ours.named_parameters(), hf.named_parameters()):
        if r.grad is not None and r.grad.abs().max() > 0:
            err = (p_.grad.float() - r.grad).abs().max().item() / r.grad.abs().max().item()
            assert err < 0.1, (n, err)


@pytest.mark.gpu
def test_packed_qkv_bias_grad_tail_tile(cuda):
    """GPT-2's fused c_attn + attention at T = 100: the kernels' per-tile bias
    partials cover ceil(T/32) tiles with the tail rows excluded."""
    from distributed_lion_pytorch_amd.ops.linear import grad_accumulation_fusion

    hip.require()
    torch.manual_seed(6)
    B, T, H, D = 2, 100, 2, 64
    C = H * D
    x = torch.randn(B, T, C, device=cuda).bfloat16().requires_grad_(True)
    w = torch.nn.Parameter((torch.randn(C, 3 * C, device=cuda) / C ** 0.5).bfloat16())
    b = torch.nn.Parameter((0.1 * torch.randn(3 * C, device=cuda)).bfloat16())
    dy = torch.randn(B, T, C, device=cuda).bfloat16()
    with grad_accumulation_fusion(False):
        y = fused.qkv_attention(x, w, b, H, 0.0)
        y.backward(dy)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    qkv = (xr @ wr + br).view(B, T, 3, H, D)
    yr = fused.reference_attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], 0.0, 0).view(B, T, C)
    yr.backward(dy.float())
    rel = lambda a, r: ((a.float() - r).abs().max() / (r.abs().max() + 1e-6)).item()  # noqa: E731
    assert rel(y, yr) < 2e-2
    for got, ref in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        assert rel(got, ref) < 3e-2, rel(got, ref)


def test_unsupported_head_dim_uses_math_sdpa_only(monkeypatch):
    """head_dim 80 has no flash kernel: the fallback is the math backend
    (ATen matmul + softmax), never the Triton-built flash / efficient ones."""
    from torch.nn.attention import SDPBackend

    seen = []
    import torch.nn.attention as att

    real = att.sdpa_kernel

    def spy(backends, *a, **k):
        seen.append(list(backends))
        return real(backends, *a, **k)

    monkeypatch.setattr(att, "sdpa_kernel", spy)
    q = torch.randn(1, 16, 2, 80)
    y = fused.causal_attention_gqa(q, q.clone(), q.clone())
    assert y.shape == (1, 16, 160)
    assert seen == [[SDPBackend.MATH]]
