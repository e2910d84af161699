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


def test_swiglu_on_fused_halves_and_fused_grad(cuda):
    """gate/up as the two column halves of one [.., 2F] buffer: read in place,
    backward returns [dgate | dup] as views of one buffer; matches fp32."""
    hip.require()
    torch.manual_seed(3)
    B, T, F = 2, 16, 96
    gu = torch.randn(B, T, 2 * F, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    g, u = gu[..., :F], gu[..., F:]
    h = fused.swiglu(g, u)
    dh = torch.randn_like(h)
    h.backward(dh)
    ref = gu.detach().float().requires_grad_(True)
    hr = torch.nn.functional.silu(ref[..., :F]) * ref[..., F:]
    hr.backward(dh.float())
    torch.testing.assert_close(h.float(), hr, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(gu.grad.float(), ref.grad, rtol=3e-2, atol=3e-2)


def test_rope_strided_token_rows(cuda):
    """q / k column slices of a fused projection output (token stride > H*D)."""
    hip.require()
    torch.manual_seed(4)
    B, T, H, D, extra = 2, 32, 4, 64, 128
    buf = torch.randn(B, T, H * D + extra, device=cuda, dtype=torch.bfloat16)
    x = buf[..., : H * D].view(B, T, H, D)
    cos = torch.randn(T, D, device=cuda, dtype=torch.bfloat16)
    sin = torch.randn(T, D, device=cuda, dtype=torch.bfloat16)
    assert fused._token_strided_ok(x)
    y = fused.rope(x, cos, sin)
    torch.testing.assert_close(y.float(), fused.rope_reference(x.float(), cos.float(), sin.float()),
                               rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("fuse", [False, True])
def test_linear_multi_matches_separate(fuse, cuda):
    """One GEMM on [Wq; Wk; Wv] == three linears: outputs, dx and every dW,
    accumulated over two micro-batches (gradient-accumulation fusion on/off)."""
    from distributed_lion_pytorch_amd.ops.linear import grad_accumulation_fusion, linear_multi_nk

    hip.require()
    torch.manual_seed(5)
    C, sizes = 256, (256, 64, 64)
    ws = [torch.nn.Parameter((torch.randn(n, C, device=cuda) * 0.05).to(torch.bfloat16)) for n in sizes]
    refs = [w.detach().float().clone().requires_grad_(True) for w in ws]
    xs = [torch.randn(2, 64, C, device=cuda, dtype=torch.bfloat16) for _ in range(2)]
    dxs = []
    with grad_accumulation_fusion(fuse):
        for x in xs:
            xx = x.clone().requires_grad_(True)
            outs = linear_multi_nk(xx, ws)
            loss = sum((o.float() * (i + 1)).sum() for i, o in enumerate(outs))
            loss.backward()
            dxs.append(xx.grad)
    for x, dx in zip(xs, dxs):
        xr = x.float().requires_grad_(True)
        outs = [xr @ w.t() for w in refs]
        sum((o * (i + 1)).sum() for i, o in enumerate(outs)).backward()
        torch.testing.assert_close(dx.float(), xr.grad, rtol=2e-2, atol=5e-2)
    for w, r in zip(ws, refs):
        err = (w.grad.float() - r.grad).abs().max().item() / r.grad.abs().max().item()
        assert err < 2e-2, err


@pytest.mark.parametrize("fused_bwd", [True, False])
@pytest.mark.parametrize("H,Hkv,T", [(4, 4, 128), (8, 2, 128), (8, 2, 100)])
def test_rope_attention_packed_grads(H, Hkv, T, fused_bwd, cuda, monkeypatch):
    """Fused RoPE + GQA attention on column views of a fused q|k|v output: the
    values and gradients match rope_reference + SDPA in fp32, and the three
    gradients come back as adjacent column blocks of one buffer (the fused
    projection's backward then needs no concatenation)."""
    from distributed_lion_pytorch_amd.ops import fused
    from distributed_lion_pytorch_amd.ops.linear import _adjacent_views

    hip.require()
    # fused_bwd: the attention backward kernels store dq / dk through the inverse
    # rotation; else a separate in-place rope pass over dq | dk
    monkeypatch.setattr(fused, "_ROPE_BWD_FUSED", fused_bwd)
    torch.manual_seed(H)
    B, D = 2, 128
    W = (H + 2 * Hkv) * D
    qkv = torch.randn(B, T, W, device=cuda).bfloat16().requires_grad_(True)
    q = qkv[..., :H * D].view(B, T, H, D)
    k = qkv[..., H * D:(H + Hkv) * D].view(B, T, Hkv, D)
    v = qkv[..., (H + Hkv) * D:].view(B, T, Hkv, D)
    inv = 1.0 / (10000 ** (torch.arange(0, D, 2, device=cuda).float() / D))
    f = torch.outer(torch.arange(T, device=cuda).float(), inv)
    emb = torch.cat([f, f], -1)
    cos, sin = emb.cos().bfloat16(), emb.sin().bfloat16()
    y = fused.rope_attention(q, k, v, cos, sin)
    dy = torch.randn_like(y)
    gq, gk, gv = torch.autograd.grad(y, (q, k, v), dy)
    assert _adjacent_views([g.reshape(B, T, -1) for g in (gq, gk, gv)]) is not None
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    qh = fused.rope_reference(qr, cos.float(), sin.float()).transpose(1, 2)
    kh = fused.rope_reference(kr, cos.float(), sin.float()).transpose(1, 2).repeat_interleave(H // Hkv, 1)
    vh = vr.transpose(1, 2).repeat_interleave(H // Hkv, 1)
    yr = torch.nn.functional.scaled_dot_product_attention(qh, kh, vh, is_causal=True).transpose(1, 2).reshape(B, T, -1)
    rq, rk, rv = torch.autograd.grad(yr, (qr, kr, vr), dy.float())
    rel = lambda a, r: ((a.float() - r).abs().max() / (r.abs().max() + 1e-6)).item()  # noqa: E731
    assert rel(y, yr) < 2e-2
    for got, ref in ((gq, rq), (gk, rk), (gv, rv)):
        assert rel(got, ref) < 3e-2, rel(got, ref)


def test_swiglu_bwd_transposed_copy(cuda):
    """swiglu_bwd_fused_t: the same dgu as swiglu_bwd_fused, plus dgu^T bit for bit."""
    hip.require()
    torch.manual_seed(11)
    rows, F = 256, 192
    gu = torch.randn(rows, 2 * F, device=cuda).to(torch.bfloat16)
    g, u = gu[:, :F], gu[:, F:]
    dh = torch.randn(rows, F, device=cuda).to(torch.bfloat16)
    ref = hip.ops().swiglu_bwd_fused(dh, g, u)
    dgu, dgut = hip.ops().swiglu_bwd_fused_t(dh, g, u)
    assert torch.equal(dgu, ref)
    assert torch.equal(dgut, dgu.t())


def test_gate_up_weight_gradient_uses_the_swiglu_transposed_copy(cuda, monkeypatch):
    """With the transposed-copy NT form picked for the gate/up weight
    gradient, the SwiGLU backward writes dgu^T itself and the weight gradient
    takes it instead of transposing dgu; all gradients match fp32."""
    from distributed_lion_pytorch_amd.ops import linear as L

    hip.require()
    torch.manual_seed(12)
    M, C, F = 4096, 1536, 1024  # C != 2F: the two operands' shapes differ
    x = torch.randn(M, C, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    wg = torch.nn.Parameter((torch.randn(F, C, device=cuda) / C ** 0.5).to(torch.bfloat16))
    wu = torch.nn.Parameter((torch.randn(F, C, device=cuda) / C ** 0.5).to(torch.bfloat16))
    dh = torch.randn(M, F, device=cuda, dtype=torch.bfloat16)
    monkeypatch.setattr(L, "_GEMM_PICK", {})
    monkeypatch.setattr(L, "_TT_A", {(M, 2 * F)})
    s, _ = L.wgrad_splits(torch.empty(M, 2 * F, device=cuda, dtype=torch.bfloat16), x.detach())
    L._GEMM_PICK[("wgrad", M, 2 * F, C, 2 * F, C, s)] = "lt_tt"
    shapes = []
    orig = L.fast_transpose
    monkeypatch.setattr(L, "fast_transpose", lambda t, *a: shapes.append(tuple(t.shape)) or orig(t, *a))
    with L.grad_accumulation_fusion(True, micro_batches=1):
        gate, up = L.linear_multi_nk(x, [wg, wu])
        fused.swiglu(gate, up).backward(dh)
    assert (M, 2 * F) not in shapes and (M, C) in shapes, shapes  # dgu^T came from the SwiGLU kernel
    assert not L._TCOPY
    xr, gr, ur = (t.detach().float().requires_grad_() for t in (x, wg, wu))
    (torch.nn.functional.silu(xr @ gr.t()) * (xr @ ur.t())).backward(dh.float())
    for got, ref in ((wg.grad, gr.grad), (wu.grad, ur.grad), (x.grad, xr.grad)):
        assert (got.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()


def test_swiglu_fwd_transposed_copy(cuda):
    """swiglu_fwd_t: the same h as swiglu_fwd, plus h^T bit for bit."""
    hip.require()
    torch.manual_seed(13)
    rows, F = 320, 128
    gu = torch.randn(rows, 2 * F, device=cuda).to(torch.bfloat16)
    g, u = gu[:, :F], gu[:, F:]
    h, ht = hip.ops().swiglu_fwd_t(g, u)
    assert torch.equal(h, hip.ops().swiglu_fwd(g, u))
    assert torch.equal(ht, h.t())


def test_down_proj_weight_gradient_uses_the_swiglu_forward_copy(cuda, monkeypatch):
    """The SwiGLU forward writes h^T when the down projection's weight
    gradient runs on token-contiguous copies; that gradient takes it."""
    from distributed_lion_pytorch_amd.ops import linear as L

    hip.require()
    torch.manual_seed(14)
    M, F, C = 8192, 1536, 1024  # h [M, F] feeds down_proj [C, F]; 2 M F C >= 2^34: a timed shape
    gu = torch.randn(M, 2 * F, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    wd = torch.nn.Parameter((torch.randn(C, F, device=cuda) / F ** 0.5).to(torch.bfloat16))
    dy = torch.randn(M, C, device=cuda, dtype=torch.bfloat16)
    monkeypatch.setattr(L, "_GEMM_PICK", {})
    monkeypatch.setattr(L, "_TT_B", {(M, F)})
    s, _ = L.wgrad_splits(dy, torch.empty(M, F, device=cuda, dtype=torch.bfloat16))
    L._GEMM_PICK[("wgrad", M, C, F, C, F, s)] = "lt_tt"
    shapes = []
    orig = L.fast_transpose
    monkeypatch.setattr(L, "fast_transpose", lambda t, *a: shapes.append(tuple(t.shape)) or orig(t, *a))
    with L.grad_accumulation_fusion(True, micro_batches=1):
        h = fused.swiglu(gu[:, :F], gu[:, F:])
        assert len(L._TCOPY) == 1
        L.linear_nk(h, wd).backward(dy)
    assert (M, F) not in shapes and (M, C) in shapes, shapes  # h^T came from the forward kernel
    assert not L._TCOPY
    gr = gu.detach().float()
    hr = torch.nn.functional.silu(gr[:, :F]) * gr[:, F:]
    ref = dy.float().t() @ hr
    assert (wd.grad.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()


def test_swiglu_forward_copy_only_when_a_backward_consumes_it(cuda, monkeypatch):
    """the SwiGLU forward writes h^T only when the down projection's
    weight gradient will take it -- not under no_grad (a frozen DPO reference
    model), not for frozen inputs, not inside a multi-micro-batch window
    (deferred / accumulated weight gradients read the row-major operand), and
    grad_accumulation_fusion's exit drops any unconsumed copy."""
    from distributed_lion_pytorch_amd.ops import linear as L

    hip.require()
    M, F = 256, 128
    gu = torch.randn(M, 2 * F, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    monkeypatch.setattr(L, "_TT_B", {(M, F)})
    with L.grad_accumulation_fusion(True, micro_batches=1):
        with torch.no_grad():
            fused.swiglu(gu[:, :F], gu[:, F:])
        assert not L._TCOPY
        frozen = gu.detach()
        fused.swiglu(frozen[:, :F], frozen[:, F:])
        assert not L._TCOPY
        h = fused.swiglu(gu[:, :F], gu[:, F:])  # the one case that writes it
        assert len(L._TCOPY) == 1
    assert not L._TCOPY  # unconsumed: dropped at the window's exit
    with L.grad_accumulation_fusion(True, micro_batches=4):
        fused.swiglu(gu[:, :F], gu[:, F:])
        assert not L._TCOPY
    del h
