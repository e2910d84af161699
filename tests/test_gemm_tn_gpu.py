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
        assert bool(L._ST.wdefer) == defer
        assert w.grad is None  # nothing reduced before the window closes
    assert not L._ST.wdefer
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
    assert not L._ST.wdefer
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


@pytest.mark.parametrize("M,N,rows,nseg", [(256, 256, 128, 1), (776, 264, 256, 2), (1024, 4096, 1024, 1)])
def test_gemm_tn_bf16_out_matches_fp32(cuda, M, N, rows, nseg):
    """Unsplit bf16 output (the gradient written from the accumulators, no fp32
    partials) and its accumulate form: bf16(P^T Q + old) as sum_partials rounds."""
    hip.require()
    torch.manual_seed(2)
    P = [torch.randn(rows, M, device=cuda, dtype=torch.bfloat16) for _ in range(nseg)]
    Q = [torch.randn(rows, N, device=cuda, dtype=torch.bfloat16) for _ in range(nseg)]
    ref = torch.cat(P).float().t() @ torch.cat(Q).float()
    out = torch.full((M, N), float("nan"), device=cuda, dtype=torch.bfloat16)
    hip.ops().gemm_tn_(P, Q, out, False)
    assert (out.float() - ref).abs().max().item() <= 1e-2 * ref.abs().max().item()
    # same rounding as the fp32-partial path it replaces
    part = hip.ops().gemm_tn(P, Q, 1)
    assert torch.equal(out, hip.ops().sum_partials(part.view(1, -1)).view(M, N))
    old = torch.randn(M, N, device=cuda, dtype=torch.bfloat16)
    acc = old.clone()
    hip.ops().gemm_tn_(P, Q, acc, True)
    exp = old.clone()
    hip.ops().sum_partials_acc_(part.view(1, -1), exp.view(-1))
    assert torch.equal(acc, exp)


def test_unsplit_wgrad_into_and_fused_projection_grads(cuda):
    """Llama-sized weights take the unsplit bf16 path in wgrad_into / the fused
    q/k/v weight gradient (ops/linear.py); grads equal autograd's."""
    from distributed_lion_pytorch_amd.ops import linear as L

    hip.require()
    torch.manual_seed(3)
    T, K = 1024, 4096
    ws = [torch.nn.Parameter((torch.randn(n, K, device=cuda) * 0.02).to(torch.bfloat16)) for n in (2048, 1024, 1024)]
    assert L.wgrad_splits(torch.empty(T, 4096, device=cuda, dtype=torch.bfloat16),
                          torch.empty(T, K, device=cuda, dtype=torch.bfloat16)) == (1, True)
    x = torch.randn(T, K, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    refs = [w.detach().float().requires_grad_() for w in ws]
    for step in range(2):  # one-micro-batch windows (TrainStep, grad_accum 1); the second accumulates
        with L.grad_accumulation_fusion(True, micro_batches=1):
            outs = L.linear_multi_nk(x, ws)
            gs = [torch.randn_like(o) for o in outs]
            torch.autograd.backward(outs, gs)
        ro = [x.detach().float() @ r.t() for r in refs]
        torch.autograd.backward(ro, [g.float() for g in gs])
    for w, r in zip(ws, refs):
        assert (w.grad.float() - r.grad).abs().max().item() <= 2e-2 * r.grad.abs().max().item()
    base = L._adjacent_rows([w.grad for w in ws])
    assert base is not None and base.shape == (4096, K)
    # single linear: wgrad_into s == 1
    w1 = torch.nn.Parameter((torch.randn(4096, K, device=cuda) * 0.02).to(torch.bfloat16))
    with L.grad_accumulation_fusion(True, micro_batches=1):
        y = L.linear_nk(x, w1)
        g = torch.randn_like(y)
        y.backward(g)
    ref = g.float().t() @ x.detach().float()
    assert (w1.grad.float() - ref).abs().max().item() <= 1e-2 * ref.abs().max().item()


def test_cat_weights_refreshes_in_place_after_step(cuda):
    """Trainable fused-projection weights: after an optimizer step the cached
    concatenation is refreshed into the same buffer (no reallocation)."""
    from distributed_lion_pytorch_amd.ops import linear as L

    ws = [torch.nn.Parameter(torch.randn(n, 256, device=cuda, dtype=torch.bfloat16)) for n in (256, 128, 128)]
    c1 = L.cat_weights(ws)
    assert torch.equal(c1, torch.cat([w.detach() for w in ws]))
    ptr = c1.data_ptr()
    assert L.cat_weights(ws) is c1  # cached within a step
    with torch.no_grad():
        for w in ws:
            w.add_(1.0)
    L.bump_weight_generation()
    c2 = L.cat_weights(ws)
    assert c2.data_ptr() == ptr and torch.equal(c2, torch.cat([w.detach() for w in ws]))


def test_pack_projections_zero_copy_fused_weights(cuda):
    """Trainable q/k/v-style weights are re-pointed at one buffer on first fused
    use: the concatenation is then a view (no per-step copy), the HIP Lion step
    -- whose pointer table was built before the move -- updates the new storage,
    and the state dict still round-trips."""
    from distributed_lion_pytorch_amd import Lion
    from distributed_lion_pytorch_amd.ops import linear as L

    hip.require()
    torch.manual_seed(11)
    ws = [torch.nn.Parameter((0.02 * torch.randn(n, 256, device=cuda)).to(torch.bfloat16)) for n in (256, 128, 128)]
    opt = Lion(ws, lr=1e-2, weight_decay=0.0)
    x = torch.randn(384, 256, device=cuda, dtype=torch.bfloat16)
    for w in ws:
        w.grad = torch.randn_like(w)
    opt.step()  # plan + pointer table on the original storage
    before = [w.detach().clone() for w in ws]
    outs = L.linear_multi_nk(x, ws)  # packs
    assert L._adjacent_rows([w.detach() for w in ws]) is not None
    for o, w in zip(outs, before):
        ref = x.float() @ w.float().t()
        assert (o.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()
    cat = L.cat_weights(ws)
    assert cat.data_ptr() == ws[0].data_ptr() and L.cat_weights(ws) is cat
    grads = [torch.randn_like(w) for w in ws]
    for w, g in zip(ws, grads):
        w.grad = g.clone()
    opt.step()  # must write through the new pointers
    for w, b0 in zip(ws, before):
        assert not torch.equal(w.detach(), b0), "the step did not reach the packed storage"
    L.bump_weight_generation()
    assert torch.equal(L.cat_weights(ws), torch.cat([w.detach() for w in ws]))
    sd = {f"w{i}": w.detach().clone() for i, w in enumerate(ws)}
    with torch.no_grad():
        for w in ws:
            w.zero_()
        for i, w in enumerate(ws):
            w.copy_(sd[f"w{i}"])
    assert all(torch.equal(w.detach(), sd[f"w{i}"]) for i, w in enumerate(ws))


def test_gemm_autotune_candidates_agree(cuda):
    """Every candidate the per-shape GEMM choice may pick (ATen NN/NT, own NT,
    tuned hipBLASLt) computes the same product; the pick is cached per shape."""
    from distributed_lion_pytorch_amd.ops import linear as L

    hip.require()
    torch.manual_seed(5)
    M, N, K = 4096, 4096, 1536
    x = torch.randn(M, K, device=cuda, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) * 0.02).to(torch.bfloat16)
    ref = x.float() @ w.float().t()
    for name, fn in L._nt_candidates(x, w, "").items():
        assert (fn().float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item(), name
    y = L.gemm_fwd(x, w)
    assert ("fwd", M, N, K, x.stride(0), w.stride(0), False) in L._GEMM_PICK
    assert (y.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()
    dy = torch.randn(M, N, device=cuda, dtype=torch.bfloat16)
    dref = dy.float() @ w.float()
    for frozen in (True, False):
        dx = L.gemm_dgrad(dy, w, frozen)
        assert (dx.float() - dref).abs().max().item() <= 2e-2 * dref.abs().max().item()
    assert ("dgrad", M, N, K, dy.stride(0), False) in L._GEMM_PICK
    # a trainable weight's W^T follows the weight across an optimizer step
    wp = torch.nn.Parameter(w.clone())
    L._GEMM_PICK[("dgrad", M, N, K, dy.stride(0), False)] = "nt_aten"
    d1 = L.gemm_dgrad(dy, wp, False)
    with torch.no_grad():
        wp.mul_(-1.0)
    L.bump_weight_generation()
    d2 = L.gemm_dgrad(dy, wp, False)
    assert (d2.float() + dref).abs().max().item() <= 2e-2 * dref.abs().max().item()  # the new weight's W^T
    assert (d1.float() - dref).abs().max().item() <= 2e-2 * dref.abs().max().item()


@pytest.mark.parametrize("choice", ["tn", "blas", "lt", "lt_tt", "split"])
def test_unsplit_wgrad_choices(cuda, choice):
    """Every candidate of the timed weight gradient (own TN bf16 epilogue,
    ATen's hipBLASLt TN, hipBLASLt TN with the searched algorithm and beta = 1,
    own split-K partials + reduction) writes and accumulates the same gradient."""
    from distributed_lion_pytorch_amd.ops import linear as L

    hip.require()
    torch.manual_seed(6)
    M, K, N = 2048, 2048, 4096
    a = torch.randn(M, K, device=cuda, dtype=torch.bfloat16)
    b = torch.randn(M, N, device=cuda, dtype=torch.bfloat16)
    split = 2 if choice == "split" else 1
    L._GEMM_PICK[("wgrad", M, K, N, a.stride(0), b.stride(0), split)] = choice
    ref = a.float().t() @ b.float()
    out = torch.empty(K, N, device=cuda, dtype=torch.bfloat16)
    L._unsplit_wgrad(a, b, out, False, split)
    assert (out.float() - ref).abs().max().item() <= 1e-2 * ref.abs().max().item()
    L._unsplit_wgrad(a, b, out, True, split)
    assert (out.float() - 2 * ref).abs().max().item() <= 2e-2 * ref.abs().max().item()


def test_direct_split_weight_gradient_goes_through_the_timed_pick(cuda, monkeypatch):
    """Outside a multi-micro-batch window a split weight gradient (Llama-3-8B
    q/k/v at s = 2) is timed against the unsplit candidates; the fused q/k/v
    gradient blocks come out right whichever wins."""
    from distributed_lion_pytorch_amd.ops import linear as L

    hip.require()
    torch.manual_seed(7)
    M, K = 4096, 2048
    sizes = [2048, 512, 512]
    monkeypatch.setattr(L, "tn_split_factor", lambda *a, **k: 2)
    monkeypatch.setattr(L, "_GEMM_PICK", {})
    dy = torch.randn(M, sum(sizes), device=cuda, dtype=torch.bfloat16)
    x = torch.randn(M, K, device=cuda, dtype=torch.bfloat16)
    ps = [torch.nn.Parameter(torch.zeros(n, K, device=cuda, dtype=torch.bfloat16)) for n in sizes]
    assert L._direct_split_pick(dy, x, 2, True)
    with L.grad_accumulation_fusion(True, micro_batches=1):
        L._multi_wgrad_into(dy, x, ps, sizes)
    key = [k for k in L._GEMM_PICK if k[0] == "wgrad"]
    assert key and key[0][-1] == 2, L._GEMM_PICK
    ref = dy.float().t() @ x.float()
    got = torch.cat([p.grad.float() for p in ps], 0)
    assert (got - ref).abs().max().item() <= 1e-2 * ref.abs().max().item()
