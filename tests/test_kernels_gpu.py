"""gfx950 kernel numerics vs the PyTorch oracle (same GPU, same inputs).

Multi-voter behaviour is exercised on ONE GPU by feeding the vote kernels W
locally generated bit planes ("fake voters")."""
import pytest
import torch

from distributed_lion_pytorch_amd.ops import hip
from distributed_lion_pytorch_amd.ops import reference as ref
from distributed_lion_pytorch_amd.optim.executors import HParams, HipExecutor, TorchExecutor
from distributed_lion_pytorch_amd.optim.plan import FlatPlan

pytestmark = pytest.mark.gpu

SIZES = [1, 7, 8, 13, 2047, 2048, 2049, 8192, 8193, 50257 * 3, 300_001]
DTYPES = [torch.float32, torch.bfloat16, torch.float16]


def _tensors(dtype, dev, seed=0, sizes=SIZES, misaligned=True):
    g = torch.Generator(device="cpu").manual_seed(seed)
    ps, gs, ms = [], [], []
    for i, n in enumerate(sizes):
        p = torch.randn(n, generator=g).to(dtype)
        gr = torch.randn(n, generator=g).to(dtype)
        m = (torch.randn(n, generator=g) * 0.5).to(dtype)
        if misaligned and i % 3 == 1:  # storage offset by one element: not 16-B aligned
            p = torch.cat([p.new_zeros(1), p])[1:]
        ps.append(p.to(dev))
        gs.append(gr.to(dev))
        ms.append(m.to(dev))
    return ps, gs, ms


def _clone(ts):
    return [t.clone() for t in ts]


def _assert_close(a, b, dtype, exact=True):
    """bf16: bit-exact with ATen-HIP (fma with fp32 alpha, RNE after every op;
    tools/probe_aten_numerics.py).  fp32: fp32 fma ordering may differ by an
    ulp.  fp16 and the fractional `average` deltas: within one ulp."""
    if dtype == torch.float32:
        torch.testing.assert_close(a, b, rtol=2e-7, atol=1e-7)
    elif dtype == torch.float16:
        # ATen-HIP's fp16 add(alpha) contracts to fma in its vectorised body but
        # not in the scalar tail of a tensor (tools/probe_fp16.py: all mismatches
        # sit in the last <1000 elements); the kernel always uses fma -> <= 1 ulp.
        torch.testing.assert_close(a.float(), b.float(), rtol=1e-3, atol=1e-5)
    elif not exact:
        torch.testing.assert_close(a.float(), b.float(), rtol=8e-3, atol=1e-5)
        assert (a != b).float().mean().item() < 1e-3
    else:
        assert torch.equal(a, b), (a - b).abs().max()


@pytest.fixture(autouse=True)
def _need_hip(cuda):
    hip.require()


@pytest.mark.parametrize("dtype", DTYPES)
def test_local_kernel_matches_oracle(dtype, cuda):
    ps, gs, ms = _tensors(dtype, cuda)
    plan = FlatPlan([(p, 0) for p in ps], world=1, bucket_bytes=1 << 14, device=cuda)
    hp = HParams(lr=1e-3, wd=0.1, beta1=0.9, beta2=0.99)
    p2, m2 = _clone(ps), _clone(ms)
    hx = HipExecutor(plan)
    meta = plan.meta(gs, ms)
    for b in plan.buckets:
        hx.local(meta, b, hp)
    for p, g, m in zip(p2, gs, m2):
        ref.update_fn(p, g, m, hp.lr, hp.wd, hp.beta1, hp.beta2)
    torch.cuda.synchronize()
    for a, b in zip(ps, p2):
        _assert_close(a, b, dtype)
    for a, b in zip(ms, m2):
        _assert_close(a, b, dtype)


@pytest.mark.parametrize("dtype", DTYPES)
def test_encode_kernel_matches_oracle(dtype, cuda):
    ps, gs, ms = _tensors(dtype, cuda, seed=1)
    plan = FlatPlan([(p, 0) for p in ps], world=4, bucket_bytes=1 << 13, device=cuda)
    hp = HParams(lr=1e-3, wd=0.0, beta1=0.9, beta2=0.99)
    bits_h = torch.full((plan.total_bytes,), 0xAB, dtype=torch.uint8, device=cuda)
    bits_t = torch.zeros_like(bits_h)
    m2 = _clone(ms)
    hx, tx = HipExecutor(plan), TorchExecutor(plan)
    meta = plan.meta(gs, ms)
    for b in plan.buckets:
        sl = slice(b.byte_off, b.byte_off + b.nbytes)
        used = sum((s.numel + 2047) // 2048 * 256 for s in b.segments)
        bits_h[b.byte_off + used:b.byte_off + b.nbytes] = 0  # bucket padding is not written by the kernel
        hx.encode(meta, b, bits_h[sl], hp)
        tx.encode(None, b, bits_t[sl], hp, grads=gs, moms=m2)
    torch.cuda.synchronize()
    assert torch.equal(bits_h, bits_t)
    for a, b in zip(ms, m2):
        _assert_close(a, b, dtype)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("world", [2, 3, 4, 8])
@pytest.mark.parametrize("mode,tie", [(ref.VOTE_MAJORITY, ref.TIE_NEGATIVE), (ref.VOTE_MAJORITY, ref.TIE_ZERO),
                                      (ref.VOTE_MAJORITY, ref.TIE_POSITIVE), (ref.VOTE_AVERAGE, 0)])
def test_vote_apply_kernel_fake_voters(dtype, world, mode, tie, cuda):
    ps, gs, ms = _tensors(dtype, cuda, seed=2)
    plan = FlatPlan([(p, 0) for p in ps], world=world, bucket_bytes=1 << 15, device=cuda)
    hp = HParams(lr=3e-3, wd=0.05, beta1=0.9, beta2=0.99)
    gen = torch.Generator(device="cpu").manual_seed(world)
    planes = torch.randint(0, 256, (world * plan.total_bytes,), generator=gen, dtype=torch.uint8).to(cuda)
    alive = torch.ones(world, dtype=torch.uint8, device=cuda)
    if world > 2:
        alive[1] = 0
    p2 = _clone(ps)
    hx, tx = HipExecutor(plan), TorchExecutor(plan)
    meta = plan.meta(gs, ms)
    agree = torch.zeros(2, dtype=torch.int64, device=cuda)  # [agreements, ties]
    agree_t = torch.zeros(2, dtype=torch.int64, device=cuda)
    for b in plan.buckets:
        pl = planes[world * b.byte_off: world * (b.byte_off + b.nbytes)]
        own = pl[: b.nbytes]
        hx.apply(meta, b, pl, b.nbytes, alive, mode, tie, None, hp, own=own, agree=agree)
        # oracle segments see the same p tensors through a plan over p2
        b2 = _rebind(b, p2, plan)
        tx.apply(None, b2, pl, b.nbytes, alive, mode, tie, None, hp, own=own, agree=agree_t)
    torch.cuda.synchronize()
    for a, b in zip(ps, p2):
        _assert_close(a, b, dtype, exact=mode != ref.VOTE_AVERAGE)
    assert agree.tolist() == agree_t.tolist()
    if mode == ref.VOTE_MAJORITY and world in (2, 3):  # an even live count (alive[1] = 0 for W > 2)
        assert agree[1].item() > 0  # even live count: random planes tie somewhere


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("tie", [ref.TIE_NEGATIVE, ref.TIE_ZERO])
def test_prevoted_apply_matches_oracle(dtype, tie, cuda):
    """K2 mode 2 (a2a path: one voted plane, optional neg plane) without
    telemetry -- the path of the two-chunks-per-block kernel: odd chunk counts,
    partial and misaligned tensors, full chunk pairs."""
    ps, gs, ms = _tensors(dtype, cuda, seed=3)
    plan = FlatPlan([(p, 0) for p in ps], world=4, bucket_bytes=1 << 16, device=cuda)
    hp = HParams(lr=3e-3, wd=0.05, beta1=0.9, beta2=0.99)
    gen = torch.Generator(device="cpu").manual_seed(7 + tie)
    pos = torch.randint(0, 256, (plan.total_bytes,), generator=gen, dtype=torch.uint8).to(cuda)
    neg = (torch.randint(0, 256, (plan.total_bytes,), generator=gen, dtype=torch.uint8).to(cuda) & ~pos
           if tie == ref.TIE_ZERO else None)
    alive = torch.ones(4, dtype=torch.uint8, device=cuda)
    p2 = _clone(ps)
    hx, tx = HipExecutor(plan), TorchExecutor(plan)
    meta = plan.meta(gs, ms)
    for b in plan.buckets:
        sl = slice(b.byte_off, b.byte_off + b.nbytes)
        ng = neg[sl] if neg is not None else None
        hx.apply(meta, b, pos[sl], b.nbytes, alive, ref.VOTE_PREVOTED, tie, ng, hp)
        tx.apply(None, _rebind(b, p2, plan), pos[sl], b.nbytes, alive, ref.VOTE_PREVOTED, tie, ng, hp)
    torch.cuda.synchronize()
    for a, b in zip(ps, p2):
        _assert_close(a, b, dtype)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("world", [3, 8])
@pytest.mark.parametrize("tie", [ref.TIE_NEGATIVE, ref.TIE_ZERO])
def test_majority_apply_without_telemetry(dtype, world, tie, cuda):
    """K2 majority (all-gather exchange) without the agreement counters: the
    two-chunks-per-block kernel when built with it, else the one-chunk kernel."""
    ps, gs, ms = _tensors(dtype, cuda, seed=4)
    plan = FlatPlan([(p, 0) for p in ps], world=world, bucket_bytes=1 << 16, device=cuda)
    hp = HParams(lr=3e-3, wd=0.05, beta1=0.9, beta2=0.99)
    gen = torch.Generator(device="cpu").manual_seed(11 * world + tie)
    planes = torch.randint(0, 256, (world * plan.total_bytes,), generator=gen, dtype=torch.uint8).to(cuda)
    alive = torch.ones(world, dtype=torch.uint8, device=cuda)
    alive[1] = 0
    p2 = _clone(ps)
    hx, tx = HipExecutor(plan), TorchExecutor(plan)
    meta = plan.meta(gs, ms)
    for b in plan.buckets:
        pl = planes[world * b.byte_off: world * (b.byte_off + b.nbytes)]
        hx.apply(meta, b, pl, b.nbytes, alive, ref.VOTE_MAJORITY, tie, None, hp)
        tx.apply(None, _rebind(b, p2, plan), pl, b.nbytes, alive, ref.VOTE_MAJORITY, tie, None, hp)
    torch.cuda.synchronize()
    for a, b in zip(ps, p2):
        _assert_close(a, b, dtype)


def _rebind(bucket, new_params, plan):
    import copy

    b2 = copy.copy(bucket)
    b2.segments = [copy.copy(s) for s in bucket.segments]
    for s in b2.segments:
        s.param = new_params[s.index]
    return b2


@pytest.mark.parametrize("world", [2, 5, 8])
@pytest.mark.parametrize("tie", [ref.TIE_NEGATIVE, ref.TIE_ZERO, ref.TIE_POSITIVE])
def test_vote_reduce_and_prevoted_apply(world, tie, cuda):
    nbytes = 4096 * 3
    gen = torch.Generator(device="cpu").manual_seed(tie * 10 + world)
    recv = torch.randint(0, 256, (world * nbytes,), generator=gen, dtype=torch.uint8).to(cuda)
    alive = torch.ones(world, dtype=torch.uint8, device=cuda)
    alive[world - 1] = 0
    outs = []
    for ex in (_bare_hip(), TorchExecutor.__new__(TorchExecutor)):
        pos = torch.zeros(nbytes, dtype=torch.uint8, device=cuda)
        neg = torch.zeros(nbytes, dtype=torch.uint8, device=cuda)
        ties = torch.zeros(1, dtype=torch.int64, device=cuda)
        ex.vote_reduce(recv, nbytes, alive, tie, pos, neg, ties)
        outs.append((pos, neg, ties))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    # tie telemetry (K4 under a2a): identical counts, non-zero exactly for an even live count
    assert outs[0][2].item() == outs[1][2].item()
    assert (outs[0][2].item() > 0) == ((world - 1) % 2 == 0)


def _bare_hip():
    h = HipExecutor.__new__(HipExecutor)
    h.ops = hip.ops()
    return h


def test_stochastic_encode_statistics(cuda):
    n = 1 << 20
    g = torch.zeros(n, dtype=torch.bfloat16, device=cuda)
    m = torch.zeros(n, dtype=torch.bfloat16, device=cuda)
    big = torch.full((n,), 50.0, dtype=torch.bfloat16, device=cuda)
    plan = FlatPlan([(g, 0), (big, 0)], world=2, device=cuda)
    meta = plan.meta([g, big], [m, m.clone()])
    hx = HipExecutor(plan)
    hp = HParams(lr=1e-3, wd=0.0, beta1=0.9, beta2=0.99)
    bits = torch.zeros(plan.total_bytes, dtype=torch.uint8, device=cuda)
    hx.encode(meta, plan.buckets[0], bits, hp, update_m=False, stochastic=True, rr=(1 + 1 / 0.9) * 1.0, seed=5,
              step=0)
    unpacked = ref.unpack_bits(bits)
    s0 = plan.buckets[0].segments[0]
    s1 = plan.buckets[0].segments[1]
    frac0 = unpacked[s0.bit_off:s0.bit_off + n].float().mean().item()  # u = 0 -> p = 1/2
    frac1 = unpacked[s1.bit_off:s1.bit_off + n].float().mean().item()  # u >> r -> p clamped to 1
    assert abs(frac0 - 0.5) < 0.01
    assert frac1 == 1.0
    bits2 = torch.zeros_like(bits)
    hx.encode(meta, plan.buckets[0], bits2, hp, update_m=False, stochastic=True, rr=(1 + 1 / 0.9), seed=5, step=1)
    assert not torch.equal(bits, bits2)  # fresh draws every step


def test_lion_optimizer_gpu_single_rank_matches_cpu_oracle(cuda):
    from distributed_lion_pytorch_amd import Lion

    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(64, 257), torch.nn.GELU(), torch.nn.Linear(257, 64)).bfloat16()
    net_ref = torch.nn.Sequential(torch.nn.Linear(64, 257), torch.nn.GELU(), torch.nn.Linear(257, 64)).bfloat16()
    net_ref.load_state_dict(net.state_dict())
    net, net_ref = net.to(cuda), net_ref.to(cuda)
    opt = Lion(net.parameters(), lr=1e-3, weight_decay=0.1)
    assert opt.backend == "auto"
    moms = [torch.zeros_like(p) for p in net_ref.parameters()]
    for step in range(3):
        x = torch.randn(16, 64, device=cuda).bfloat16()
        opt.zero_grad()
        net(x).float().pow(2).mean().backward()
        opt.step()
        net_ref.zero_grad()
        net_ref(x).float().pow(2).mean().backward()
        with torch.no_grad():
            for p, m in zip(net_ref.parameters(), moms):
                ref.update_fn(p, p.grad, m, 1e-3, 0.1, 0.9, 0.99)
    assert type(opt._executor).__name__ == "HipExecutor"
    for a, b in zip(net.parameters(), net_ref.parameters()):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dtype", DTYPES)
def test_fused_clip_matches_prescaled_grads(dtype, cuda):
    """grad_sumsq + clip_coef give the total L2 norm and clip_grad_norm_'s
    coefficient on the device; the update kernels fed that coefficient equal
    the same kernels run on gradients scaled in place (round(g * coef))."""
    ps, gs, ms = _tensors(dtype, cuda, seed=5)
    plan = FlatPlan([(p, 0) for p in ps], world=1, bucket_bytes=1 << 14, device=cuda)
    hp = HParams(lr=1e-3, wd=0.1, beta1=0.9, beta2=0.99)
    hx = HipExecutor(plan)
    meta = plan.meta(gs, ms)
    part = torch.empty(plan.total_chunks, dtype=torch.float32, device=cuda)
    out = torch.empty(2, dtype=torch.float32, device=cuda)
    for b in plan.buckets:
        hx.grad_sumsq(meta, b, part)
    max_norm = 1.0
    hx.clip_coef(part, plan.total_chunks, max_norm, out)
    norm = torch.linalg.vector_norm(torch.cat([g.double().reshape(-1) for g in gs]))
    torch.testing.assert_close(out[0].double(), norm, rtol=1e-5, atol=0)
    coef = min(1.0, max_norm / (out[0].item() + 1e-6))
    assert abs(out[1].item() - coef) <= 1e-6 * coef
    p0, m0 = _clone(ps), _clone(ms)
    bits_a = torch.zeros(plan.total_bytes, dtype=torch.uint8, device=cuda)
    bits_b = torch.zeros_like(bits_a)

    # fused: local step + encode read g and scale on load
    for b in plan.buckets:
        hx.local(meta, b, hp, gscale=out)
    pa, ma = _clone(ps), _clone(ms)
    for t, s in zip(ms, m0):
        t.copy_(s)
    for b in plan.buckets:
        hx.encode(meta, b, bits_a[b.byte_off:b.byte_off + b.nbytes], hp, gscale=out)
    ma_enc = _clone(ms)
    # reference: scale the gradients in place first, then the plain kernels
    for t, s in zip(ps, p0):
        t.copy_(s)
    for t, s in zip(ms, m0):
        t.copy_(s)
    for g in gs:
        g.copy_((g.float() * out[1]).to(dtype))
    for b in plan.buckets:
        hx.local(meta, b, hp)
    pb, mb = _clone(ps), _clone(ms)
    for t, s in zip(ms, m0):
        t.copy_(s)
    for b in plan.buckets:
        hx.encode(meta, b, bits_b[b.byte_off:b.byte_off + b.nbytes], hp)
    torch.cuda.synchronize()
    for a, b in zip(pa, pb):
        assert torch.equal(a, b)
    for a, b in zip(ma, mb):
        assert torch.equal(a, b)
    for a, b in zip(ma_enc, ms):
        assert torch.equal(a, b)
    assert torch.equal(bits_a, bits_b)


@pytest.mark.parametrize("n,rows,nseg", [(768, 1024, 1), (2304, 1024, 8), (3072, 256, 3), (64, 4096, 2)])
def test_sum_partials_tall_narrow_stacks(n, rows, nseg, cuda):
    """Narrow, tall fp32 partial stacks (bias / norm parameter gradients of a
    fusion window) take the row-split two-pass reduction: bf16 of the fp32 sum,
    deterministic, accumulate and scaled forms included."""
    hip.require()
    ops = hip.ops()
    torch.manual_seed(0)
    parts = [torch.randn(rows, n, device=cuda) for _ in range(nseg)]
    ref = torch.cat(parts).double().sum(0)
    out = torch.empty(n, device=cuda, dtype=torch.bfloat16)
    ops.sum_partials_multi_(parts, out, False)
    assert torch.allclose(out.double(), ref, rtol=1e-2, atol=1e-3 * ref.abs().max().item())
    out2 = torch.empty_like(out)
    ops.sum_partials_multi_(parts, out2, False)
    assert torch.equal(out, out2)
    acc = torch.ones(n, device=cuda, dtype=torch.bfloat16)
    ops.sum_partials_multi_(parts, acc, True)
    assert torch.allclose(acc.double(), ref + 1, rtol=1e-2, atol=1e-3 * ref.abs().max().item())
    single = ops.sum_partials(parts[0])
    ref0 = parts[0].double().sum(0)
    assert torch.allclose(single.double(), ref0, rtol=1e-2, atol=1e-3 * ref0.abs().max().item())
    s = torch.tensor([0.5], device=cuda)
    sc = torch.zeros(n, device=cuda, dtype=torch.bfloat16)
    ops.sum_partials_scaled_(parts[0], s, sc, False)
    assert torch.allclose(sc.double(), 0.5 * ref0, rtol=1e-2, atol=1e-3 * ref0.abs().max().item())
    # a row-strided slice (one of the [S, 3, C] norm parameter blocks)
    wide = torch.randn(rows, 3 * n, device=cuda)
    sl = wide[:, n:2 * n]
    assert torch.allclose(ops.sum_partials(sl).double(), sl.double().sum(0), rtol=1e-2,
                          atol=1e-3 * sl.double().sum(0).abs().max().item())


@pytest.mark.parametrize("R,C,Rp,dt", [(768, 3072, 768, torch.bfloat16), (3072, 768, 3072, torch.bfloat16),
                                        (50257, 768, 50304, torch.bfloat16), (100, 136, 104, torch.float16)])
def test_transpose_pad(R, C, Rp, dt, cuda):
    hip.require()
    x = torch.randn(R, C, device=cuda).to(dt)
    out = hip.ops().transpose_pad(x, Rp)
    assert out.shape == (C, Rp)
    assert torch.equal(out[:, :R], x.t())
    assert (out[:, R:] == 0).all()
    # row-strided input (a column slice of a wider matrix)
    wide = torch.randn(R, C + 16, device=cuda).to(dt)
    assert torch.equal(hip.ops().transpose_pad(wide[:, :C], Rp)[:, :R], wide[:, :C].t())
