"""Numerics of the gfx950 NT GEMM (csrc/gemm.hip) against fp32 PyTorch references."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ops():
    from distributed_lion_pytorch_amd.ops import hip

    hip.require()
    return hip.ops()


def _ref(a, b, bias=None):
    out = a.float() @ b.float().t()
    if bias is not None:
        out = out + bias.float()
    return out


def _check(got, ref, K):
    # bf16 output rounding (2^-8 relative) + fp32-accumulation-order noise
    err = (got.float() - ref).abs()
    tol = 1e-2 * ref.abs() + 2e-3 * (K ** 0.5)
    bad = (err > tol).sum().item()
    assert bad == 0, f"{bad} / {err.numel()} elements off; max err {err.max().item():.4g}"


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (512, 768, 768), (20480 // 8, 2304, 768), (300, 136, 256),
                                   (1000, 50304 // 4, 768), (2048, 768, 3072),
                                   # > 256 tiles: persistent blocks walk several tiles (edge tiles too)
                                   (4160, 4352, 256), (8448, 2048, 128), (5000, 3000, 384)])
def test_gemm_nt_plain_and_bias(M, N, K):
    ops = _ops()
    torch.manual_seed(0)
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    bias = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    _check(ops.gemm_nt(a, b, None), _ref(a, b), K)
    _check(ops.gemm_nt(a, b, bias), _ref(a, b, bias), K)


def test_gemm_nt_asymmetric_exact():
    """Small-integer operands: every product and partial sum is exact in fp32,
    so any transposed / misplaced element shows up as an exact mismatch."""
    ops = _ops()
    torch.manual_seed(1)
    M, N, K = 512, 512, 256
    a = torch.randint(-3, 4, (M, K), device="cuda").to(torch.bfloat16)
    b = torch.randint(-3, 4, (N, K), device="cuda").to(torch.bfloat16)
    b[:, 0] += torch.arange(N, device="cuda").to(torch.bfloat16) % 7  # asymmetric in (row, col)
    ref = _ref(a, b).to(torch.bfloat16).float()  # exact sums, one RNE rounding either way
    assert torch.equal(ops.gemm_nt(a, b, None).float(), ref)


def test_gemm_nt_strided_rows_and_out():
    ops = _ops()
    torch.manual_seed(2)
    big = torch.randn(512, 3 * 256, device="cuda", dtype=torch.bfloat16)
    a = big[:, 256:512]  # row stride 768
    b = torch.randn(384, 256, device="cuda", dtype=torch.bfloat16) * 0.1
    out = torch.full((512, 512), 7.0, device="cuda", dtype=torch.bfloat16)
    ops.gemm_nt_out(a, b, None, out[:, :384])
    _check(out[:, :384], _ref(a, b), 256)
    assert torch.all(out[:, 384:] == 7.0)


def test_transposed_weight_cache_follows_lion_updates():
    """linear_kn runs the Conv1D forward on a cached W^T; a Lion step writes the
    weights through raw pointers and must invalidate that copy."""
    from distributed_lion_pytorch_amd import Lion
    from distributed_lion_pytorch_amd.ops.linear import linear_kn

    _ops()
    torch.manual_seed(4)
    w = torch.nn.Parameter(torch.randn(256, 384, device="cuda", dtype=torch.bfloat16))
    x = torch.randn(64, 256, device="cuda", dtype=torch.bfloat16)
    y0 = linear_kn(x, w)
    _check(y0, x.float() @ w.float(), 256)
    w.grad = torch.randn_like(w)
    Lion([w], lr=0.05).step()
    y1 = linear_kn(x, w)
    _check(y1, x.float() @ w.float(), 256)
    assert not torch.equal(y0, y1)


@pytest.mark.parametrize("exact", [False, True])
def test_gemm_nt_gelu_matches_unfused(exact):
    ops = _ops()
    torch.manual_seed(3)
    M, N, K = 1024, 3072, 768
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    bias = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    h, z = ops.gemm_nt_gelu(a, b, bias, exact)
    z_ref = ops.gemm_nt(a, b, None)
    assert torch.equal(z, z_ref)
    assert torch.equal(h, ops.bias_gelu_fwd(z_ref, bias, exact))
    ref = torch.nn.functional.gelu(_ref(a, b, bias), approximate="none" if exact else "tanh")
    _check(h, ref, K)
