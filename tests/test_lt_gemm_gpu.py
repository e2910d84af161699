"""hipBLASLt GEMMs with fused epilogues (csrc/lt_gemm.cpp) vs fp32 PyTorch:
plain, + bias, gelu_tanh(z + bias); strided operand rows; and the GPT-2 MLP's
no-grad forward that uses the GELU epilogue."""
import pytest
import torch
import torch.nn.functional as F

from distributed_lion_pytorch_amd.ops import hip

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-6)).item()


@pytest.mark.parametrize("M,N,K", [(2048, 3072, 768), (512, 384, 256), (1000, 520, 128)])
@pytest.mark.parametrize("epi", [0, 1, 2])
def test_lt_gemm_epilogues(M, N, K, epi, cuda):
    hip.require()
    torch.manual_seed(epi)
    a = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    b = (torch.randn(N, K, device=cuda) / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, device=cuda).to(torch.bfloat16) if epi else None
    out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    assert hip.ops().lt_gemm_nt(a, b, bias, epi, out), f"hipBLASLt has no kernel for epilogue {epi}"
    ref = a.float() @ b.float().t()
    if epi:
        ref = ref + bias.float()
    if epi == 2:
        ref = F.gelu(ref, approximate="tanh")
    assert _rel(out, ref) < 1.5e-2, (epi, _rel(out, ref))
    # the cached (tuned) algorithm gives the same result on a second call
    out2 = torch.empty_like(out)
    assert hip.ops().lt_gemm_nt(a, b, bias, epi, out2)
    assert torch.equal(out, out2)


@pytest.mark.parametrize("M,N,K", [(2048, 768, 3072), (1000, 520, 136)])
def test_lt_gemm_nn(M, N, K, cuda):
    """out = a . b with b [K, N] row-major (the input gradient dY . W without a W^T copy)."""
    hip.require()
    torch.manual_seed(3)
    a = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    b = (torch.randn(K, N, device=cuda) / K ** 0.5).to(torch.bfloat16)
    out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    assert hip.ops().lt_gemm_nn(a, b, out)
    assert _rel(out, a.float() @ b.float()) < 1e-2
    out2 = torch.empty_like(out)
    assert hip.ops().lt_gemm_nn(a, b, out2) and torch.equal(out, out2)


@pytest.mark.parametrize("accumulate", [False, True])
def test_lt_gemm_tn(accumulate, cuda):
    """out (+)= a^T . b over the token axis (a weight gradient), beta = 1 when accumulating."""
    hip.require()
    torch.manual_seed(4)
    a = torch.randn(1024, 384, device=cuda).to(torch.bfloat16)
    b = (torch.randn(1024, 256, device=cuda) / 32).to(torch.bfloat16)
    init = torch.randn(384, 256, device=cuda).to(torch.bfloat16)
    out = init.clone()
    assert hip.ops().lt_gemm_tn(a, b, out, accumulate)
    ref = a.float().t() @ b.float() + (init.float() if accumulate else 0)
    assert _rel(out, ref) < 1e-2
    out2 = init.clone()  # the tuning runs went to a scratch output: a second call adds once more
    assert hip.ops().lt_gemm_tn(a, b, out2, accumulate) and torch.equal(out, out2)


def test_lt_gemm_strided_rows(cuda):
    hip.require()
    torch.manual_seed(1)
    base = torch.randn(256, 3 * 256, device=cuda).to(torch.bfloat16)
    a = base[:, 256:512]  # row stride 768
    b = torch.randn(384, 256, device=cuda).to(torch.bfloat16)
    out = torch.empty(256, 384, device=cuda, dtype=torch.bfloat16)
    assert hip.ops().lt_gemm_nt(a, b, None, 0, out)
    assert _rel(out, a.float() @ b.float().t()) < 1e-2


def test_linear_gelu_no_grad_uses_epilogue(cuda):
    """Evaluation forward of the GPT-2 MLP up-projection: one GEMM with the
    GELU epilogue; same values as the training path (GEMM + bias_gelu)."""
    from distributed_lion_pytorch_amd.ops import fused

    hip.require()
    torch.manual_seed(2)
    x = torch.randn(512, 256, device=cuda).to(torch.bfloat16)
    w = torch.nn.Parameter((torch.randn(256, 1024, device=cuda) * 0.05).to(torch.bfloat16))
    b = torch.nn.Parameter((torch.randn(1024, device=cuda) * 0.05).to(torch.bfloat16))
    train = fused.linear_gelu(x, w, b)
    with torch.no_grad():
        ev = fused.linear_gelu(x, w, b)
    ref = F.gelu(x.float() @ w.float() + b.float(), approximate="tanh")
    assert _rel(train, ref) < 1.5e-2 and _rel(ev, ref) < 1.5e-2
    assert _rel(ev, train) < 1.5e-2


@pytest.mark.parametrize("layout", [0, 1, 2, 3])
def test_lt_gemm_layouts(layout, cuda):
    """lt_gemm_layout: NT / NN / TN / TT operand layouts, with and without beta = 1."""
    hip.require()
    torch.manual_seed(10 + layout)
    M, N, K = 384, 256, 512
    A = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    B = (torch.randn(K, N, device=cuda) / 16).to(torch.bfloat16)
    a = A.t().contiguous() if layout >= 2 else A          # stored [K, M] for TN / TT
    b = B.t().contiguous() if layout in (0, 3) else B     # stored [N, K] for NT / TT
    ref = A.float() @ B.float()
    init = torch.randn(M, N, device=cuda).to(torch.bfloat16)
    for acc in (False, True):
        out = init.clone()
        assert hip.ops().lt_gemm_layout(a, b, out, layout, acc)
        assert _rel(out, ref + (init.float() if acc else 0)) < 1e-2, (layout, acc)
