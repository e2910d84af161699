"""Fixed-shape driver for PMC passes over the own TN and NT GEMMs
(tools/pmc_gemm_tn.sh): C[4096,4096] over K = 8192, 5 launches each."""
import torch

from distributed_lion_pytorch_amd.ops import hip

ops = hip.ops()
M = N = 4096
K = 8192
p = torch.randn(K, M, device="cuda", dtype=torch.bfloat16)
q = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
for _ in range(5):
    ops.gemm_tn([p], [q], 1)
    ops.gemm_nt(a, b, None)
torch.cuda.synchronize()
