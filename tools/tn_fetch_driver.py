"""Fixed-shape driver for an HBM-traffic pass over the own TN kernel at the
GPT-2 window weight-gradient shapes (8 micro-batch segments of 20480 tokens,
the step's split counts): rocprofv3 --pmc FETCH_SIZE shows whether the
column tiles that share an output-gradient slab re-read it from HBM.
Ideal bytes per launch = every operand read once (printed)."""
import torch

from distributed_lion_pytorch_amd.ops import hip, linear

ops = hip.ops()
T, nmb = 20480, 8
for role, R, C in (("LM head", 50304, 768), ("MLP up", 3072, 768), ("c_attn", 2304, 768)):
    P = [torch.randn(T, R, device="cuda", dtype=torch.bfloat16) for _ in range(nmb)]
    Q = [torch.randn(T, C, device="cuda", dtype=torch.bfloat16) for _ in range(nmb)]
    s = linear.tn_split_factor(T * nmb, R, C, max_split=min(32, T * nmb // 128))
    ideal = T * nmb * (R + C) * 2 + s * R * C * 4
    print(f"{role}: R {R} C {C} splits {s}: ideal fetch {ideal / 2**30:.2f} GiB (operands once) + write {s * R * C * 4 / 2**20:.0f} MiB",
          flush=True)
    for _ in range(2):
        ops.gemm_tn(P, Q, s)
    torch.cuda.synchronize()
    del P, Q
    torch.cuda.empty_cache()
