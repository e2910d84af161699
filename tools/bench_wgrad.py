"""Weight-gradient GEMM variants at the GPT-2 shapes: dW[K,N] = x[M,K]^T dy[M,N].
Split-K factor sweep of the bmm(fp32 out) + fused reduction path vs hipBLASLt's own."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_lion_pytorch_amd.ops import hip  # noqa: E402


def t(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    ops = hip.ops()
    M = 20480
    for K, N in ((768, 2304), (768, 768), (768, 3072), (3072, 768)):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        g = torch.zeros(K, N, device="cuda", dtype=torch.bfloat16)
        fl = 2 * M * K * N
        res = {}
        for _ in range(3):
            res.setdefault("hipblaslt x^T dy", []).append(t(lambda: x.t() @ dy))
            for S in (2, 4, 8, 16, 32):
                xs, dys = x.view(S, M // S, K), dy.view(S, M // S, N)
                res.setdefault(f"splitK{S:2d} gemm only", []).append(
                    t(lambda: torch.bmm(xs.transpose(1, 2), dys, out_dtype=torch.float32)))
                res.setdefault(f"splitK{S:2d} +acc", []).append(
                    t(lambda: ops.sum_partials_acc_(torch.bmm(xs.transpose(1, 2), dys, out_dtype=torch.float32), g)))
        print(f"K={K} N={N}")
        for key, v in res.items():
            us = statistics.median(v)
            print(f"   {key:22s} {us:8.1f} us  {fl / us / 1e6:7.1f} TF/s")


if __name__ == "__main__":
    main()
