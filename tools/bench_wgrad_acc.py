"""Split-K weight gradients under gradient accumulation, GPT-2 shapes.

A: per micro-batch bmm(fp32 partials) + sum_partials_acc_ into the bf16 grad
   (current path: one reduction launch per weight per micro-batch).
B: per micro-batch baddbmm(beta=1) into a persistent fp32 [S, K, N]
   accumulator (the GEMM epilogue reads and rewrites the partials), reduced to
   the bf16 grad once per optimizer step (1/GA of a sum_partials per micro-batch).
Prints us per micro-batch at GA = 8 and checks B against an fp32 reference."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_lion_pytorch_amd.ops import hip  # noqa: E402
from distributed_lion_pytorch_amd.ops.linear import split_k_factor  # noqa: E402

GA = 8


def t(fn, reps=GA * 3):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn(0)
    torch.cuda.synchronize()
    s.record()
    for i in range(reps):
        fn(i)
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
        s0 = split_k_factor(M, K, N)
        res = {}
        for S in sorted({s0, max(1, s0 // 2), min(32, s0 * 2)}):
            xs, dys = x.view(S, M // S, K).transpose(1, 2), dy.view(S, M // S, N)
            acc = torch.zeros(S, K, N, device="cuda", dtype=torch.float32)

            def cur(i):
                ops.sum_partials_acc_(torch.bmm(xs, dys, out_dtype=torch.float32), g)

            def new(i):
                if i % GA == 0:
                    torch.bmm(xs, dys, out_dtype=torch.float32, out=acc)
                else:
                    torch.baddbmm(acc, xs, dys, out_dtype=torch.float32, out=acc)
                if i % GA == GA - 1:
                    ops.sum_partials_acc_(acc, g)

            for _ in range(3):
                res.setdefault(f"S={S:2d} bmm+reduce/mb", []).append(t(cur))
                res.setdefault(f"S={S:2d} baddbmm acc", []).append(t(new))
            # numerics: GA micro-batches accumulated in fp32 == GA x (x^T dy)
            acc.zero_()
            for i in range(GA):
                new(i)
            ref = (x.float().t() @ dy.float())
            got = acc.sum(0)
            err = ((got - GA * ref).abs().max() / (GA * ref).abs().max()).item()
            res[f"S={S:2d} rel err"] = [err]
        print(f"K={K} N={N} (default S={s0})")
        for key, v in res.items():
            if key.endswith("rel err"):
                print(f"   {key:24s} {v[0]:.2e}")
                continue
            us = statistics.median(v)
            print(f"   {key:24s} {us:8.1f} us  {fl / us / 1e6:7.1f} TF/s")


if __name__ == "__main__":
    main()
