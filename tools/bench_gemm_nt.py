"""Own gfx950 NT GEMM (csrc/gemm.hip) vs hipBLASLt (torch.matmul) on the GPT-2
training shapes, random operands, interleaved rounds in one process (guide
§5.4 rules 24/25).  Prints median us and TF/s per variant.

  python tools/bench_gemm_nt.py [M]
"""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from distributed_lion_pytorch_amd.ops import hip  # noqa: E402


def timed(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 20480
    ops = hip.ops()
    dt = torch.bfloat16
    # (name, N, K): forward y = x W^T-style and input-gradient shapes of GPT-2 small
    shapes = [("qkv fwd", 2304, 768), ("proj fwd", 768, 768), ("fc fwd", 3072, 768), ("fc_proj fwd", 768, 3072),
              ("qkv dgrad", 768, 2304), ("fc dgrad", 768, 3072), ("fc_proj dgrad", 3072, 768),
              ("lm_head fwd", 50304, 768)]
    for name, N, K in shapes:
        a = torch.rand(M, K, device="cuda", dtype=dt) * 2 - 1
        b = (torch.rand(N, K, device="cuda", dtype=dt) * 2 - 1) * 0.05
        bias = torch.rand(N, device="cuda", dtype=dt)
        fl = 2.0 * M * N * K
        variants = {
            "hipblaslt a@b.T": lambda: a @ b.t(),
            "hipblaslt linear+bias": lambda: torch.nn.functional.linear(a, b, bias),
            "own gemm_nt": lambda: ops.gemm_nt(a, b, None),
            "own gemm_nt+bias": lambda: ops.gemm_nt(a, b, bias),
        }
        if name == "fc fwd":
            variants["hipblaslt + bias_gelu"] = lambda: ops.bias_gelu_fwd(a @ b.t(), bias, False)
            variants["own gemm_nt_gelu"] = lambda: ops.gemm_nt_gelu(a, b, bias, False)
        for f in variants.values():
            f()
        torch.cuda.synchronize()
        res = {k: [] for k in variants}
        for _ in range(5):
            for k, f in variants.items():
                res[k].append(timed(f))
        print(f"{name:14s} M={M} N={N} K={K}", flush=True)
        for k, v in res.items():
            us = statistics.median(v)
            print(f"    {k:24s} {us:9.1f} us  {fl / us / 1e6:7.1f} TF/s  (min {min(v):.1f})", flush=True)


if __name__ == "__main__":
    main()
