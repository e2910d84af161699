"""Microbenchmark of the fused add+norm kernels (GPT-2 bench shape by default).

python tools/bench_norm.py [--rows 20480] [--C 768] [--parts 128,256,512,1024]
Prints per-call time and effective HBM bandwidth of add_norm_fwd / add_norm_bwd
(+ the partial reduction) and bias_gelu fwd/bwd.
"""
import argparse

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_lion_pytorch_amd.ops import hip


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=20480)
    ap.add_argument("--C", type=int, default=768)
    ap.add_argument("--parts", default="64,128,256,512,1024,2048")
    a = ap.parse_args()
    ops = hip.ops()
    dev = "cuda"
    R, C = a.rows, a.C
    x = torch.randn(R, C, device=dev, dtype=torch.bfloat16)
    y = torch.randn_like(x)
    g = torch.ones(C, device=dev, dtype=torch.bfloat16)
    b = torch.zeros_like(g)
    xo, h, mean, rstd = ops.add_norm_fwd(x, y, b, g, b, 1e-5, False, 0.1, 7)
    t = timeit(lambda: ops.add_norm_fwd(x, y, b, g, b, 1e-5, False, 0.1, 7))
    print(f"add_norm_fwd   {t:8.1f} us  {4 * R * C * 2 / t / 1e3:7.1f} GB/s")
    dh, dxo = torch.randn_like(x), torch.randn_like(x)
    for p in [int(v) for v in a.parts.split(",")]:
        t = timeit(lambda: ops.add_norm_bwd(dh, dxo, xo, g, mean, rstd, False, 0.1, 7, True, p))
        t2 = timeit(lambda: ops.sum_partials(ops.add_norm_bwd(dh, dxo, xo, g, mean, rstd, False, 0.1, 7, True, p)[2]))
        print(f"add_norm_bwd parts={p:5d} {t:8.1f} us  {5 * R * C * 2 / t / 1e3:7.1f} GB/s   +sum {t2:8.1f} us")
    N = 4 * C
    z = torch.randn(R, N, device=dev, dtype=torch.bfloat16)
    bb = torch.zeros(N, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: ops.bias_gelu_fwd(z, bb, False))
    print(f"bias_gelu_fwd  {t:8.1f} us  {2 * R * N * 2 / t / 1e3:7.1f} GB/s")
    dz = torch.randn_like(z)
    for p in (256, 1024, 2560):
        t = timeit(lambda: ops.bias_gelu_bwd(dz, z, bb, False, p))
        t2 = timeit(lambda: ops.sum_partials(ops.bias_gelu_bwd(dz, z, bb, False, p)[1]))
        print(f"bias_gelu_bwd parts={p:5d} {t:8.1f} us  {3 * R * N * 2 / t / 1e3:7.1f} GB/s   +sum {t2:8.1f} us")


if __name__ == "__main__":
    main()
