"""Host-side (CPU) cost per launch of the ops on the training path: time N
back-to-back launches without synchronising (the GPU queue is kept deep by a
long warm-up kernel, so no launch ever blocks on the device)."""
import time

import torch
import torch.nn.functional as F

from distributed_lion_pytorch_amd.ops import hip


def host_us(fn, n=200):
    big = torch.empty(1 << 28, device="cuda", dtype=torch.bfloat16)
    for _ in range(40):  # ~queue a few ms of GPU work so launches below never wait
        big.mul_(1.0001)
    for _ in range(5):
        fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) / n * 1e6


def main():
    hip.require()
    ops = hip.ops()
    dev = torch.device("cuda")
    M, C, F4 = 2048, 768, 3072  # small M: the GPU side stays shorter than the host side
    x = torch.randn(M, C, device=dev).to(torch.bfloat16)
    w = torch.randn(F4, C, device=dev).to(torch.bfloat16)
    b = torch.randn(F4, device=dev).to(torch.bfloat16)
    out = torch.empty(M, F4, device=dev, dtype=torch.bfloat16)
    a3 = x.view(4, M // 4, C).transpose(1, 2)
    y3 = torch.randn(4, M // 4, F4, device=dev).to(torch.bfloat16)
    part = torch.randn(4, C * F4, device=dev)
    ops.lt_gemm_nt(x, w, None, None, 0, out)
    res = {
        "F.linear (hipBLASLt via ATen)": host_us(lambda: F.linear(x, w)),
        "F.linear + bias": host_us(lambda: F.linear(x, w, b)),
        "x @ w.t()": host_us(lambda: x @ w.t()),
        "bmm out_dtype=f32 (split-K wgrad)": host_us(lambda: torch.bmm(a3, y3, out_dtype=torch.float32)),
        "dlion lt_gemm_nt (cached algo)": host_us(lambda: ops.lt_gemm_nt(x, w, None, None, 0, out)),
        "dlion sum_partials": host_us(lambda: ops.sum_partials(part)),
        "x + x (ATen elementwise)": host_us(lambda: x + x),
        "empty_like": host_us(lambda: torch.empty_like(x)),
        "dlion bias_gelu_fwd": host_us(lambda: ops.bias_gelu_fwd(out, b, False)),
        "F.linear, 64 rows (launch-bound)": host_us(lambda: F.linear(x[:64], w)),
    }
    for k, v in res.items():
        print(f"{k:40s} {v:8.1f} us host/launch")


if __name__ == "__main__":
    main()
