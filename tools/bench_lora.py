"""Per-kernel timings of the LoRA streams (csrc/lora.hip) at the Llama-2-7B
LoRA SFT shape: 4096 tokens, K = N = 4096, r = 8, o / dout as column views of
a fused q|k|v projection output (row stride 12288).  Prints us and the
effective HBM bandwidth of each kernel's compulsory traffic."""
import argparse

import torch

from distributed_lion_pytorch_amd.ops import hip


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=4096)
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--r", type=int, default=8)
    a = ap.parse_args()
    ops = hip.ops()
    M, K, N, r = a.tokens, a.k, a.n, a.r
    dev = "cuda"
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    wide = torch.randn(M, 3 * N, device=dev, dtype=torch.bfloat16)
    o = wide[:, :N]
    A = torch.randn(r, K, device=dev, dtype=torch.bfloat16) * 0.05
    B = torch.randn(N, r, device=dev, dtype=torch.bfloat16) * 0.05
    u = ops.lora_rows(x, A, 1.0, 0.05, 1)
    du = ops.lora_rows(o, B.t().contiguous(), 2.0, 0.0, 0)
    mb = 1 << 20
    rows = [
        ("rows down (drop)", lambda: ops.lora_rows(x, A, 1.0, 0.05, 1), M * K * 2),
        ("rows du", lambda: ops.lora_rows(o, B.t().contiguous(), 2.0, 0.0, 0), M * N * 2),
        ("up", lambda: ops.lora_up(o, u, B, 2.0), 2 * M * N * 2),
        ("cols dB", lambda: ops.lora_cols(o, u, None, 2.0, 0.0, 0), M * N * 2),
        ("cols dA+dx", lambda: ops.lora_cols(x, du, A, 1.0, 0.05, 1), 2 * M * K * 2),
    ]
    calib = [("copy strided o", lambda: o.contiguous(), 2 * M * N * 2), ("clone x", lambda: x.clone(), 2 * M * K * 2),
             ("sum x (read)", lambda: x.sum(), M * K * 2)]
    tot = 0.0
    for name, fn, nbytes in rows:
        us = timeit(fn)
        tot += us
        print(f"{name:18s} {us:8.1f} us  {nbytes / mb:6.0f} MB  {nbytes / us / 1e6:5.2f} TB/s", flush=True)
    print(f"{'total':18s} {tot:8.1f} us")
    for name, fn, nbytes in calib:
        us = timeit(fn)
        print(f"{name:18s} {us:8.1f} us  {nbytes / mb:6.0f} MB  {nbytes / us / 1e6:5.2f} TB/s  (ATen calibration)")


if __name__ == "__main__":
    main()
