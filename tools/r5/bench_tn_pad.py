"""Own TN weight-gradient kernel vs operand row-stride padding at the
Llama-3-8B shapes (8192 tokens, unsplit bf16 output), and the own NT kernel
with padded / unpadded leading dimensions at the o_proj shape: does a
power-of-two row stride cost the kernel, and which operand?
python tools/r5/bench_tn_pad.py"""
import torch

from distributed_lion_pytorch_amd.ops import hip


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def rows(T, n, pad):
    return torch.randn(T, n + pad, device="cuda", dtype=torch.bfloat16)[:, :n]


ops = hip.ops()
T = 8192
for name, R, C in [("o", 4096, 4096), ("qkv", 6144, 4096), ("down", 4096, 14336), ("gate_up", 28672, 4096)]:
    out = torch.empty(R, C, device="cuda", dtype=torch.bfloat16)
    line = f"{name:8s} [{R}x{C}]"
    for pp, pq in [(0, 0), (64, 0), (0, 64), (64, 64), (8, 8), (128, 128), (256, 256)]:
        dy, x = rows(T, R, pp), rows(T, C, pq)
        t = timeit(lambda: ops.gemm_tn_([dy], [x], out, False))
        line += f" | P+{pp} Q+{pq} {t:7.1f}us {2.0 * T * R * C / t / 1e9:4.2f}PF"
        del dy, x
    print(line, flush=True)
    torch.cuda.empty_cache()
# NT (own kernel): C[4096, 4096] = A[4096, 8192] . B[4096, 8192]^T, padded leading dims
line = "NT o-shape"
for pad in (0, 64, 128):
    a, b = rows(4096, 8192, pad), rows(4096, 8192, pad)
    t = timeit(lambda: ops.gemm_nt(a, b, None))
    line += f" | ld+{pad} {t:7.1f}us"
print(line, flush=True)
