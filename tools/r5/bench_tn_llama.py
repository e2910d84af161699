"""Own TN weight-gradient kernel at the Llama-3-8B shapes (8192 tokens):
unsplit bf16 output vs split fp32 partials, plus the own NT kernel and
hipBLASLt's NT GEMM at the same FLOPs (dW = dY^T X with token-contiguous
copies), and the effect of padding the operand row stride (channel camping
check).  python tools/r5/bench_tn_llama.py"""
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


ops = hip.ops()
T = 8192
for name, R, C in [("o", 4096, 4096), ("qkv", 6144, 4096), ("down", 4096, 14336), ("gate_up", 28672, 4096)]:
    flop = 2.0 * T * R * C
    dy = torch.randn(T, R, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, C, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(R, C, device="cuda", dtype=torch.bfloat16)
    line = f"{name:8s} [{R}x{C}] "
    t1 = timeit(lambda: ops.gemm_tn_([dy], [x], out, False))
    line += f"TN s=1 bf16 {t1:7.1f}us {flop / t1 / 1e9:4.2f}PF"
    for s in (2, 3, 4):
        part = torch.empty(s, R, C, device="cuda", dtype=torch.float32)
        ts = timeit(lambda: ops.gemm_tn_([dy], [x], part, False))
        tr = timeit(lambda: ops.sum_partials(part.view(s, -1)))
        line += f" | s={s} {ts:7.1f}+{tr:5.1f}us"
        del part
    # padded row strides (+64 elements)
    dyp = torch.randn(T, R + 64, device="cuda", dtype=torch.bfloat16)[:, :R]
    xp = torch.randn(T, C + 64, device="cuda", dtype=torch.bfloat16)[:, :C]
    tp = timeit(lambda: ops.gemm_tn_([dyp], [xp], out, False))
    line += f" | padded-ld {tp:7.1f}us"
    print(line, flush=True)
    del dyp, xp
    # NT forms at equal FLOPs: C[R, C] = A[R, T] . B[C, T]^T
    a = dy.t().contiguous()
    b = x.t().contiguous()
    tn_own = timeit(lambda: ops.gemm_nt(a, b, None))
    tb = timeit(lambda: a @ b.t())
    print(f"{'':8s} own NT {tn_own:7.1f}us {flop / tn_own / 1e9:4.2f}PF   hipBLASLt NT {tb:7.1f}us {flop / tb / 1e9:4.2f}PF"
          f"   hipBLASLt TN {timeit(lambda: dy.t() @ x):7.1f}us", flush=True)
    del a, b, dy, x, out
    torch.cuda.empty_cache()
