"""Own TN (csrc/gemm_tn.hip) vs own NT (csrc/gemm.hip) GEMM at equal work:
C[M,N] = sum over K of one 256x256 tile per CU-sized grid, so per-CU
efficiency can be compared directly."""
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
for M, N, K, splits in [(768, 3072, 20480, 1), (768, 3072, 20480, 7), (4096, 4096, 4096, 1), (4096, 4096, 8192, 1)]:
    flop = 2.0 * M * N * K
    p = torch.randn(K, M, device="cuda", dtype=torch.bfloat16)
    q = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    tn = timeit(lambda: ops.gemm_tn([p], [q], splits))
    line = f"M={M} N={N} K={K} s={splits}: TN {tn:8.1f}us {flop / tn / 1e9:5.2f}PF"
    if splits == 1:
        nt = timeit(lambda: ops.gemm_nt(a, b, None))
        line += f"   NT {nt:8.1f}us {flop / nt / 1e9:5.2f}PF   hipBLASLt-NT {timeit(lambda: a @ b.t()):8.1f}us"
        line += f"   hipBLASLt-TN {timeit(lambda: p.t() @ q):8.1f}us"
    print(line, flush=True)

# accumulate (read-add-write of the fp32 split accumulator) vs plain store, c_fc wgrad shape
T, R, C, s = 20480, 768, 3072, 7
x = torch.randn(T, R, device="cuda", dtype=torch.bfloat16)
y = torch.randn(T, C, device="cuda", dtype=torch.bfloat16)
out = torch.zeros(s, R, C, device="cuda", dtype=torch.float32)
st = timeit(lambda: ops.gemm_tn_([x], [y], out, False))
ac = timeit(lambda: ops.gemm_tn_([x], [y], out, True))
flush = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")  # evict L2 / MALL between calls


def cold(acc):
    flush.zero_()
    ops.gemm_tn_([x], [y], out, acc)


base = timeit(lambda: flush.zero_())
print(f"c_fc s=7: store {st:.1f}us  accumulate {ac:.1f}us  cold store {timeit(lambda: cold(False)) - base:.1f}us  "
      f"cold accumulate {timeit(lambda: cold(True)) - base:.1f}us", flush=True)
