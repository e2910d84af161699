"""Own NT GEMM (csrc/gemm.hip) vs hipBLASLt as K grows at M = 20480, N = 3072:
separates the per-tile fixed cost (prologue + epilogue) from the K loop."""
import torch

from distributed_lion_pytorch_amd.ops import hip


def bench(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1000


def main():
    hip.require()
    ops = hip.ops()
    M, N = 20480, 3072
    for K in (256, 512, 768, 1536, 3072):
        a = torch.randn(M, K, device="cuda").bfloat16()
        b = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
        own = bench(lambda: ops.gemm_nt(a, b, None))
        lt = bench(lambda: a @ b.t())
        fl = 2.0 * M * N * K
        print(f"K={K:5d}  own {own:7.1f} us ({fl / own / 1e6:6.0f} TF/s)  hipBLASLt {lt:7.1f} us ({fl / lt / 1e6:6.0f} TF/s)")


if __name__ == "__main__":
    main()
