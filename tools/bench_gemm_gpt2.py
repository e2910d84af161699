"""Own NT GEMM vs hipBLASLt on every K = 768 GEMM of the GPT-2 bench step
(M = 20480 tokens): which shapes the own kernel should take."""
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
    M, K = 20480, 768
    for name, N, bias in (("qkv fwd (+bias)", 2304, True), ("attn proj fwd / dgrad", 768, False),
                          ("fc fwd", 3072, False), ("LM head fwd", 50304, False)):
        a = torch.randn(M, K, device="cuda").bfloat16()
        b = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
        bb = torch.randn(N, device="cuda").bfloat16() if bias else None
        own = bench(lambda: ops.gemm_nt(a, b, bb), n=5 if N > 10000 else 20)
        lt = bench(lambda: torch.nn.functional.linear(a, b, bb), n=5 if N > 10000 else 20)
        print(f"{name:24s} N={N:6d}  own {own:8.1f} us   hipBLASLt {lt:8.1f} us   own/lt {own / lt:5.2f}")
    # the K = 2304 / 3072 GEMMs (N = 768): MLP down-projection forward, c_fc and c_attn input gradients
    for name, K in (("mlp proj fwd / fc dgrad", 3072), ("c_attn dgrad", 2304)):
        a = torch.randn(M, K, device="cuda").bfloat16()
        b = (torch.randn(768, K, device="cuda") / K ** 0.5).bfloat16()
        own = bench(lambda: ops.gemm_nt(a, b, None))
        lt = bench(lambda: torch.nn.functional.linear(a, b))
        print(f"{name:24s} K={K:6d}  own {own:8.1f} us   hipBLASLt {lt:8.1f} us   own/lt {own / lt:5.2f}")


if __name__ == "__main__":
    main()
