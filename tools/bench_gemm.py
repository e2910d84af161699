"""hipBLASLt GEMM throughput for the GPT-2 training shapes, per operand layout.

For each linear layer (x[M,K] -> y[M,N]) the three training GEMMs are timed:
fwd y = x W, dgrad dx = dy W^T, wgrad dW = x^T dy, with W stored either
[K, N] (HF Conv1D) or [N, K] (nn.Linear)."""
import statistics
import sys

import torch


def t(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 20480
    shapes = {"qkv": (768, 2304), "proj": (768, 768), "fc": (768, 3072), "fc_proj": (3072, 768), "lm_head": (768, 50304)}
    dev, dt = "cuda", torch.bfloat16
    for name, (K, N) in shapes.items():
        x = torch.randn(M, K, device=dev, dtype=dt)
        dy = torch.randn(M, N, device=dev, dtype=dt)
        w_kn = torch.randn(K, N, device=dev, dtype=dt)
        w_nk = torch.randn(N, K, device=dev, dtype=dt)
        b = torch.randn(N, device=dev, dtype=dt)
        fl = 2 * M * K * N
        res = {}
        for _ in range(3):
            for key, fn in {
                "fwd W[K,N] addmm": lambda: torch.addmm(b, x, w_kn),
                "fwd W[N,K] linear": lambda: torch.nn.functional.linear(x, w_nk, b),
                "dgrad W[K,N]": lambda: dy @ w_kn.t(),
                "dgrad W[N,K]": lambda: dy @ w_nk,
                "wgrad ->[K,N]": lambda: x.t() @ dy,
                "wgrad ->[N,K]": lambda: dy.t() @ x,
            }.items():
                res.setdefault(key, []).append(t(fn))
        for S in (4, 8, 16):
            xs, dys = x.view(S, M // S, K), dy.view(S, M // S, N)
            for _ in range(3):
                res.setdefault(f"wgrad splitK{S} f32", []).append(
                    t(lambda: torch.bmm(xs.transpose(1, 2), dys, out_dtype=torch.float32).sum(0).to(dt)))
                res.setdefault(f"wgrad splitK{S} bf16", []).append(
                    t(lambda: torch.bmm(xs.transpose(1, 2), dys).float().sum(0).to(dt)))
        print(f"{name} M={M} K={K} N={N}")
        for key, v in res.items():
            ms = statistics.median(v)
            print(f"   {key:20s} {ms*1e3:8.1f} us  {fl / ms / 1e9:7.1f} TF/s")


if __name__ == "__main__":
    main()
