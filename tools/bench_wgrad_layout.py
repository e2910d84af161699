"""Weight-gradient layout A/B at the GPT-2 bench shapes (20480 tokens):
current split-K bmm on token-major X (TN: both operands reduce over their row
axis) vs the same split-K on a transposed activation copy X^T [in, tokens]
(NN: the layout the fast dgrad GEMMs run in).  Split reduction included."""
import statistics

import torch


def t(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    M, dt = 20480, torch.bfloat16
    for name, K, N in (("qkv", 768, 2304), ("proj", 768, 768), ("fc", 768, 3072), ("fc_proj", 3072, 768)):
        x = torch.randn(M, K, device="cuda", dtype=dt)
        xt = x.t().contiguous()
        dy = torch.randn(M, N, device="cuda", dtype=dt)
        fl = 2.0 * M * K * N
        res = {}
        for _ in range(3):
            for S in (4, 8, 16):
                kc = M // S
                xs, dys = x.view(S, kc, K), dy.view(S, kc, N)
                xts = xt.view(K, S, kc).permute(1, 0, 2)  # [S, K, kc], batch stride kc
                res.setdefault(f"TN splitK{S}", []).append(
                    t(lambda: torch.bmm(xs.transpose(1, 2), dys, out_dtype=torch.float32).sum(0)))
                res.setdefault(f"NN(X^T) splitK{S}", []).append(
                    t(lambda: torch.bmm(xts, dys, out_dtype=torch.float32).sum(0)))
            res.setdefault("transpose copy X->X^T", []).append(t(lambda: x.t().contiguous()))
        print(f"{name} M={M} K={K} N={N}", flush=True)
        for k, v in res.items():
            us = statistics.median(v)
            print(f"   {k:24s} {us:8.1f} us  {fl / us / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
