"""Split-K weight-gradient GEMMs at the GPT-2 bench shapes (20480 tokens):
times torch.baddbmm into the fp32 accumulator [s, R, C] for every split
factor s, in both operand orientations (R = input dim for HF Conv1D weights,
R = output dim for nn.Linear), and reports PF/s.  ops/linear.split_k_factor
picks s from this table."""
import argparse

import torch


def timeit(fn, iters=20):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=20480)
    ap.add_argument("--splits", default="1,2,4,5,8,10,16,20")
    ap.add_argument("--own", action="store_true", help="also time the own TN kernel (csrc/gemm_tn.hip)")
    ap.add_argument("--own_splits", default="1,2,3,4,5,6,7,8,9,10,12,14,16")
    ap.add_argument("--window", type=int, default=0, help="micro-batches of a one-GEMM window (own kernel)")
    a = ap.parse_args()
    T = a.tokens
    shapes = [("c_attn", 768, 2304), ("attn.c_proj", 768, 768), ("c_fc", 768, 3072), ("mlp.c_proj", 3072, 768),
              ("lm_head", 50304, 768)]
    for name, r, c in shapes:
        x = torch.randn(T, r, device="cuda", dtype=torch.bfloat16)
        y = torch.randn(T, c, device="cuda", dtype=torch.bfloat16)
        flop = 2.0 * T * r * c
        res = []
        for s in [int(v) for v in a.splits.split(",")]:
            if T % s:
                continue
            acc = torch.zeros(s, r, c, device="cuda", dtype=torch.float32)
            a3, b3 = x.view(s, T // s, r).transpose(1, 2), y.view(s, T // s, c)
            if acc.numel() * 4 > (2 << 30):
                continue
            us = timeit(lambda: torch.baddbmm(acc, a3, b3, out_dtype=torch.float32, out=acc))
            res.append(f"s={s}:{us:7.1f}us {flop / us / 1e9:4.2f}PF")
        print(f"{name:12s} [{r}x{c}] " + "  ".join(res), flush=True)
        if a.own:
            from distributed_lion_pytorch_amd.ops import hip

            own = []
            for s in [int(v) for v in a.own_splits.split(",")]:
                if s > T // 128:
                    continue
                us = timeit(lambda: hip.ops().gemm_tn([x], [y], s))
                own.append(f"s={s}:{us:7.1f}us {flop / us / 1e9:4.2f}PF")
            print(f"{'  own TN':12s} " + "  ".join(own), flush=True)
            if a.window > 1 and r * c < 10_000_000:  # one GEMM over the window's micro-batches (segments)
                xs = [torch.randn(T, r, device="cuda", dtype=torch.bfloat16) for _ in range(a.window)]
                ys = [torch.randn(T, c, device="cuda", dtype=torch.bfloat16) for _ in range(a.window)]
                win = []
                for s in [int(v) for v in a.own_splits.split(",")]:
                    us = timeit(lambda: hip.ops().gemm_tn(xs, ys, s), iters=5)
                    win.append(f"s={s}:{us / a.window:7.1f}us/mb {a.window * flop / us / 1e9:4.2f}PF")
                print(f"{'  window':12s} " + "  ".join(win), flush=True)
                xc, yc = torch.cat(xs), torch.cat(ys)  # hipBLASLt (ATen heuristic) on the concatenated window
                us = timeit(lambda: torch.mm(xc.t(), yc), iters=5)
                print(f"{'  blas win':12s} {us / a.window:7.1f}us/mb {a.window * flop / us / 1e9:4.2f}PF", flush=True)
                del xc, yc
                del xs, ys


if __name__ == "__main__":
    main()
