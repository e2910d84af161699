"""LM-head GEMM layout A/B at the GPT-2 bench shape (20480 tokens, C=768,
V padded to 50304), random data, interleaved rounds in one process."""
import statistics

import sys

import torch

sys.path.insert(0, ".")
from distributed_lion_pytorch_amd.ops import hip  # noqa: E402


def timed(fn, reps=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    ops = hip.ops()
    N, C, V = 20480, 768, 50304
    dt = torch.bfloat16
    h = torch.randn(N, C, device="cuda", dtype=dt)
    w = torch.randn(V, C, device="cuda", dtype=dt) * 0.02
    wt = w.t().contiguous()
    lg = torch.randn(N, V, device="cuda", dtype=dt) * 1e-3
    fl = 2.0 * N * C * V
    variants = {
        "fwd h@w.T (NT)": lambda: h @ w.t(),
        "fwd h@wt (NN)": lambda: h @ wt,
        "dgrad lg@w (NN, current)": lambda: lg @ w,
        "dgrad lg@wt.T (NT)": lambda: lg @ wt.t(),
        "wgrad lg.T@h (current)": lambda: lg.t() @ h,
        "wgrad (h.T@lg).T": lambda: (h.t() @ lg),
        "pad cat": lambda: torch.cat([w[:50257], w.new_zeros(47, C)], 0),
        "dgrad own gemm_nt(lg, wt)": lambda: ops.gemm_nt(lg, wt, None),
    }
    for f in variants.values():
        f()
    torch.cuda.synchronize()
    res = {k: [] for k in variants}
    for _ in range(5):
        for k, f in variants.items():
            res[k].append(timed(f))
    for k, v in res.items():
        us = statistics.median(v)
        print(f"{k:28s} {us:9.1f} us  {fl / us / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
