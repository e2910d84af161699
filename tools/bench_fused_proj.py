"""Llama-3-8B projection GEMMs (8192 tokens, C=4096): q/k/v (4096/1024/1024)
and gate/up (14336 each) as separate GEMMs vs one GEMM on the concatenated
weight -- forward, input gradient (+ the adds of the separate dx) and split-K
weight gradient.  Decides whether fusing the projections pays."""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from distributed_lion_pytorch_amd.ops.linear import wgrad  # noqa: E402


def timed(fn, reps=10):
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
    M, C, dt = 8192, 4096, torch.bfloat16
    x = torch.randn(M, C, device="cuda", dtype=dt)
    for name, Ns in (("qkv", (4096, 1024, 1024)), ("gate_up", (14336, 14336))):
        ws = [torch.randn(n, C, device="cuda", dtype=dt) * 0.02 for n in Ns]
        wc = torch.cat(ws, 0)
        dys = [torch.randn(M, n, device="cuda", dtype=dt) for n in Ns]
        dyc = torch.cat(dys, 1)

        def sep_dgrad():
            dx = dys[0] @ ws[0]
            for d, w in zip(dys[1:], ws[1:]):
                dx = dx + d @ w
            return dx

        variants = {
            "fwd separate": lambda: [x @ w.t() for w in ws],
            "fwd fused": lambda: x @ wc.t(),
            "dgrad separate (+adds)": sep_dgrad,
            "dgrad fused": lambda: dyc @ wc,
            "wgrad separate": lambda: [wgrad(d, x) for d in dys],
            "wgrad fused": lambda: wgrad(dyc, x),
        }
        res = {k: [] for k in variants}
        for _ in range(3):
            for k, f in variants.items():
                res[k].append(timed(f))
        print(name, flush=True)
        for k, v in res.items():
            print(f"   {k:24s} {statistics.median(v):9.1f} us", flush=True)


if __name__ == "__main__":
    main()
