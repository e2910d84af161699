"""LM-head forward + softmax-xent at the GPT-2 bench shape (20480 x 768 ->
50304): one [20480, 50304] GEMM then the xent kernel, vs row chunks whose
bf16 logits (chunk x 50304 x 2 B) fit the 256 MB Infinity Cache so the xent
pass reads them back from MALL instead of HBM."""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from distributed_lion_pytorch_amd.ops import hip  # noqa: E402


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
    ops = hip.ops()
    N, C, V, VP = 20480, 768, 50257, 50304
    h = torch.randn(N, C, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(VP, C, device="cuda", dtype=torch.bfloat16) * 0.02
    lab = torch.randint(0, V, (N,), device="cuda")
    logits = torch.empty(N, VP, device="cuda", dtype=torch.bfloat16)

    def full():
        torch.matmul(h, w.t(), out=logits)
        ops.softmax_xent_(logits, lab, V)

    def chunked(rows):
        def f():
            for r0 in range(0, N, rows):
                lg = logits[r0:r0 + rows]
                torch.matmul(h[r0:r0 + rows], w.t(), out=lg)
                ops.softmax_xent_(lg, lab[r0:r0 + rows], V)
        return f

    side = torch.cuda.Stream()

    def pipelined(nchunk):
        rows = N // nchunk

        def f():
            main = torch.cuda.current_stream()
            for i in range(nchunk):
                r0 = i * rows
                lg = logits[r0:r0 + rows]
                torch.matmul(h[r0:r0 + rows], w.t(), out=lg)
                ev = torch.cuda.Event()
                ev.record(main)
                side.wait_event(ev)
                with torch.cuda.stream(side):
                    ops.softmax_xent_(lg, lab[r0:r0 + rows], V)
            main.wait_stream(side)
        return f

    variants = {"full": full, "gemm only": lambda: torch.matmul(h, w.t(), out=logits),
                "xent only": lambda: ops.softmax_xent_(logits, lab, V)}
    for rows in (4096,):
        variants[f"chunk {rows}"] = chunked(rows)
    for n in (2, 4, 5, 8):
        variants[f"2-stream {n}"] = pipelined(n)
    res = {k: [] for k in variants}
    for _ in range(5):
        for k, f in variants.items():
            res[k].append(timed(f))
    for k, v in res.items():
        print(f"{k:12s} {statistics.median(v):9.1f} us", flush=True)


if __name__ == "__main__":
    main()
