"""Split count of the window-level weight-gradient GEMMs (own TN kernel over
the fusion window's 8 micro-batch segments of 20480 tokens), measured: for
each GPT-2 weight shape, the TN kernel into fp32 partials [s, R, C] plus the
reduction into the bf16 gradient (sum_partials_multi_, what the window's exit
runs), for split counts around ops/linear.tn_split_factor's pick.  Interleaved
rounds, median us.

  python tools/bench_tn_splits.py
"""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from distributed_lion_pytorch_amd.ops import hip, linear  # noqa: E402


def timed(fn, reps=3):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    hip.require()
    ops = hip.ops()
    T, n_mb, C = 20480, 8, 768
    for role, R, Cc in (("c_attn", 3 * C, C), ("attn c_proj", C, C), ("MLP up", 4 * C, C), ("MLP down", C, 4 * C),
                        ("LM head", 50304, C)):
        P = [(torch.rand(T, R, device="cuda", dtype=torch.bfloat16) * 2 - 1) for _ in range(n_mb)]
        Q = [(torch.rand(T, Cc, device="cuda", dtype=torch.bfloat16) * 2 - 1) for _ in range(n_mb)]
        g = torch.empty(R * Cc, device="cuda", dtype=torch.bfloat16)
        pick = linear.tn_split_factor(T * n_mb, R, Cc, max_split=min(32, T * n_mb // 128))
        cands = sorted({max(1, pick + d) for d in (-2, -1, 0, 1, 2)} | {max(1, 2 * pick), max(1, pick // 2)})
        if role == "LM head":
            cands = [c for c in cands if c <= 8]
        fns = {}
        for s in cands:
            def f(s=s):
                part = ops.gemm_tn(P, Q, s)
                ops.sum_partials_multi_([part.view(s, -1)], g, False)
            fns[s] = f
            f()
        torch.cuda.synchronize()
        res = {s: [] for s in fns}
        for _ in range(3):
            for s, f in fns.items():
                res[s].append(timed(f, 2 if role == "LM head" else 3))
        fl = 2.0 * T * n_mb * R * Cc
        line = " | ".join(f"s={s}{'*' if s == pick else ''}: {statistics.median(v):8.1f} us "
                          f"{fl / statistics.median(v) / 1e9:4.2f} PF/s" for s, v in res.items())
        print(f"{role:12s} R {R:5d} C {Cc:4d} | {line}", flush=True)
        del P, Q, g, fns
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
