"""On-box GEMM anchor: what the best library GEMM reaches on THIS MI355X, so the
own kernels' numbers can be read as % of a measured roof instead of the spec
sheet (VERDICT r5 "Next round" item 6).

Rows (random uniform [-1, 1) bf16 operands, guide §5.4 rule 25):
  * square anchors  -- hipBLASLt NT with the exhaustively searched algorithm
    (csrc/lt_gemm.cpp), ATen (torch.mm), and the own NT kernel at 8192^3 and
    16384 x 16384 x 4096;
  * the GPT-2 window weight gradients (K = 163840 tokens = 8 micro-batches x
    20480) in three forms: own TN kernel on the row-major operands (what the
    step runs), hipBLASLt TN on the same operands, and hipBLASLt NT on
    token-contiguous copies [features, tokens] (the form that producer-written
    copies would enable; copy cost NOT included);
  * the same at one micro-batch (K = 20480).

  python tools/gemm_anchor.py [--quick | --square | --tn]
"""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from distributed_lion_pytorch_amd.ops import hip  # noqa: E402
from distributed_lion_pytorch_amd.ops import linear  # noqa: E402


def timed(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def rand(*shape):
    return (torch.rand(*shape, device="cuda", dtype=torch.bfloat16) * 2 - 1).contiguous()


def run_row(role, M, N, K, cands, rounds=5, reps=5):
    for f in cands.values():
        f()
    torch.cuda.synchronize()
    res = {k: [] for k in cands}
    for _ in range(rounds):
        for k, f in cands.items():
            res[k].append(timed(f, reps))
    fl = 2.0 * M * N * K
    parts = []
    best = {}
    for k, v in res.items():
        med = statistics.median(v)
        best[k] = fl / med / 1e9
        parts.append(f"{k}: {med:9.1f} us {best[k]:5.2f} PF/s (min {fl / min(v) / 1e9:5.2f})")
    print(f"{role:34s} | M {M:6d} N {N:6d} K {K:6d} | " + " | ".join(parts), flush=True)
    return best


def square_rows():
    ops = hip.ops()
    out = {}
    for M, N, K in ((8192, 8192, 8192), (16384, 16384, 4096), (20480, 3072, 768), (20480, 768, 3072)):
        a, b = rand(M, K), rand(N, K)
        c = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        cands = {
            "hipblaslt NT (searched)": lambda a=a, b=b, c=c: ops.lt_gemm_nt(a, b, None, 0, c),
            "aten mm": lambda a=a, b=b: torch.mm(a, b.t()),
            "own NT": lambda a=a, b=b: ops.gemm_nt(a, b, None),
        }
        out[(M, N, K)] = run_row("square/plain NT", M, N, K, cands)
        del a, b, c
        torch.cuda.empty_cache()
    return out


def wgrad_rows(T):
    ops = hip.ops()
    C, rows = 768, []
    for role, R, Cc in (("c_attn wgrad", 3 * C, C), ("attn c_proj wgrad", C, C), ("MLP up wgrad", 4 * C, C),
                        ("MLP down wgrad", C, 4 * C)):
        dy, x = rand(T, R), rand(T, Cc)  # row-major [tokens, features]: what the step holds
        dyt, xt = dy.t().contiguous(), x.t().contiguous()  # token-contiguous copies
        out = torch.empty(R, Cc, dtype=torch.bfloat16, device="cuda")
        s = linear.tn_split_factor(T, R, Cc, max_split=min(32, T // 128))
        cands = {
            f"own TN ({s} splits, partials)": lambda dy=dy, x=x, s=s: ops.gemm_tn([dy], [x], s),
            "own TN unsplit -> bf16": lambda dy=dy, x=x, out=out: ops.gemm_tn_([dy], [x], out, False),
            "hipblaslt TN": lambda dy=dy, x=x, out=out: ops.lt_gemm_tn(dy, x, out, False),
            "hipblaslt NT on copies": lambda dyt=dyt, xt=xt, out=out: ops.lt_gemm_nt_acc(dyt, xt, out, False),
        }
        rows.append(run_row(f"{role} (T={T})", T, R, Cc, cands, rounds=3, reps=3))
        del dy, x, dyt, xt, out
        torch.cuda.empty_cache()
    return rows


def tn_rows():
    """The weight-gradient (TN) layout at the anchor size and at the GPT-2 LM
    head's window shape: own TN kernel (split partials, as the step runs it)
    vs hipBLASLt's TN form with the searched algorithm."""
    ops = hip.ops()
    for role, T, R, Cc in (("TN 8192^3", 8192, 8192, 8192), ("LM head wgrad (window)", 163840, 50304, 768),
                           ("LM head wgrad (1 micro-batch)", 20480, 50304, 768)):
        dy, x = rand(T, R), rand(T, Cc)
        out = torch.empty(R, Cc, dtype=torch.bfloat16, device="cuda")
        s = linear.tn_split_factor(T, R, Cc, max_split=min(32, T // 128))
        # the window passes its micro-batches as segments (one operand buffer per
        # micro-batch, as the step does); one segment must stay below 2^31 elements
        seg = 20480 if T > 20480 else T
        dys, xs = list(dy.split(seg)), list(x.split(seg))
        cands = {f"own TN ({s} splits, partials)": lambda dys=dys, xs=xs, s=s: ops.gemm_tn(dys, xs, s)}
        if T == seg:  # hipBLASLt takes one operand pair
            cands["hipblaslt TN"] = lambda dy=dy, x=x, out=out: ops.lt_gemm_tn(dy, x, out, False)
        run_row(role, T, R, Cc, cands, rounds=3, reps=2)
        del dy, x, out, dys, xs
        torch.cuda.empty_cache()


def main():
    hip.require()
    quick = "--quick" in sys.argv
    print(f"# device {torch.cuda.get_device_name()}  torch {torch.__version__}", flush=True)
    print("# us = median over interleaved rounds; PF/s = 2MNK / time", flush=True)
    sq = square_rows()
    anchor = max(sq[(8192, 8192, 8192)].values())
    print(f"# ANCHOR (best at 8192^3) = {anchor:.3f} PF/s", flush=True)
    if "--square" in sys.argv:
        return
    if "--tn" in sys.argv:
        tn_rows()
        return
    for T in ((20480,) if quick else (163840, 20480)):
        wgrad_rows(T)


if __name__ == "__main__":
    main()
