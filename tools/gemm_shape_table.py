"""Per-shape GEMM table of the GPT-2 bench step (one 20480-token micro-batch,
the fusion window's 8 micro-batches for the weight gradients): every GEMM role,
each candidate the step can pick (own NT kernel with its fused epilogue,
hipBLASLt tuned, ATen) timed interleaved, us and PF/s.  The weight gradients
run the own TN kernel over the window's K = 163840 tokens with the split count
the step uses (ops/linear.tn_split_factor), partial reduction excluded.

  python tools/gemm_shape_table.py
"""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from distributed_lion_pytorch_amd.ops import hip  # noqa: E402
from distributed_lion_pytorch_amd.ops import linear  # noqa: E402


def timed(fn, reps=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def rand(*shape, scale=1.0):
    return ((torch.rand(*shape, device="cuda", dtype=torch.bfloat16) * 2 - 1) * scale).contiguous()


def nt_roles(M=20480, C=768, V=50304):
    ops = hip.ops()
    F = torch.nn.functional
    rows = []

    def lt(a, b, bias):
        out = torch.empty(a.shape[0], b.shape[0], dtype=a.dtype, device=a.device)
        return lambda: ops.lt_gemm_nt(a, b, bias, 0 if bias is None else 1, out)

    for role, N, K, bias, epi in (("qkv fwd (+bias)", 3 * C, C, True, None),
                                  ("attn proj fwd (+bias)", C, C, True, None),
                                  ("MLP up fwd: bias+GELU+gelu'", 4 * C, C, True, "gelu_d"),
                                  ("MLP down fwd (+bias)", C, 4 * C, True, None),
                                  ("LM head fwd", V, C, False, None),
                                  ("qkv input grad", C, 3 * C, False, None),
                                  ("attn proj input grad", C, C, False, None),
                                  ("MLP down input grad * gelu'", 4 * C, C, False, "dmul"),
                                  ("MLP up input grad", C, 4 * C, False, None),
                                  ("LM head input grad", C, V, False, None)):
        a, b = rand(M, K), rand(N, K, scale=0.05)
        bv = rand(N) if bias else None
        cands = {"aten": lambda a=a, b=b, bv=bv: F.linear(a, b, bv), "hipblaslt": lt(a, b, bv)}
        if epi == "gelu_d":
            cands = {"own NT EPI6": lambda a=a, b=b, bv=bv: ops.gemm_nt_gelu_d(a, b, bv, False),
                     "hipblaslt (no epilogue)": lt(a, b, bv)}
        elif epi == "dmul":
            d = rand(M, N)
            cands = {"own NT EPI8": lambda a=a, b=b, d=d: ops.gemm_nt_dmul(a, b, d),
                     "hipblaslt (no epilogue)": lt(a, b, None)}
        else:
            cands["own NT"] = lambda a=a, b=b, bv=bv: ops.gemm_nt(a, b, bv)
        rows.append((role, M, N, K, cands))
    return rows


def tn_roles(M=20480, n_mb=8, C=768, V=50304):
    ops = hip.ops()
    rows = []
    for role, R, Cc in (("c_attn weight grad", 3 * C, C), ("attn c_proj weight grad", C, C),
                        ("MLP up weight grad", 4 * C, C), ("MLP down weight grad", C, 4 * C),
                        ("LM head weight grad", V, C)):
        P = [rand(M, R) for _ in range(n_mb)]
        Q = [rand(M, Cc) for _ in range(n_mb)]
        s = linear.tn_split_factor(M * n_mb, R, Cc, max_split=min(32, M // 128))
        rows.append((f"{role} (window, {s} splits)", M * n_mb, R, Cc, {"own TN": lambda P=P, Q=Q, s=s: ops.gemm_tn(P, Q, s)}))
    return rows


def main():
    hip.require()
    print("role | M (tokens) | N | K | candidate: us, PF/s (median of 5 interleaved rounds x 10 calls)", flush=True)
    for group in (nt_roles, tn_roles):
        for role, M, N, K, cands in group():
            for f in cands.values():
                f()
            torch.cuda.synchronize()
            res = {k: [] for k in cands}
            for _ in range(5):
                for k, f in cands.items():
                    res[k].append(timed(f))
            fl = 2.0 * M * N * K
            parts = [f"{k}: {statistics.median(v):8.1f} us {fl / statistics.median(v) / 1e9:5.2f} PF/s"
                     for k, v in res.items()]
            print(f"{role:44s} | {M:6d} | {N:5d} | {K:5d} | " + " | ".join(parts), flush=True)
            del cands
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
