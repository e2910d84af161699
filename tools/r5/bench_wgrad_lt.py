"""Llama-3-8B weight-gradient shapes (8192 tokens): the own TN kernel (unsplit
bf16 epilogue, and split-K into fp32 partials + reduction at the split count
ops/linear.tn_split_factor picks) vs hipBLASLt's TN form with the searched
algorithm (csrc/lt_gemm.cpp lt_gemm_tn) vs ATen's heuristic.  Interleaved
rounds, median per candidate.  usage: python tools/r5/bench_wgrad_lt.py"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_lion_pytorch_amd.ops import hip, linear  # noqa: E402


def timeit(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    hip.require()
    ops = hip.ops()
    dev = torch.device("cuda", 0)
    M = int(os.environ.get("TOKENS", "8192"))
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    for name, (R, C) in shapes.items():  # dW [R, C] = dY[M, R]^T X[M, C]
        dy = (torch.randn(M, R, device=dev) * 0.1).to(torch.bfloat16)
        x = torch.randn(M, C, device=dev).to(torch.bfloat16)
        out = torch.empty(R, C, device=dev, dtype=torch.bfloat16)
        s = linear.tn_split_factor(M, R, C)
        cands = {
            "own_unsplit": lambda: ops.gemm_tn_([dy], [x], out, True),
            "aten": lambda: out.addmm_(dy.t(), x),
        }
        if s > 1:
            cands[f"own_split{s}"] = lambda: ops.sum_partials_acc_(ops.gemm_tn([dy], [x], s).view(s, -1), out)
        if ops.lt_gemm_tn(dy, x, out, True):
            cands["lt_tn"] = lambda: ops.lt_gemm_tn(dy, x, out, True)
        cands["lt_nt_transposed"] = lambda: linear._wgrad_via_transposes(dy, x, out, True)
        # one-copy forms (c31, profiles/r5/wgrad_onecopy_c31.txt): never faster, not in the pick
        cands["lt_copy_dy_nn"] = lambda: ops.lt_gemm_layout(linear.fast_transpose(dy), x, out, 1, True)
        cands["lt_copy_x_tt"] = lambda: ops.lt_gemm_layout(dy, linear.fast_transpose(x), out, 3, True)
        ref = (dy.float().t() @ x.float())
        chk = torch.empty_like(out)
        assert ops.lt_gemm_tn(dy, x, chk, False)
        err = ((chk.float() - ref).abs().max() / ref.abs().max()).item()
        for fn in cands.values():
            fn()
        times = {k: [] for k in cands}
        for _ in range(5):
            for k, fn in cands.items():
                times[k].append(timeit(fn))
        flops = 2.0 * M * R * C
        res = {"shape": name, "M": M, "R": R, "C": C, "lt_rel_err": round(err, 5)}
        for k, v in times.items():
            us = statistics.median(v)
            res[k + "_us"] = round(us, 1)
            res[k + "_PFs"] = round(flops / us / 1e9, 2)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
