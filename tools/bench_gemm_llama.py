"""Llama-2-7B projection GEMMs at 4096 tokens (the SFT preset's micro-batch):
ATen's choice (what the training path calls today) vs hipBLASLt with the
tuned-algorithm cache (csrc/lt_gemm.cpp, NT form: weights K-contiguous) vs the
own gfx950 NT GEMM (csrc/gemm.hip).  Input-gradient GEMMs dX = dY.W are timed
in their NN form (ATen) and as NT against a cached W^T (frozen LoRA bases).
usage: python tools/bench_gemm_llama.py  -> one JSON line per shape"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_lion_pytorch_amd.ops import hip  # noqa: E402


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
    return s.elapsed_time(e) / iters * 1e3


def main():
    hip.require()
    ops = hip.ops()
    dev = torch.device("cuda", 0)
    M = int(os.environ.get("TOKENS", "4096"))
    bf = torch.bfloat16
    shapes = {  # name: (N, K) of the NT product x[M, K] . W[N, K]^T
        "qkv_fwd": (12288, 4096), "o_fwd": (4096, 4096), "gate_up_fwd": (22016, 4096), "down_fwd": (4096, 11008),
        # input gradients as NT against W^T: dX[M, K_in] = dY[M, N_out] . (W^T)^T with W^T [K_in, N_out]
        "qkv_dgrad": (4096, 12288), "o_dgrad": (4096, 4096), "gate_up_dgrad": (4096, 22016), "down_dgrad": (11008, 4096),
    }
    if os.environ.get("MODEL") == "llama3":  # Llama-3-8B (GQA q/k/v 6144, MLP 14336); TOKENS=8192 for its preset
        shapes = {"qkv_fwd": (6144, 4096), "o_fwd": (4096, 4096), "gate_up_fwd": (28672, 4096),
                  "down_fwd": (4096, 14336), "qkv_dgrad": (4096, 6144), "o_dgrad": (4096, 4096),
                  "gate_up_dgrad": (4096, 28672), "down_dgrad": (14336, 4096)}
    for name, (N, K) in shapes.items():
        a = torch.randn(M, K, device=dev).to(bf)
        w = (torch.randn(N, K, device=dev) * 0.02).to(bf)  # NT operand
        res = {"shape": name, "M": M, "N": N, "K": K}
        flops = 2.0 * M * N * K
        res["aten_nt_us"] = timeit(lambda: F.linear(a, w))
        if name.endswith("dgrad"):
            wt = w.t().contiguous()  # the stored nn.Linear weight [K_out... ] for the NN form
            res["aten_nn_us"] = timeit(lambda: a @ wt)
            nn_out = torch.empty(M, N, device=dev, dtype=bf)
            if ops.lt_gemm_nn(a, wt, nn_out):  # hipBLASLt NN with the searched algorithm
                res["lt_tuned_nn_us"] = timeit(lambda: ops.lt_gemm_nn(a, wt, nn_out))
            res["transpose_us"] = timeit(lambda: w.t().contiguous())  # W^T rebuild for a trainable weight
        out = torch.empty(M, N, device=dev, dtype=bf)
        ok = ops.lt_gemm_nt(a, w, None, 0, out)
        if ok:
            res["lt_tuned_nt_us"] = timeit(lambda: ops.lt_gemm_nt(a, w, None, 0, out))
        if K % 128 == 0 and N % 8 == 0:
            res["own_nt_us"] = timeit(lambda: ops.gemm_nt_out(a, w, None, out))
        for k in list(res):
            if k.endswith("_us"):
                res[k] = round(res[k], 1)
                res[k.replace("_us", "_PFs")] = round(flops / res[k] / 1e9, 2)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
