"""First-round start stagger of the own NT GEMM (set_gemm_stagger, A/B): the
MLP epilogue GEMMs at the GPT-2 shape, stagger units (x 64 cycles per CU group)
interleaved in one process; median us.  python tools/r5/bench_gemm_stagger.py"""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from distributed_lion_pytorch_amd.ops import hip  # noqa: E402


def timed(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    M, N, K = 20480, 3072, 768
    ops = hip.ops()
    dt = torch.bfloat16
    a = torch.rand(M, K, device="cuda", dtype=dt) * 2 - 1
    b = (torch.rand(N, K, device="cuda", dtype=dt) * 2 - 1) * 0.05
    bias = torch.rand(N, device="cuda", dtype=dt)
    d = torch.rand(M, N, device="cuda", dtype=dt)
    kern = {"EPI0": lambda: ops.gemm_nt(a, b, None), "EPI6": lambda: ops.gemm_nt_gelu_d(a, b, bias, False),
            "EPI8": lambda: ops.gemm_nt_dmul(a, b, d)}
    units = [0, 16, 32, 64, 96, 128]
    res = {(k, u): [] for k in kern for u in units}
    for _ in range(5):
        for u in units:
            ops.set_gemm_stagger(u)
            for k, f in kern.items():
                res[(k, u)].append(timed(f))
    ops.set_gemm_stagger(0)
    for k in kern:
        print(k, " ".join(f"u{u}: {statistics.median(res[(k, u)]):6.1f}" for u in units))


if __name__ == "__main__":
    main()
