"""Cost of the own NT GEMM's fused MLP epilogues at the GPT-2 shapes (M = 20480,
N = 3072, K = 768), random operands, interleaved rounds in one process:
plain (EPI 0), + bias (1), GELU with z aux (2), GELU with gelu' aux (6), the
backward's multiply-by-gelu' drain with bias-gradient partials (8), against
hipBLASLt's plain GEMM.  Prints median us and TF/s.

  python tools/bench_gemm_epi.py [M [N [K]]]
"""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from distributed_lion_pytorch_amd.ops import hip  # noqa: E402


def timed(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 20480
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 3072
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 768
    ops = hip.ops()
    dt = torch.bfloat16
    a = torch.rand(M, K, device="cuda", dtype=dt) * 2 - 1
    b = (torch.rand(N, K, device="cuda", dtype=dt) * 2 - 1) * 0.05
    bias = torch.rand(N, device="cuda", dtype=dt)
    d = torch.rand(M, N, device="cuda", dtype=dt)
    fl = 2.0 * M * N * K
    variants = {
        "hipblaslt a@b.T": lambda: a @ b.t(),
        "own EPI0 plain": lambda: ops.gemm_nt(a, b, None),
        "own EPI1 +bias": lambda: ops.gemm_nt(a, b, bias),
        "own EPI2 gelu,z": lambda: ops.gemm_nt_gelu(a, b, bias, False),
        "own EPI6 gelu,gelu'": lambda: ops.gemm_nt_gelu_d(a, b, bias, False),
        "own EPI8 *gelu',colsum": lambda: ops.gemm_nt_dmul(a, b, d),
    }
    for f in variants.values():
        f()
    torch.cuda.synchronize()
    res = {k: [] for k in variants}
    for _ in range(7):
        for k, f in variants.items():
            res[k].append(timed(f))
    print(f"M={M} N={N} K={K}", flush=True)
    for k, v in res.items():
        us = statistics.median(v)
        print(f"    {k:26s} {us:9.1f} us  {fl / us / 1e6:7.1f} TF/s  (min {min(v):.1f})", flush=True)


if __name__ == "__main__":
    main()
