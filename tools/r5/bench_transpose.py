"""LDS-tiled transpose kernel (csrc/elementwise_kernels.hip transpose_pad_kernel)
throughput at the Llama-3-8B operand shapes of the transposed-copy weight
gradients and the per-step W^T copies.  The round-5 A/B of a variant with
16-byte LDS stores and hardware-transposed LDS reads (tr_path, removed:
slower, profiles/r5/transpose_tr_ab_c29.jsonl) ran through this script.
usage: python tools/r5/bench_transpose.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_lion_pytorch_amd.ops import hip  # noqa: E402


def main():
    hip.require()
    ops = hip.ops()
    dev = torch.device("cuda", 0)
    for R, C in ((8192, 28672), (8192, 14336), (8192, 4096), (4096, 4096), (768, 3072)):
        x = torch.randn(R, C, device=dev).to(torch.bfloat16)
        for _ in range(3):
            ops.transpose_pad(x, R)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(20):
            ops.transpose_pad(x, R)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(json.dumps({"R": R, "C": C, "us": round(us, 1), "TB_s": round(4.0 * R * C / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
