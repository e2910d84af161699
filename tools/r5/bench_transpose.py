"""LDS-tiled transpose kernel (csrc/elementwise_kernels.hip transpose_pad_kernel)
throughput at the Llama-3-8B operand shapes of the transposed-copy weight
gradients and the per-step W^T copies.  usage: python tools/r5/bench_transpose.py"""
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
        assert torch.equal(ops.transpose_pad(x, R, True), ops.transpose_pad(x, R, False))
        best = {}
        for _ in range(3):  # interleaved rounds: tr = b128 stores + transposed reads, old = per-element LDS path
            for tr in (True, False):
                for _ in range(3):
                    ops.transpose_pad(x, R, tr)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(20):
                    ops.transpose_pad(x, R, tr)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / 20 * 1e3
                best[tr] = min(best.get(tr, 1e30), us)
        print(json.dumps({"R": R, "C": C, "tr_us": round(best[True], 1), "old_us": round(best[False], 1),
                          "tr_TB_s": round(4.0 * R * C / best[True] / 1e6, 2),
                          "old_TB_s": round(4.0 * R * C / best[False] / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
