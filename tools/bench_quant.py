"""4-bit expansion bandwidth (csrc/quant.hip dequant4) at Llama-2-7B layer
shapes, and the cost it adds around a QLoRA projection GEMM.
usage: python tools/bench_quant.py  -> one JSON line per shape"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_lion_pytorch_amd.ops.quant import code_tensor, dequantize_4bit, quantize_4bit  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    dev = torch.device("cuda", 0)
    code = code_tensor("nf4", dev)
    x = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)  # 4 x 1024 tokens
    for name, (n, k) in {"qkv_cat": (12288, 4096), "gate_up_cat": (22016, 4096), "down": (4096, 11008),
                         "lm_head_size": (32000, 4096)}.items():
        w = torch.randn(n, k, device=dev, dtype=torch.bfloat16) * 0.02
        q, a = quantize_4bit(w, code)
        out = torch.empty_like(w)
        us = timeit(lambda: dequantize_4bit(q, a, code, w.shape, torch.bfloat16, out=out))
        bytes_moved = q.numel() + a.numel() * 4 + out.numel() * 2
        xin = torch.randn(4096, k, device=dev, dtype=torch.bfloat16)
        gemm_us = timeit(lambda: torch.nn.functional.linear(xin, w), iters=20)
        print(json.dumps({"shape": name, "n": n, "k": k, "dequant_us": round(us, 1),
                          "dequant_TBps": round(bytes_moved / us / 1e6, 2), "gemm_4096tok_us": round(gemm_us, 1),
                          "overhead_vs_gemm": round(us / gemm_us, 3)}), flush=True)
    del x


if __name__ == "__main__":
    main()
