"""Sliding-window flash attention at Mistral-7B shapes (H 32, Hkv 8, D 128):
fwd + bwd time with window 4096 vs plain causal, per sequence length.
usage: python tools/r5/bench_window.py  -> one JSON line per (T, window)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_lion_pytorch_amd.ops import fused, hip  # noqa: E402


def main():
    hip.require()
    dev = torch.device("cuda", 0)
    H, Hkv, D = 32, 8, 128
    for T in (4096, 8192, 16384):
        B = max(1, 16384 // T)
        q = torch.randn(B, T, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
        k = torch.randn(B, T, Hkv, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
        v = torch.randn(B, T, Hkv, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
        dout = torch.randn(B, T, H * D, device=dev, dtype=torch.bfloat16)
        for window in (0, 4096):
            def step():
                out = fused._FlashAttn.apply(q, k, v, 0.0, 1, window if window < T else 0)
                out.view(B, T, H * D).backward(dout)
            for _ in range(2):
                step()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(5):
                step()
            e1.record()
            torch.cuda.synchronize()
            print(json.dumps({"B": B, "T": T, "window": window, "fwd_bwd_ms": round(e0.elapsed_time(e1) / 5, 3)}),
                  flush=True)


if __name__ == "__main__":
    main()
