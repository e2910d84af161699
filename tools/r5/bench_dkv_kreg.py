"""dK/dV at D = 128 without dropout: K tile in registers (2 waves per SIMD)
vs in LDS (1 wave per SIMD), interleaved via DLION_DKV_KREG128, at the
Llama-2-7B SFT shape (H = Hkv = 32, T 1024) and the Llama-3-8B GQA shape
(H 32, Hkv 8, T 2048).  usage: python tools/r5/bench_dkv_kreg.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_lion_pytorch_amd.ops import fused, hip  # noqa: E402


def main():
    hip.require()
    dev = torch.device("cuda", 0)
    for B, T, H, Hkv in ((4, 1024, 32, 32), (4, 2048, 32, 8)):
        D = 128
        q = torch.randn(B, T, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
        k = torch.randn(B, T, Hkv, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
        v = torch.randn(B, T, Hkv, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
        dout = torch.randn(B, T, H * D, device=dev, dtype=torch.bfloat16)

        def step():
            fused._FlashAttn.apply(q, k, v, 0.0, 1).view(B, T, H * D).backward(dout)

        grads = {}
        best = {}
        for _ in range(4):
            for mode in ("1", "0"):
                os.environ["DLION_DKV_KREG128"] = mode
                for t in (q, k, v):
                    t.grad = None
                step()
                grads[mode] = [t.grad.clone() for t in (q, k, v)]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(10):
                    step()
                e1.record()
                torch.cuda.synchronize()
                best[mode] = min(best.get(mode, 1e30), e0.elapsed_time(e1) / 10)
        same = all(torch.equal(a, b) for a, b in zip(grads["1"], grads["0"]))
        print(json.dumps({"B": B, "T": T, "H": H, "Hkv": Hkv, "fwd_bwd_ms_kreg": round(best["1"], 3),
                          "fwd_bwd_ms_lds": round(best["0"], 3), "grads_bit_identical": same}), flush=True)


if __name__ == "__main__":
    main()
