"""Microbenchmark: gfx950 flash attention vs PyTorch SDPA at the GPT-2 bench shape
(B=20, T=1024, H=12, D=64, causal, dropout 0.1).  Interleaved rounds in one
process (cdna_hip_programming.md §5.4 rule 24); prints median ms and TFLOP/s."""
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_lion_pytorch_amd.ops import fused  # noqa: E402


def timeit(fn, reps=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    argv = [x for x in sys.argv[1:] if x != "--ours-only"]
    B, T, H, D = [int(x) for x in (argv[0:4] if len(argv) > 3 else (20, 1024, 12, 64))]
    p = float(argv[4]) if len(argv) > 4 else 0.1
    dev = "cuda"
    qkv = torch.randn(B, T, 3, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    dout = torch.randn(B, T, H * D, device=dev, dtype=torch.bfloat16)
    flops_f = 4 * B * H * T * T * D / 2
    res = {"ours_fwd": [], "ours_fb": [], "sdpa_fwd": [], "sdpa_fb": []}

    def ours_fwd():
        with torch.no_grad():
            fused._FlashAttnPacked.apply(qkv, p, 1)

    def ours_fb():
        out = fused._FlashAttnPacked.apply(qkv, p, 1)
        out.backward(dout.view(B, T, H, D))

    def sdpa(bwd):
        q, k, v = qkv.permute(2, 0, 3, 1, 4).unbind(0)
        y = F.scaled_dot_product_attention(q, k, v, dropout_p=p, is_causal=True)
        y = y.transpose(1, 2).reshape(B, T, H * D)
        if bwd:
            y.backward(dout)

    def sdpa_fwd():
        with torch.no_grad():
            sdpa(False)

    only_ours = "--ours-only" in sys.argv  # PMC passes: our kernels only
    for _ in range(5):
        res["ours_fwd"].append(timeit(ours_fwd))
        res["ours_fb"].append(timeit(ours_fb))
        if not only_ours:
            res["sdpa_fwd"].append(timeit(sdpa_fwd))
            res["sdpa_fb"].append(timeit(lambda: sdpa(True)))
    for k, v in res.items():
        if not v:
            continue
        ms = statistics.median(v)
        fl = flops_f if k.endswith("fwd") else 3.5 * flops_f
        print(f"{k:10s} {ms:8.3f} ms  {fl / ms / 1e9:8.1f} TFLOP/s")


if __name__ == "__main__":
    main()
