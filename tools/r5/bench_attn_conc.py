"""Attention backward, sequential (dQ then dK/dV) vs concurrent (delta
pre-pass, dK/dV on a side stream beside dQ): fwd+bwd time at the GPT-2 and
Llama-3-8B shapes, interleaved rounds.  python tools/r5/bench_attn_conc.py"""
import torch

from distributed_lion_pytorch_amd.ops import fused, hip


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


ops = hip.ops()
for name, B, T, H, Hkv, D, p in [("gpt2", 20, 1024, 12, 12, 64, 0.1), ("llama3", 4, 2048, 32, 8, 128, 0.0)]:
    q = torch.randn(B, T, H, D, device="cuda", dtype=torch.bfloat16).requires_grad_()
    k = torch.randn(B, T, Hkv, D, device="cuda", dtype=torch.bfloat16).requires_grad_()
    v = torch.randn(B, T, Hkv, D, device="cuda", dtype=torch.bfloat16).requires_grad_()
    dout = torch.randn(B, T, H * D, device="cuda", dtype=torch.bfloat16)
    out = fused._FlashAttn.apply(q, k, v, p, 5).view(B, T, H * D)

    def bwd():
        torch.autograd.grad(out, (q, k, v), dout, retain_graph=True)

    res = {0: [], 1: []}
    for _ in range(3):
        for mode in (0, 1):
            ops.set_attn_bwd_concurrent(mode)
            res[mode].append(timeit(bwd))
    ops.set_attn_bwd_concurrent(0)
    print(f"{name:7s} bwd sequential " + " ".join(f"{t:7.1f}" for t in res[0]) + " us | concurrent "
          + " ".join(f"{t:7.1f}" for t in res[1]) + " us", flush=True)
