"""Weight gradients of the 12 GPT-2 layers: per layer split-K (current) vs one
GEMM batched over the layers (no split-K: 12x the output tiles, full-length
token reduction).  M = 20480 tokens per micro-batch; 'x8' = the 8 micro-batches
of an optimizer step in one reduction."""
import torch

from distributed_lion_pytorch_amd.ops import hip
from distributed_lion_pytorch_amd.ops.linear import split_k_factor


def bench(fn, n=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1000


def main():
    hip.require()
    ops = hip.ops()
    dev = torch.device("cuda")
    L, M = 12, 20480
    shapes = {"qkv": (768, 2304), "attn_proj": (768, 768), "fc": (768, 3072), "mlp_proj": (3072, 768)}
    tot = {}
    for name, (K, N) in shapes.items():
        X = torch.randn(L, M, K, device=dev).to(torch.bfloat16)
        dY = torch.randn(L, M, N, device=dev).to(torch.bfloat16)
        s = split_k_factor(M, K, N)

        def per_layer():
            for l in range(L):
                a3 = X[l].view(s, M // s, K).transpose(1, 2)
                b3 = dY[l].view(s, M // s, N)
                ops.sum_partials(torch.bmm(a3, b3, out_dtype=torch.float32))

        def batched_bf16():
            torch.bmm(X.transpose(1, 2), dY)

        def batched_f32():
            torch.bmm(X.transpose(1, 2), dY, out_dtype=torch.float32)

        fl = 2.0 * L * M * K * N
        r = {"per-layer split-K (S=%d) + sum" % s: bench(per_layer), "batched L=12 bf16 out": bench(batched_bf16),
             "batched L=12 fp32 out": bench(batched_f32)}
        for k, us in r.items():
            print(f"{name:9s} {k:32s} {us:9.1f} us  {fl / us / 1e6:7.1f} TF/s")
            tot[k.split(" (")[0]] = tot.get(k.split(" (")[0], 0) + us
        del X, dY
    X8 = torch.randn(L, 8 * M, 768, device=dev).to(torch.bfloat16)
    dY8 = torch.randn(L, 8 * M, 2304, device=dev).to(torch.bfloat16)
    us = bench(lambda: torch.bmm(X8.transpose(1, 2), dY8, out_dtype=torch.float32), n=3)
    print(f"qkv x8 micro-batches batched fp32: {us:9.1f} us  {2.0 * L * 8 * M * 768 * 2304 / us / 1e6:7.1f} TF/s"
          f"  (per micro-batch {us / 8:.1f} us)")
    for k, v in tot.items():
        print(f"TOTAL per micro-batch {k:28s} {v / 1000:7.3f} ms")


if __name__ == "__main__":
    main()
