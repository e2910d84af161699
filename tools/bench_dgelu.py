"""GPT-2 MLP down-projection backward at the bench shape (20480 tokens, C=768,
4C=3072): hipBLASLt dgrad + bias_gelu_bwd vs the own GEMM with the DGELU epilogue."""
import torch

from distributed_lion_pytorch_amd.ops import hip


def bench(fn, n=20):
    for _ in range(3):
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
    M, C, F4 = 20480, 768, 3072
    dy = torch.randn(M, C, device=dev).to(torch.bfloat16)
    w = (torch.randn(F4, C, device=dev) * 0.02).to(torch.bfloat16)  # Conv1D [in=4C, out=C]
    b = (torch.randn(F4, device=dev) * 0.02).to(torch.bfloat16)
    z = torch.randn(M, F4, device=dev).to(torch.bfloat16)
    res = {
        "hipBLASLt dgrad only": bench(lambda: dy @ w.t()),
        "hipBLASLt dgrad + bias_gelu_bwd": bench(lambda: ops.bias_gelu_bwd(dy @ w.t(), z, b, False, 1024)),
        "own NT GEMM plain": bench(lambda: ops.gemm_nt(dy, w, None)),
        "own NT GEMM + DGELU epilogue": bench(lambda: ops.gemm_nt_dgelu(dy, w, b, z, False)),
    }
    x = torch.randn(M, C, device=dev).to(torch.bfloat16)
    wt = (torch.randn(F4, C, device=dev) * 0.02).to(torch.bfloat16)  # [out, in] (cached W^T)
    res["fwd: hipBLASLt linear + bias_gelu_fwd"] = bench(lambda: ops.bias_gelu_fwd(torch.nn.functional.linear(x, wt), b, False))
    res["fwd: own NT GEMM + GELU epilogue (aux z)"] = bench(lambda: ops.gemm_nt_gelu(x, wt, b, False))
    for k, v in res.items():
        print(f"{k:36s} {v:8.1f} us")


if __name__ == "__main__":
    main()
