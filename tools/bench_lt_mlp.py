"""GPT-2 MLP at the bench shape (20480 tokens, C=768, 4C=3072): hipBLASLt
epilogue fusion (GELU_AUX_BIAS forward, DGELU_BGRAD input gradient) vs GEMM +
separate bias+GELU kernels."""
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
    x = torch.randn(M, C, device=dev).to(torch.bfloat16)
    wfc_t = (torch.randn(F4, C, device=dev) * 0.02).to(torch.bfloat16)  # [out, in]
    bfc = (torch.randn(F4, device=dev) * 0.02).to(torch.bfloat16)
    wproj = (torch.randn(F4, C, device=dev) * 0.02).to(torch.bfloat16)  # Conv1D [in=4C, out=C]
    dy = torch.randn(M, C, device=dev).to(torch.bfloat16)
    h = torch.empty(M, F4, device=dev, dtype=torch.bfloat16)
    aux = torch.empty_like(h)
    dz = torch.empty_like(h)
    bg = torch.empty(F4, device=dev, dtype=torch.bfloat16)

    res = {}
    res["fwd unfused: linear + bias_gelu_fwd"] = bench(lambda: ops.bias_gelu_fwd(torch.nn.functional.linear(x, wfc_t), bfc, False))
    res["fwd linear only"] = bench(lambda: torch.nn.functional.linear(x, wfc_t))
    res["fwd lt GELU_AUX_BIAS"] = bench(lambda: ops.lt_gemm_nt(x, wfc_t, bfc, aux, 2, h))
    res["fwd lt plain"] = bench(lambda: ops.lt_gemm_nt(x, wfc_t, None, None, 0, h))
    z = torch.nn.functional.linear(x, wfc_t)
    res["bwd unfused: dgrad + bias_gelu_bwd"] = bench(
        lambda: ops.bias_gelu_bwd(dy @ wproj.t(), z, bfc, False, 1024))
    res["bwd dgrad only"] = bench(lambda: dy @ wproj.t())
    res["bwd lt DGELU_BGRAD"] = bench(lambda: ops.lt_gemm_nt(dy, wproj, bg, aux, 4, dz))
    res["bwd lt DGELU"] = bench(lambda: ops.lt_gemm_nt(dy, wproj, None, aux, 3, dz))
    for k, v in res.items():
        print(f"{k:40s} {v:8.1f} us")


if __name__ == "__main__":
    main()
