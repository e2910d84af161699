"""Attention forward diagnostics at the Llama shape: separate q/k/v with
Hkv = 32 / 8, and with K/V broadcast (batch/head stride 0: every block reads
the same 1 MB, L2-resident) to separate memory latency from the loop's own cost."""
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from distributed_lion_pytorch_amd.ops import hip  # noqa: E402


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    B, T, H, D = 4, 2048, 32, 128
    fl = 4 * B * H * T * T * D / 2
    ops = hip.ops()
    q = torch.randn(B, T, H, D, device="cuda", dtype=torch.bfloat16)
    cases = {}
    for hkv in (32, 8):
        k = torch.randn(B, T, hkv, D, device="cuda", dtype=torch.bfloat16)
        v = torch.randn_like(k)
        cases[f"hkv{hkv}"] = (k, v)
    k1 = torch.randn(1, T, 1, D, device="cuda", dtype=torch.bfloat16)
    cases["shared_kv"] = (k1.expand(B, T, 8, D), torch.randn_like(k1).expand(B, T, 8, D))
    res = {c: [] for c in cases}
    for _ in range(5):
        for c, (k, v) in cases.items():
            res[c].append(timeit(lambda: ops.attn_fwd(q, k, v, 0.0, 1)))
    for c, v in res.items():
        ms = statistics.median(v)
        print(f"fwd {c:10s} {ms:8.3f} ms {fl / ms / 1e9:8.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
