"""Where the own GEMM's per-tile time goes: per-block s_memtime stamps from the
diagnostic build (gemm_nt_stamped) -- prologue, K loop, park, drain -- and the
block start/end timeline (s_memrealtime, 100 MHz) of the whole launch."""
import sys

import torch

from distributed_lion_pytorch_amd.ops import hip


def main():
    hip.require()
    ops = hip.ops()
    M, N = 20480, 3072
    for K in [int(k) for k in (sys.argv[1:] or ["768", "1536"])]:
        a = torch.randn(M, K, device="cuda").bfloat16()
        b = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
        blocks = (M // 256) * (N // 256)
        st = torch.zeros(blocks, 8, dtype=torch.int64, device="cuda")
        for _ in range(3):
            c = ops.gemm_nt_stamped(a, b, st)
        torch.cuda.synchronize()
        assert (c.float() - (a.float() @ b.float().t())).abs().max().item() < 0.5
        s = st.cpu().double()
        seg = {"prologue": s[:, 1] - s[:, 0], "k_loop": s[:, 2] - s[:, 1], "park": s[:, 3] - s[:, 2],
               "drain": s[:, 4] - s[:, 3]}
        tot = s[:, 4] - s[:, 0]
        print(f"K={K}: {blocks} blocks, cycles per block (median): total {tot.median():.0f}")
        for k, v in seg.items():
            print(f"   {k:9s} {v.median():8.0f}  ({100 * v.median() / tot.median():4.1f} %)")
        t0, t1 = s[:, 5], s[:, 6]  # realtime (10 ns ticks)
        span = (t1.max() - t0.min()) / 100.0
        busy = ((t1 - t0) / 100.0).sum() / 256
        starts = ((t0 - t0.min()) / 100.0).sort().values
        print(f"   launch span {span:.1f} us, mean per-CU busy {busy:.1f} us ({100 * busy / span:.0f} %), "
              f"block time median {((t1 - t0) / 100.0).median():.2f} us")
        print(f"   start times (us) at block 0/256/512/768/last: "
              f"{[round(float(starts[i]), 1) for i in (0, 255, 511, 767, blocks - 1)]}")


if __name__ == "__main__":
    main()
