"""Cycle accounting of the dQ kernel (build with -D DLION_DQ_STAMP=1): runs the
GPT-2-shape attention forward + backward and prints where a dQ wave's loop
time goes (s_memtime deltas, summed over the loop; the stamps themselves wait
for LDS / scalar traffic, so absolute numbers are perturbed).

  DLION_LIB=variants/_dlion_C_dqstamp.so python tools/attn_dq_stamps.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_lion_pytorch_amd.ops import fused, hip  # noqa: E402


def main():
    ops = hip.ops()
    B, T, H, D = 20, 1024, 12, 64
    torch.manual_seed(0)
    qkv = torch.randn(B, T, 3, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    dout = torch.randn(B, T, H, D, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):  # warm-up
        fused._FlashAttnPacked.apply(qkv, 0.1, 1).backward(dout)
    torch.cuda.synchronize()
    ops.attn_dq_stamps(True)
    fused._FlashAttnPacked.apply(qkv, 0.1, 1).backward(dout)
    torch.cuda.synchronize()
    st = ops.attn_dq_stamps(False)
    names = ["wait + barrier (step top)", "S/dP MFMA -> exp results", "dS VALU + dQ MFMA issue"]
    tot = sum(st[:3])
    print(f"waves {st[5]}, steps computed {st[3]}, steps idle {st[4]}")
    for i, n in enumerate(names):
        print(f"  {n:28s} {st[i] / max(1, st[5]):12.0f} cycles per wave  {100.0 * st[i] / max(1, tot):5.1f} %")
    print(f"  of which the DMA wait (vm_wait before the barrier): {st[6] / max(1, st[5]):.0f} cycles per wave "
          f"({100.0 * st[6] / max(1, st[0]):.1f} % of the top wait)")
    print(f"  per computed step: barrier {st[0] / max(1, st[3] + st[4]):.0f} (per step incl. idle), "
          f"S/dP->exp {st[1] / max(1, st[3]):.0f}, dS+dQ {st[2] / max(1, st[3]):.0f} cycles")


if __name__ == "__main__":
    main()
