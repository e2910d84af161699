"""Fused LM-head softmax-xent kernel at the GPT-2 bench shape (20460 x 50304 bf16)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_lion_pytorch_amd.ops import hip  # noqa: E402

N, V = (int(a) for a in sys.argv[1:3]) if len(sys.argv) > 2 else (20460, 50304)
Vp = (V + 63) // 64 * 64
ops = hip.ops()
x0 = torch.randn(N, Vp, device="cuda", dtype=torch.bfloat16)
lab = torch.randint(0, V, (N,), device="cuda")
x = x0.clone()
loss = ops.softmax_xent_(x, lab, V)
ref = torch.nn.functional.cross_entropy(x0[:, :V].float(), lab, reduction="none")
print("max loss err", (loss - ref).abs().max().item())
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(3):
    x.copy_(x0)
    torch.cuda.synchronize()
    s.record()
    ops.softmax_xent_(x, lab, V)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e)
print(f"xent {ms*1e3:8.1f} us  {2 * N * Vp * 2 / ms / 1e9:7.2f} TB/s (read + write of the row)")
