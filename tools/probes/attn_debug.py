"""Localise a forward-attention mismatch: T=32 (one tile), B=H=1, D=64, no dropout.
Prints where the kernel output differs from the fp32 reference."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_lion_pytorch_amd.ops import fused, hip  # noqa: E402

ops = hip.ops()
torch.manual_seed(0)
T, D = int(sys.argv[1]) if len(sys.argv) > 1 else 64, 64
q = torch.randn(1, T, 1, D, device="cuda").bfloat16()
k = torch.randn(1, T, 1, D, device="cuda").bfloat16()
# V = one-hot rows: O[q, d] = sum_key P[q, key] * V[key, d] -> reveals the key/d mapping
v = torch.zeros(1, T, 1, D, device="cuda")
for key in range(T):
    v[0, key, 0, key % D] = 1.0 + key // D
v = v.bfloat16()
out, lse = ops.attn_fwd(q, k, v, 0.0, 0)
ref = fused.reference_attention(q.float(), k.float(), v.float(), 0.0, 0).view(1, T, 1, D)
err = (out.float() - ref).abs()
print("max err", err.max().item())
bad = (err > 0.02).nonzero()
print("bad count", bad.shape[0])
print(bad[:20].tolist())
qq = 5
print("row q=5 out", [round(x, 3) for x in out[0, qq, 0, :16].float().tolist()])
print("row q=5 ref", [round(x, 3) for x in ref[0, qq, 0, :16].tolist()])
