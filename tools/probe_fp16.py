"""Locate fp16 mismatches between the HIP local-Lion kernel and ATen-HIP."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributed_lion_pytorch_amd.ops import reference as ref
from distributed_lion_pytorch_amd.optim.executors import HParams, HipExecutor
from distributed_lion_pytorch_amd.optim.plan import FlatPlan

dev = "cuda"
g0 = torch.Generator().manual_seed(0)
n = 300_001
dt = torch.float16
p = torch.randn(n, generator=g0).to(dt).to(dev)
g = torch.randn(n, generator=g0).to(dt).to(dev)
m = (torch.randn(n, generator=g0) * 0.5).to(dt).to(dev)
p2, m2 = p.clone(), m.clone()
plan = FlatPlan([(p, 0)], world=1, device=torch.device(dev))
HipExecutor(plan).local(plan.meta([g], [m]), plan.buckets[0], HParams(1e-3, 0.1, 0.9, 0.99))
m1 = m2.clone().mul_(0.99)
ref.update_fn(p2, g, m2, 1e-3, 0.1, 0.9, 0.99)
bad = (m != m2).nonzero().flatten()
print("m mismatches", bad.numel(), "p mismatches", (p != p2).sum().item())
for i in bad[:5].tolist():
    mo = (m2[i].float() - 0.01 * g[i].float()) / 0.99
    print(i, "g", g[i].item(), "m1(aten)", m1[i].item(), "hip", m[i].item(), "aten", m2[i].item(),
          "fp32 exact", (m1[i].float() + g[i].float() * 0.01).item())
