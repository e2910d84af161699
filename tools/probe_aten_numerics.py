"""Probe how ATen-HIP rounds the ops the reference optimizer uses (fma vs
mul+add in `add(alpha=)`, alpha rounding for reduced dtypes, torch.mode tie
rule on GPU) so that the gfx950 kernels can replicate it bit-for-bit."""
import torch

dev = "cuda"
torch.manual_seed(0)
n = 1 << 20
a = torch.randn(n, device=dev)
b = torch.randn(n, device=dev)
s = 0.1
ref = a.clone().add_(b, alpha=s)
fma = (a.double() + b.double() * torch.tensor(s, dtype=torch.float32).double()).float()
two = a + (b * s)
print("fp32 add(alpha): mismatches vs fma", (ref != fma).sum().item(), "vs mul+add", (ref != two).sum().item())
for dt in (torch.bfloat16, torch.float16):
    a16, b16 = a.to(dt), b.to(dt)
    ref = a16.clone().add_(b16, alpha=s)
    fma = (a16.double() + b16.double() * torch.tensor(s, dtype=torch.float32).double()).float().to(dt)
    two = (a16.float() + (b16.float() * s)).to(dt)
    alpha_r = (a16.float() + b16.float() * torch.tensor(s).to(dt).float()).to(dt)
    print(dt, "add(alpha): vs fma", (ref != fma).sum().item(), "vs mul+add", (ref != two).sum().item(),
          "vs alpha-rounded", (ref != alpha_r).sum().item())
    sign = torch.randint(0, 2, (n,), device=dev) * 2 - 1
    r2 = a16.clone().add_(sign, alpha=-s)
    print(dt, "add(int64 other, alpha): vs float alpha", (r2 != (a16.float() - s * sign.float()).to(dt)).sum().item(),
          "vs rounded alpha", (r2 != (a16.float() + torch.tensor(-s).to(dt).float() * sign.float()).to(dt)).sum().item())
x = torch.stack([torch.tensor([True, False, True, False] * 4, device=dev), torch.tensor([False, True, True, False] * 4, device=dev)])
print("torch.mode tie on GPU:", torch.mode(x, 0).values.tolist()[:4], "(expect [False, False, True, False])")

for dt in (torch.bfloat16, torch.float16):
    m16 = (torch.randn(n, device=dev) * 0.5).to(dt)
    r = m16.clone().mul_(0.99)
    f = (m16.float() * 0.99).to(dt)
    h = (m16.float() * torch.tensor(0.99).to(dt).float()).to(dt)
    print(dt, "mul_(scalar): vs fp32-scalar", (r != f).sum().item(), "vs rounded scalar", (r != h).sum().item())
