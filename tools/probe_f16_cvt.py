"""How does ATen-HIP round fp32 -> fp16 / bf16 on the device?  (RNE vs RTZ)"""
import numpy as np
import torch

x = torch.randn(1 << 20) * 3
g = x.cuda().to(torch.float16).cpu().view(torch.int16).numpy().view(np.uint16)
rne = x.numpy().astype(np.float16).view(np.uint16)
u = x.numpy().view(np.uint32)
sign = (u >> 16) & 0x8000
ax = u & 0x7FFFFFFF
e = (ax >> 23).astype(np.int64)
rtz = np.where(e >= 113, sign | (((e - 112) << 10) | ((ax & 0x7FFFFF) >> 13)), rne).astype(np.uint16)
print("fp16 device vs RNE mismatches", int((g != rne).sum()), "vs RTZ", int((g != rtz).sum()))
cpu = x.to(torch.float16).view(torch.int16).numpy().view(np.uint16)
print("fp16 cpu vs RNE", int((cpu != rne).sum()))
m = (torch.randn(1 << 20) * 0.5).to(torch.float16).cuda()
r1 = m.clone().mul_(0.99)
r2 = (m.float() * 0.99).to(torch.float16)
print("mul_ vs float-then-cast", int((r1 != r2).sum()))
