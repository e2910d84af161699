"""Short driver for PMC passes on the own NT GEMM (rocprofv3 --pmc) next to
hipBLASLt on the same shape (qkv dgrad: 20480 x 768 x 2304), 5 launches each.

  rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT \
      SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -- python3 tools/pmc_gemm.py"""
import sys

import torch

sys.path.insert(0, ".")
from distributed_lion_pytorch_amd.ops import hip  # noqa: E402

ops = hip.ops()
T = 20480
a = torch.rand(T, 2304, device="cuda", dtype=torch.bfloat16) - 0.5
b = torch.rand(768, 2304, device="cuda", dtype=torch.bfloat16) - 0.5
for _ in range(5):
    ops.gemm_nt(a, b, None)
for _ in range(5):
    a @ b.t()
torch.cuda.synchronize()
