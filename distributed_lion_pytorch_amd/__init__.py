"""distributed_lion_pytorch_amd -- MI355X-native Distributed Lion training engine.

Capabilities of kyleliang919/distributed-lion-pytorch (Lion optimizer with
majority-vote sign aggregation, AsyncTrainer family, run_clm / sft / dpo
entrypoints), re-designed for gfx950: fused HIP kernels for the optimizer hot
path, 1-bit vote planes over RCCL/xGMI, native GPT-2 / Llama models.
"""
from .optim.lion import Lion  # noqa: F401

__version__ = "0.1.0"

__all__ = ["Lion", "__version__"]
