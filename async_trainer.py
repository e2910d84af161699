"""Drop-in module name of the reference trainers (``from async_trainer import AsyncTrainer``).

Re-exports the HF-5.x-native implementations (reference: /root/reference/async_trainer.py);
``AsyncSFTTrainer`` / ``AsyncDPOTrainer`` are built on our native SFT/DPO
trainers because trl is not part of this stack.
"""
from distributed_lion_pytorch_amd.trainer.async_trainer import AsyncTrainer, AsyncTrainingArguments  # noqa: F401
from distributed_lion_pytorch_amd.trainer.dpo import AsyncDPOTrainer, DPOTrainer  # noqa: F401
from distributed_lion_pytorch_amd.trainer.sft import AsyncSFTTrainer, SFTTrainer  # noqa: F401

__all__ = ["AsyncTrainer", "AsyncSFTTrainer", "AsyncDPOTrainer", "AsyncTrainingArguments", "SFTTrainer",
           "DPOTrainer"]
