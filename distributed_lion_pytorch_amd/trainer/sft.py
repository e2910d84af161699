"""Supervised fine-tuning trainer (native replacement for trl's SFTTrainer).

The reference's SFT script (/root/reference/sft_llama2.py) relies on
``trl.SFTTrainer`` for LoRA injection (peft_config) and sequence packing
(``packing=True`` + ``ConstantLengthDataset``); trl/peft are not installed
here, so this is the same contract built on HF ``Trainer`` + our LoRA and
packing.  ``AsyncSFTTrainer`` adds the no-gradient-sync training step
(reference async_trainer.py:37-62).
"""
from __future__ import annotations

from typing import Callable, Optional

from transformers import Trainer, default_data_collator

from ..models.lora import LoraConfig, inject_lora
from ..utils.data import ConstantLengthDataset, prepare_sample_text
from .async_trainer import AsyncMixin, RankShardedLoaderMixin


def _is_packed(ds) -> bool:
    if ds is None:
        return True
    try:
        item = ds[0]
    except Exception:
        return True
    return isinstance(item, dict) and "input_ids" in item


class SFTTrainer(RankShardedLoaderMixin, Trainer):
    def __init__(self, model=None, args=None, train_dataset=None, eval_dataset=None, tokenizer=None,
                 processing_class=None, peft_config: Optional[LoraConfig] = None, packing: bool = True,
                 max_seq_length: int = 1024, formatting_func: Optional[Callable] = None, data_collator=None,
                 **kwargs):
        tok = processing_class if processing_class is not None else tokenizer
        if peft_config is not None:
            inject_lora(model, peft_config)
        fmt = formatting_func or prepare_sample_text
        if packing and not _is_packed(train_dataset):
            train_dataset = ConstantLengthDataset(tok, train_dataset, fmt, seq_length=max_seq_length)
        if packing and not _is_packed(eval_dataset):
            eval_dataset = ConstantLengthDataset(tok, eval_dataset, fmt, seq_length=max_seq_length)
        super().__init__(model=model, args=args, train_dataset=train_dataset, eval_dataset=eval_dataset,
                         processing_class=tok, data_collator=data_collator or default_data_collator, **kwargs)


class AsyncSFTTrainer(AsyncMixin, SFTTrainer):
    """SFT with per-worker gradients; replicas synchronised by Lion's vote."""
