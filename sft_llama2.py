#!/usr/bin/env python
"""Llama-2 supervised fine-tuning with Distributed Lion -- drop-in for
/root/reference/sft_llama2.py (same ScriptArguments + HF TrainingArguments,
``--lion`` / ``--async_grad``), MI355X-native underneath:

* one full bf16 replica per GPU by default (288 GB HBM holds it), native
  Llama with the gfx950 attention / LM-head kernels; ``--load_in_4bit``
  reproduces the reference's 4-bit NF4 base model (sft_llama2.py:141-149,
  bitsandbytes) with the native 4-bit layers (models/quant.py, QLoRA);
* LoRA (r=8, alpha=16, dropout 0.05, q_proj/v_proj, sft_llama2.py:44-51) via
  the native adapter implementation (peft absent) -- ``--use_lora false``
  trains all weights;
* the optimizer is built over the trainable (adapter) parameters AFTER
  injection (the reference builds it over the frozen base: no-op, D12);
* packed "Question: ...\\n\\nAnswer: ..." samples, the reference's data
  semantics (take / skip + seeded shuffle buffer, or a seeded random split;
  an infinite packed training stream read lazily and sharded per rank);
  ``--dataset_name`` is read like the reference's ``load_dataset(name,
  data_dir=subset, split=split, streaming=...)`` (sft_llama2.py:99-107):
  a local dataset directory (e.g. a stack-exchange-paired mirror with
  data/finetune parquet shards), a json/jsonl/parquet/csv file, or a hub name
  present in the HF cache; a name that resolves to nothing is an error, and
  ``--synthetic_data`` trains on a synthetic corpus of the same format;
* every Lion knob of run_clm (``--lion_beta1/2``, ``--lion_vote``,
  ``--lion_tie_break``, ``--lion_wire``, ``--lion_bucket_mb``,
  ``--lion_stochastic_max_norm``, ``--lion_dropout_schedule`` and
  ``--lion_elastic_timeout`` for real worker dropout);
* saves the adapter (final_checkpoint/) and the merged model
  (final_merged_checkpoint/, safetensors) like sft_llama2.py:183-199.
"""
from __future__ import annotations

import logging
import os
import sys
from dataclasses import dataclass, field
from typing import Optional

import torch
import transformers
from transformers import HfArgumentParser, TrainingArguments

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_lion_pytorch_amd.models.lora import (LoraConfig, load_adapter, merge_and_unload,  # noqa: E402
                                                      print_trainable_parameters, save_adapter)
from distributed_lion_pytorch_amd.models.registry import build_model, load_config  # noqa: E402
from distributed_lion_pytorch_amd.trainer.async_trainer import (LionArguments, apply_lion_args, legacy_training_arguments,  # noqa: E402
                                                                build_lion, warn_unsynced)
from distributed_lion_pytorch_amd.trainer.sft import AsyncSFTTrainer, SFTTrainer  # noqa: E402
from distributed_lion_pytorch_amd.utils.data import (ConstantLengthDataset, PackedStream, RowSlice,  # noqa: E402
                                                     Rows, ShuffledRows, chars_token_ratio, load_named_rows,
                                                     load_tokenizer, prepare_sample_text, random_split,
                                                     synthetic_qa)
from distributed_lion_pytorch_amd.utils.metrics import JsonlMetricsCallback  # noqa: E402

logger = logging.getLogger(__name__)


@dataclass
class ScriptArguments:
    model_name: Optional[str] = field(default="meta-llama/Llama-2-7b-hf", metadata={"help": "size name or local dir"})
    dataset_name: Optional[str] = field(default="lvwerra/stack-exchange-paired", metadata={
        "help": "local dataset directory or data file, or a hub name in the HF cache"})
    subset: Optional[str] = field(default="data/finetune", metadata={"help": "data_dir inside --dataset_name"})
    split: Optional[str] = field(default="train")
    size_valid_set: Optional[int] = field(default=4000)
    streaming: Optional[bool] = field(default=True)
    shuffle_buffer: Optional[int] = field(default=5000)
    seq_length: Optional[int] = field(default=1024)
    num_workers: Optional[int] = field(default=4)
    packing: Optional[bool] = field(default=True)
    lora_alpha: Optional[float] = field(default=16)
    lora_dropout: Optional[float] = field(default=0.05)
    lora_r: Optional[int] = field(default=8)
    use_lora: Optional[bool] = field(default=True, metadata={"help": "False: full fine-tune"})
    lion: Optional[bool] = field(default=False, metadata={"help": "whether to use lion optimizer"})
    async_grad: Optional[bool] = field(default=False, metadata={"help": "do not sync gradients between workers"})
    synthetic_data: Optional[bool] = field(default=False, metadata={
        "help": "train on a synthetic corpus of the stack-exchange format instead of --dataset_name"})
    synthetic_samples: Optional[int] = field(default=20000)
    model_overrides: Optional[str] = field(default=None, metadata={"help": "config overrides, e.g. num_hidden_layers=4"})
    torch_dtype: Optional[str] = field(default="bfloat16")
    load_in_4bit: Optional[bool] = field(default=False, metadata={
        "help": "frozen base weights in 4-bit (the reference's BitsAndBytesConfig, sft_llama2.py:141-145)"})
    bnb_4bit_quant_type: Optional[str] = field(default="nf4", metadata={"help": "nf4 | fp4"})
    final_save: Optional[bool] = field(default=True, metadata={
        "help": "save the trained model / adapter at the end (false: throughput runs of 7B models)"})


def build_base(script_args, seed):
    """The compute-dtype base model: loaded from ``model_name`` when it is a
    local checkpoint, else randomly initialised from the seed -- so calling it
    again with the same seed rebuilds exactly the same weights (the 4-bit
    merge below relies on that)."""
    transformers.set_seed(seed)
    config = load_config(script_args.model_name, overrides=script_args.model_overrides)
    return build_model(config, model_name_or_path=script_args.model_name, torch_dtype=script_args.torch_dtype)


def load_samples(script_args, seed):
    """Row source (re-iterable dict rows): ``--dataset_name`` through
    ``load_named_rows`` (data_dir = ``--subset``, ``--split``, ``--streaming``,
    ``--num_workers``; a json-lines file is read lazily), or the synthetic
    corpus of the reference's format with ``--synthetic_data``.  A name that
    resolves to nothing raises (utils/data.DatasetUnavailable)."""
    if script_args.synthetic_data:
        logger.info("--synthetic_data: training on %d synthetic stack-exchange-format rows",
                    script_args.synthetic_samples)
        return Rows(synthetic_qa(script_args.synthetic_samples, seed=seed))
    rows = load_named_rows(script_args.dataset_name, data_dir=script_args.subset, split=script_args.split,
                           streaming=script_args.streaming, num_workers=script_args.num_workers)
    logger.info("SFT rows from %s (data_dir=%s, split=%s, streaming=%s)", script_args.dataset_name,
                script_args.subset, script_args.split, script_args.streaming)
    return rows


def _count_rows(rows, cap: int) -> int:
    """Rows in the source, counting at most ``cap`` (a stream is not read to its end)."""
    import itertools

    if isinstance(rows, Rows) and isinstance(rows.source, list):
        return min(len(rows.source), cap)
    try:
        return min(len(rows), cap)  # a map-style datasets.Dataset
    except TypeError:  # a stream or a lazily read file
        return sum(1 for _ in itertools.islice(iter(rows), cap))


def create_datasets(tokenizer, script_args, seed):
    """The reference's splits (sft_llama2.py:99-138):
    * ``--streaming`` (default): the first ``size_valid_set`` rows are the
      validation set (``take``), the rest (``skip``) go through a
      ``shuffle_buffer``-row shuffle buffer, seeded by the training seed;
    * otherwise a seeded random ``train_test_split(test_size=0.005)``.
    Training data is an infinite packed stream (ConstantLengthDataset
    ``infinite=True``, buffer sized by the measured chars/token) read lazily
    and sharded per rank; the (bounded) validation set is packed up front."""
    rows = load_samples(script_args, seed)
    if script_args.streaming:
        # a corpus smaller than size_valid_set would leave nothing to train on: keep 95 % for training
        n_rows = _count_rows(rows, 20 * script_args.size_valid_set)
        n_valid = min(script_args.size_valid_set, max(1, n_rows // 20))
        valid_rows = list(RowSlice(rows, 0, n_valid))
        train_rows = ShuffledRows(RowSlice(rows, n_valid), script_args.shuffle_buffer, seed)
    else:
        if hasattr(rows, "train_test_split"):  # a datasets.Dataset: split in Arrow, seeded (sft_llama2.py:114)
            split = rows.train_test_split(test_size=0.005, seed=seed)
            train_rows, valid_rows = split["train"], split["test"]
        else:
            train_rows, valid_rows = random_split(rows, 0.005, seed)
        logger.info(f"Size of the train set: {len(train_rows)}. Size of the validation set: {len(valid_rows)}")
    ratio = chars_token_ratio(train_rows, tokenizer)
    logger.info(f"The character to token ratio of the dataset is: {ratio:.2f}")
    train = PackedStream(tokenizer, train_rows, prepare_sample_text, seq_length=script_args.seq_length,
                         infinite=True, chars_per_token=ratio)
    valid = ConstantLengthDataset(tokenizer, valid_rows, prepare_sample_text, seq_length=script_args.seq_length)
    return train, valid


def main(argv=None):
    legacy = legacy_training_arguments()  # --group_by_length on transformers >= 5
    parser = HfArgumentParser((ScriptArguments, LionArguments, TrainingArguments) + legacy)
    parsed = parser.parse_args_into_dataclasses(args=argv)
    script_args, lion_args, training_args = parsed[:3]
    logging.basicConfig(level=logging.INFO, handlers=[logging.StreamHandler(sys.stdout)])
    group_by_length = parsed[3].group_by_length if legacy else getattr(training_args, "group_by_length", False)
    if group_by_length and script_args.packing:
        raise ValueError("Cannot use both packing and group by length")
    # packing + gradient checkpointing is allowed here (the reference forbids
    # checkpointing because of a peft/trl issue, sft_llama2.py:58-59)
    training_args.lion = script_args.lion
    training_args.async_grad = script_args.async_grad
    apply_lion_args(training_args, lion_args)  # --lion_* knobs, incl. --lion_elastic_timeout (worker dropout)
    transformers.set_seed(training_args.seed)

    tokenizer = load_tokenizer(script_args.model_name)
    model = build_base(script_args, training_args.seed)
    if script_args.load_in_4bit:
        from distributed_lion_pytorch_amd.models.quant import QuantConfig, quantize_model

        quantize_model(model, QuantConfig(bnb_4bit_quant_type=script_args.bnb_4bit_quant_type,
                                          bnb_4bit_compute_dtype=getattr(torch, script_args.torch_dtype)))
    if training_args.gradient_checkpointing:
        model.gradient_checkpointing_enable()
    peft_config = None
    if script_args.use_lora:
        peft_config = LoraConfig(r=script_args.lora_r, lora_alpha=int(script_args.lora_alpha),
                                 lora_dropout=script_args.lora_dropout, target_modules=["q_proj", "v_proj"],
                                 bias="none", task_type="CAUSAL_LM")
        from distributed_lion_pytorch_amd.models.lora import inject_lora

        inject_lora(model, peft_config)  # before the optimizer is built (D12)
    print_trainable_parameters(model)

    train_dataset, eval_dataset = create_datasets(tokenizer, script_args, training_args.seed)
    params = [p for p in model.parameters() if p.requires_grad]
    if script_args.lion:
        optimizer = build_lion(model, training_args)
    else:
        optimizer = torch.optim.AdamW(params, lr=training_args.learning_rate, weight_decay=0.1)
    sched = (transformers.get_cosine_schedule_with_warmup(optimizer, training_args.warmup_steps, training_args.max_steps)
             if training_args.max_steps > 0 else None)

    trainer_class = AsyncSFTTrainer if script_args.async_grad else SFTTrainer
    trainer = trainer_class(model=model, train_dataset=train_dataset, eval_dataset=eval_dataset, peft_config=None,
                            packing=script_args.packing, max_seq_length=script_args.seq_length, tokenizer=tokenizer,
                            args=training_args, optimizers=(optimizer, sched),
                            callbacks=[JsonlMetricsCallback(training_args.output_dir, script_args.seq_length)])
    warn_unsynced(training_args)
    trainer.train()
    if not script_args.final_save:
        return trainer
    trainer.save_model(training_args.output_dir)

    if trainer.is_world_process_zero():
        out = os.path.join(training_args.output_dir, "final_checkpoint")
        if script_args.use_lora:
            save_adapter(trainer.model, out)
            if script_args.load_in_4bit:
                # like the reference (sft_llama2.py:195-196: AutoPeftModelForCausalLM reloads the base in
                # the compute dtype), the adapters are merged into the ORIGINAL weights, not into
                # dequant(quant(W)): the merged model carries no 4-bit rounding error
                merged = merge_and_unload(load_adapter(build_base(script_args, training_args.seed), out))
            else:
                merged = merge_and_unload(trainer.accelerator.unwrap_model(trainer.model))
            merged.save_pretrained(os.path.join(training_args.output_dir, "final_merged_checkpoint"),
                                   safe_serialization=True)
        else:
            trainer.accelerator.unwrap_model(trainer.model).save_pretrained(out)
    return trainer


if __name__ == "__main__":
    main()
