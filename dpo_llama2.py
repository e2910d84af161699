#!/usr/bin/env python
"""Llama-2 DPO with Distributed Lion -- a working counterpart of
/root/reference/dpo_llama2.py (which does not parse: ``Option[bool]`` and an
unclosed ``{``; and uses an undefined ``base_model``, D9).

Same ScriptArguments (beta, lr, schedule, LoRA, lengths, steps, ``--lion``,
``--async_grad``) and the same in-code TrainingArguments
(dpo_llama2.py:171-190), MI355X-native underneath:
* policy + frozen reference replicas in bf16 on each GPU by default;
  ``--load_in_4bit`` stores both frozen bases in 4-bit NF4 like the reference
  (dpo_llama2.py:133-152 ``load_in_4bit=True``) with the native 4-bit layers
  (models/quant.py); native Llama kernels;
* DPO sigmoid loss with chosen/rejected concatenated in one policy forward
  (native trainer: trl is not installed);
* LoRA targets use Llama module names (q_proj, k_proj, v_proj -- the modules
  that actually matched in the reference's GPT-J-style list, D11);
* the optimizer sees the adapter parameters and ``--weight_decay`` (0.05 by
  default) is actually forwarded to it (D10, D12);
* every Lion knob of run_clm (``--lion_*``, incl. ``--lion_elastic_timeout``
  for real worker dropout and ``--ddp_backend`` for the process group).
Data: ``--dataset_name`` (default lvwerra/stack-exchange-paired) is read like
the reference's ``get_stack_exchange_paired`` (dpo_llama2.py:84-125): a local
dataset directory (its ``--subset``, default data/rl, for training and
``--eval_subset``, default data/evaluation, capped at 1000 rows like the
reference's ``sanity_check=True`` eval load, :164), a data file, or a hub name
in the HF cache; question/response_j/response_k rows are mapped to
prompt/chosen/rejected, rows already in that form pass through.  A name that
resolves to nothing is an error; ``--synthetic_data`` trains on synthetic
triples of the same format.
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

from distributed_lion_pytorch_amd.models.lora import LoraConfig, print_trainable_parameters  # noqa: E402
from distributed_lion_pytorch_amd.models.registry import build_model, load_config  # noqa: E402
from distributed_lion_pytorch_amd.trainer.async_trainer import (LionArguments, apply_lion_args,  # noqa: E402
                                                                build_lion, warn_unsynced)
from distributed_lion_pytorch_amd.trainer.dpo import AsyncDPOTrainer, DPOTrainer  # noqa: E402
from distributed_lion_pytorch_amd.utils.data import (DatasetUnavailable, _pair_length_ok,  # noqa: E402
                                                     load_named_rows, load_tokenizer, stack_exchange_pairs,
                                                     stack_exchange_pairs_dataset, synthetic_paired)
from distributed_lion_pytorch_amd.utils.metrics import JsonlMetricsCallback  # noqa: E402

logger = logging.getLogger(__name__)


@dataclass
class ScriptArguments:
    beta: Optional[float] = field(default=0.1, metadata={"help": "the beta parameter for DPO loss"})
    model_name_or_path: Optional[str] = field(default="../sft/results/final_checkpoint",
                                              metadata={"help": "SFT model dir, or a size name (random init)"})
    learning_rate: Optional[float] = field(default=5e-4)
    lr_scheduler_type: Optional[str] = field(default="cosine")
    warmup_steps: Optional[int] = field(default=100)
    weight_decay: Optional[float] = field(default=0.05)
    optimizer_type: Optional[str] = field(default="paged_adamw_32bit")
    per_device_train_batch_size: Optional[int] = field(default=4)
    per_device_eval_batch_size: Optional[int] = field(default=1)
    gradient_accumulation_steps: Optional[int] = field(default=4)
    gradient_checkpointing: Optional[bool] = field(default=True)
    checkpointing_policy: Optional[str] = field(default="auto", metadata={
        "help": "auto: keep activations when policy + reference + activations fit in HBM (288 GB on MI355X), "
                "checkpoint otherwise (trainer/memory.py); reference: --gradient_checkpointing as given"})
    lora_alpha: Optional[float] = field(default=16)
    lora_dropout: Optional[float] = field(default=0.05)
    lora_r: Optional[int] = field(default=8)
    use_lora: Optional[bool] = field(default=True)
    max_prompt_length: Optional[int] = field(default=512)
    max_length: Optional[int] = field(default=1024)
    max_steps: Optional[int] = field(default=1000)
    logging_steps: Optional[int] = field(default=10)
    save_steps: Optional[int] = field(default=100)
    eval_steps: Optional[int] = field(default=100)
    output_dir: Optional[str] = field(default="./results")
    log_freq: Optional[int] = field(default=1)
    sanity_check: Optional[bool] = field(default=False, metadata={"help": "only train on 1000 samples"})
    report_to: Optional[str] = field(default="none")
    ignore_bias_buffers: Optional[bool] = field(default=False)
    lion: Optional[bool] = field(default=False, metadata={"help": "whether to use lion optimizer"})
    async_grad: Optional[bool] = field(default=False, metadata={"help": "do not sync gradients between workers"})
    dataset_name: Optional[str] = field(default="lvwerra/stack-exchange-paired", metadata={
        "help": "local dataset directory or data file (question/response_j/response_k or prompt/chosen/rejected "
                "rows), or a hub name in the HF cache"})
    subset: Optional[str] = field(default="data/rl", metadata={"help": "training data_dir inside --dataset_name"})
    eval_subset: Optional[str] = field(default="data/evaluation", metadata={
        "help": "evaluation data_dir inside --dataset_name (a single file: its first 5 %% is held out instead)"})
    split: Optional[str] = field(default="train")
    num_workers: Optional[int] = field(default=None, metadata={"help": "num_proc of the dataset load"})
    synthetic_data: Optional[bool] = field(default=False, metadata={
        "help": "train on synthetic prompt/chosen/rejected triples instead of --dataset_name"})
    synthetic_samples: Optional[int] = field(default=10000)
    synthetic_chars: Optional[int] = field(default=None, metadata={
        "help": "pad every synthetic prompt + response to about this many characters (throughput runs)"})
    model_overrides: Optional[str] = field(default=None)
    torch_dtype: Optional[str] = field(default="bfloat16")
    load_in_4bit: Optional[bool] = field(default=False, metadata={"help": "4-bit frozen bases (dpo_llama2.py:133-152)"})
    bnb_4bit_quant_type: Optional[str] = field(default="nf4")
    final_save: Optional[bool] = field(default=True, metadata={
        "help": "save the trained model / adapter at the end (false: throughput runs of 7B models)"})
    bf16: Optional[bool] = field(default=True)
    seed: Optional[int] = field(default=0)
    use_cpu: Optional[bool] = field(default=False)
    ddp_backend: Optional[str] = field(default=None, metadata={"help": "nccl (RCCL) | gloo; default: HF's choice"})


def _length_filter(rows, max_length):
    """dpo_llama2.py:157-161 / :165-168 (characters, like the reference)."""
    return [r for r in rows if _pair_length_ok(r, max_length)]


def _is_dataset(rows) -> bool:
    return hasattr(rows, "select") and hasattr(rows, "map") and hasattr(rows, "__len__")


def load_pairs(args, data_dir=None, sanity_check=None):
    """prompt / chosen / rejected rows of ``data_dir`` (default ``--subset``)
    in ``--dataset_name``, mapped and length-filtered like the reference
    (dpo_llama2.py:84-125, :157-161): a ``datasets.Dataset`` stays one (batched
    map + filter, ``--num_workers`` processes), a lazily read json-lines file
    becomes a list; synthetic triples with ``--synthetic_data``.
    ``sanity_check`` keeps the first 1000 rows (before the length filter, as
    the reference's ``select(range(1000))``)."""
    import itertools

    sanity_check = args.sanity_check if sanity_check is None else sanity_check
    ddir = args.subset if data_dir is None else data_dir
    if args.synthetic_data:
        rows = synthetic_paired(args.synthetic_samples, seed=args.seed, target_chars=args.synthetic_chars)
        return _length_filter(rows[:1000] if sanity_check else rows, args.max_length)
    src = load_named_rows(args.dataset_name, data_dir=ddir, split=args.split, num_workers=args.num_workers)
    if _is_dataset(src):
        if sanity_check:
            src = src.select(range(min(len(src), 1000)))
        rows = stack_exchange_pairs_dataset(src, args.max_length, num_proc=args.num_workers)
    else:
        rows = _length_filter(stack_exchange_pairs(itertools.islice(iter(src), 1000) if sanity_check else src),
                              args.max_length)
    logger.info("DPO rows from %s (data_dir=%s): %d", args.dataset_name, ddir, len(rows))
    return rows


def train_eval_pairs(args):
    """(train, eval) rows: eval from ``--eval_subset`` of a dataset directory
    (first 1000 rows, the reference's ``sanity_check=True`` eval load,
    dpo_llama2.py:164), else the front 5 % of the training rows (a single
    file or synthetic data has no evaluation subset)."""
    rows = load_pairs(args)
    name = args.dataset_name
    if not args.synthetic_data and args.eval_subset and name and not os.path.isfile(name):
        try:
            return rows, load_pairs(args, data_dir=args.eval_subset, sanity_check=True)
        except DatasetUnavailable as e:
            logger.warning("no evaluation subset (%s); holding out the front of the training rows", e)
    n_eval = max(1, min(len(rows) // 20, 1000))
    if _is_dataset(rows):
        return rows.select(range(n_eval, len(rows))), rows.select(range(n_eval))
    return rows[n_eval:], rows[:n_eval]


def main(argv=None):
    parser = HfArgumentParser((ScriptArguments, LionArguments))
    script_args, lion_args = parser.parse_args_into_dataclasses(args=argv)
    logging.basicConfig(level=logging.INFO, handlers=[logging.StreamHandler(sys.stdout)])
    transformers.set_seed(script_args.seed)

    config = load_config(script_args.model_name_or_path, overrides=script_args.model_overrides)
    tokenizer = load_tokenizer(script_args.model_name_or_path)
    model = build_model(config, model_name_or_path=script_args.model_name_or_path,
                        torch_dtype=script_args.torch_dtype)
    model_ref = build_model(config, model_name_or_path=script_args.model_name_or_path,
                            torch_dtype=script_args.torch_dtype)
    model_ref.load_state_dict(model.state_dict())  # identical frozen reference (also for random init)
    model_ref.requires_grad_(False)
    if script_args.load_in_4bit:
        from distributed_lion_pytorch_amd.models.quant import QuantConfig, quantize_model

        qc = QuantConfig(bnb_4bit_quant_type=script_args.bnb_4bit_quant_type,
                         bnb_4bit_compute_dtype=getattr(torch, script_args.torch_dtype))
        quantize_model(model, qc)
        quantize_model(model_ref, qc)
    train_rows, eval_rows = train_eval_pairs(script_args)

    training_args = TrainingArguments(
        per_device_train_batch_size=script_args.per_device_train_batch_size,
        per_device_eval_batch_size=script_args.per_device_eval_batch_size,
        max_steps=script_args.max_steps,
        logging_steps=script_args.logging_steps,
        save_steps=script_args.save_steps,
        gradient_accumulation_steps=script_args.gradient_accumulation_steps,
        gradient_checkpointing=False,  # decided on the native model below
        learning_rate=script_args.learning_rate,
        eval_strategy="steps" if script_args.eval_steps else "no",
        eval_steps=script_args.eval_steps,
        output_dir=script_args.output_dir,
        report_to=script_args.report_to,
        lr_scheduler_type=script_args.lr_scheduler_type,
        warmup_steps=script_args.warmup_steps,
        weight_decay=script_args.weight_decay,
        bf16=script_args.bf16 and not script_args.use_cpu,
        remove_unused_columns=False,
        run_name="dpo_llama2",
        seed=script_args.seed,
        use_cpu=script_args.use_cpu,
        ddp_backend=script_args.ddp_backend,
    )
    apply_lion_args(training_args, lion_args)  # --lion_* knobs, incl. --lion_elastic_timeout (worker dropout)

    peft_config = None
    if script_args.use_lora:
        peft_config = LoraConfig(r=script_args.lora_r, lora_alpha=int(script_args.lora_alpha),
                                 lora_dropout=script_args.lora_dropout,
                                 target_modules=["q_proj", "v_proj", "k_proj"], bias="none",
                                 task_type="CAUSAL_LM")
        from distributed_lion_pytorch_amd.models.lora import inject_lora

        inject_lora(model, peft_config)
    print_trainable_parameters(model)
    # decided after LoRA injection and with the reference frozen: the estimate counts a
    # gradient + momentum only for what trains (all-trainable counting overstated it 3x
    # and checkpointed a batch that fits)
    from distributed_lion_pytorch_amd.trainer.memory import should_checkpoint

    tokens = 2 * script_args.per_device_train_batch_size * script_args.max_length  # chosen + rejected
    if should_checkpoint(script_args.gradient_checkpointing, script_args.checkpointing_policy, config, tokens,
                         model, model_ref):
        model.gradient_checkpointing_enable()
    elif script_args.gradient_checkpointing:
        logger.info("gradient checkpointing not needed: activations fit in device memory (--checkpointing_policy auto)")

    params = [p for p in model.parameters() if p.requires_grad]
    if script_args.lion:
        optimizer = build_lion(model, training_args)  # weight_decay = script_args.weight_decay (D10)
    else:
        optimizer = torch.optim.AdamW(params, lr=script_args.learning_rate, weight_decay=0.1)
    sched = transformers.get_cosine_schedule_with_warmup(optimizer, script_args.warmup_steps, script_args.max_steps)

    trainer_class = AsyncDPOTrainer if script_args.async_grad else DPOTrainer
    trainer = trainer_class(model, model_ref, args=training_args, beta=script_args.beta, train_dataset=train_rows,
                            eval_dataset=eval_rows, tokenizer=tokenizer, max_prompt_length=script_args.max_prompt_length,
                            max_length=script_args.max_length, peft_config=None, optimizers=(optimizer, sched),
                            callbacks=[])
    # tokens/s counts what the policy actually processed (chosen + rejected, padded), not max_length
    trainer.add_callback(JsonlMetricsCallback(script_args.output_dir, token_count=lambda: trainer.tokens_seen))
    training_args.lion, training_args.async_grad = script_args.lion, script_args.async_grad
    warn_unsynced(training_args)
    trainer.train()
    if not script_args.final_save:
        return trainer
    trainer.save_model(script_args.output_dir)
    if trainer.is_world_process_zero():
        from distributed_lion_pytorch_amd.models.lora import save_adapter

        out = os.path.join(script_args.output_dir, "final_checkpoint")
        if script_args.use_lora:
            save_adapter(trainer.model, out)
        else:
            trainer.accelerator.unwrap_model(trainer.model).save_pretrained(out)
    return trainer


if __name__ == "__main__":
    main()
