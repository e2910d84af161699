#!/usr/bin/env python
"""Causal-LM (GPT-2 / Llama) pretraining with Distributed Lion -- drop-in for
/root/reference/run_clm.py (same CLI: ModelArguments, DataTrainingArguments,
TrainingArguments + ``--lion`` / ``--async_grad``), MI355X-native underneath:

* the model is our native GPT-2/Llama (HF checkpoint format, gfx950 kernels)
  unless ``--native_model false`` selects the stock HF class;
* ``--lion`` builds the distributed Lion (1-bit vote exchange over RCCL);
  ``--async_grad`` trains with per-rank gradients (``AsyncTrainer``);
* runs offline: ``--synthetic_data`` (or no dataset) trains on random token
  blocks; ``--train_file`` / ``--validation_file`` are read by extension
  (txt / csv / json / jsonl, the "text" column or the first one) like the
  reference, and ``--streaming`` tokenizes and groups them lazily (a corpus
  larger than host memory streams through); configs come from the built-in
  size registry (``--config_name gpt2``) or a local directory;
* no wandb login, no hub telemetry; AdamW fallback keeps the
  reference's hard-coded weight_decay=0.1 (D17) and warns about it.

  torchrun --nproc_per_node 8 run_clm.py --config_name gpt2 --synthetic_data \
      --per_device_train_batch_size 20 --gradient_accumulation_steps 8 --bf16 \
      --torch_dtype bfloat16 --max_steps 100 --lion --async_grad --output_dir out
"""
from __future__ import annotations

import logging
import math
import os
import sys
from dataclasses import dataclass, field
from typing import Optional

import torch
import transformers
from transformers import HfArgumentParser, set_seed
from transformers.trainer_utils import get_last_checkpoint

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_lion_pytorch_amd.models.registry import build_model, load_config  # noqa: E402
from distributed_lion_pytorch_amd.trainer.async_trainer import (  # noqa: E402
    AsyncTrainer, AsyncTrainingArguments, LocalTrainer, build_lion, warn_unsynced)
from distributed_lion_pytorch_amd.utils.data import (CLMStream, SyntheticCLMDataset, clm_blocks,  # noqa: E402
                                                     column_texts, default_cache_dir, load_local_splits,
                                                     load_tokenizer)
from distributed_lion_pytorch_amd.utils.metrics import JsonlMetricsCallback  # noqa: E402

logger = logging.getLogger(__name__)


@dataclass
class ModelArguments:
    model_name_or_path: Optional[str] = field(default=None, metadata={"help": "checkpoint dir for weight init"})
    model_type: Optional[str] = field(default=None, metadata={"help": "gpt2 | llama when training from scratch"})
    config_overrides: Optional[str] = field(default=None, metadata={"help": "e.g. n_embd=10,resid_pdrop=0.2"})
    config_name: Optional[str] = field(default=None, metadata={"help": "size name (gpt2, llama-2-7b, ...) or dir"})
    tokenizer_name: Optional[str] = field(default=None, metadata={"help": "local tokenizer dir (else byte-level)"})
    cache_dir: Optional[str] = field(default=None)
    use_fast_tokenizer: bool = field(default=True)
    model_revision: str = field(default="main")
    use_auth_token: bool = field(default=False)
    torch_dtype: Optional[str] = field(default=None, metadata={"help": "auto | bfloat16 | float16 | float32"})
    low_cpu_mem_usage: bool = field(default=False)
    native_model: bool = field(default=True, metadata={"help": "native MI355X model (False: stock HF class)"})


@dataclass
class DataTrainingArguments:
    dataset_name: Optional[str] = field(default=None)
    dataset_config_name: Optional[str] = field(default=None)
    train_file: Optional[str] = field(default=None, metadata={"help": "local csv / json / jsonl / txt file"})
    validation_file: Optional[str] = field(default=None)
    max_train_samples: Optional[int] = field(default=None)
    max_eval_samples: Optional[int] = field(default=None)
    streaming: bool = field(default=False)
    block_size: Optional[int] = field(default=None)
    overwrite_cache: bool = field(default=False)
    validation_split_percentage: Optional[int] = field(default=5)
    preprocessing_num_workers: Optional[int] = field(default=None)
    keep_linebreaks: bool = field(default=True)
    synthetic_samples: int = field(default=100_000, metadata={"help": "size of the synthetic train set"})


def split_train_validation(texts, pct: int):
    """The reference's split when a corpus has no validation part
    (/root/reference/run_clm.py:326-341, 364-380): ``validation = train[:pct%]``,
    ``train = train[pct%:]`` -- disjoint, validation taken from the front (HF
    percent slicing rounds the boundary to the closest row)."""
    n_val = int(round(len(texts) * pct / 100.0))
    return texts[n_val:], texts[:n_val]


def _blocks(texts, tokenizer, block_size, data_args=None, train_args=None):
    """Tokenize + group_texts as the reference's two batched ``datasets.map``
    calls (run_clm.py:463-544: 1000-text batches, no separator, per-batch
    remainder dropped), honouring ``preprocessing_num_workers`` and
    ``overwrite_cache``; ranks other than the main one wait and read the cache."""
    workers = getattr(data_args, "preprocessing_num_workers", None)
    overwrite = bool(getattr(data_args, "overwrite_cache", False))
    cache = default_cache_dir()
    first = getattr(train_args, "main_process_first", None)
    if first is None:
        return clm_blocks(texts, tokenizer, block_size, workers, cache, overwrite)
    with first(desc="dataset map tokenization"):
        return clm_blocks(texts, tokenizer, block_size, workers, cache, overwrite)


def _cap(ds, n: Optional[int]):
    """``max_train_samples`` / ``max_eval_samples``: the first n blocks
    (reference run_clm.py:550-560 ``select(range(n))``)."""
    if n is None or ds is None or len(ds) <= n:
        return ds
    return torch.utils.data.Subset(ds, range(n))


def build_datasets(data_args, train_args, tokenizer, vocab_size, block_size, cache_dir=None):
    pct = data_args.validation_split_percentage if data_args.validation_split_percentage is not None else 5
    if data_args.dataset_name and not train_args.synthetic_data:
        import datasets

        name = data_args.dataset_name
        try:
            if os.path.isdir(name) and (os.path.isfile(os.path.join(name, "dataset_dict.json"))
                                        or os.path.isfile(os.path.join(name, "state.json"))):
                raw = datasets.load_from_disk(name)  # a save_to_disk directory
            else:  # a local dataset repository (data files) or a hub name in the HF cache
                raw = datasets.load_dataset(name, data_args.dataset_config_name)
        except Exception as e:  # a name that resolves to nothing is an error, never random words
            raise FileNotFoundError(
                f"dataset {name!r} could not be loaded ({type(e).__name__}: {e}); point --dataset_name at a local "
                "dataset directory, use --train_file, or pass --synthetic_data") from e
        col = "text" if "text" in raw["train"].column_names else raw["train"].column_names[0]
        if "validation" in raw:  # the dataset's own validation split
            tr, va = list(raw["train"][col]), list(raw["validation"][col])
        else:
            tr, va = split_train_validation(list(raw["train"][col]), pct)
        return (_cap(_blocks(tr, tokenizer, block_size, data_args, train_args), data_args.max_train_samples),
                _cap(_blocks(va, tokenizer, block_size, data_args, train_args), data_args.max_eval_samples))
    if (data_args.train_file or data_args.validation_file) and not train_args.synthetic_data:
        # by extension through datasets.load_dataset (reference run_clm.py:343-381)
        tr, va, col = load_local_splits(data_args.train_file, data_args.validation_file, data_args.keep_linebreaks,
                                        pct, streaming=data_args.streaming, cache_dir=cache_dir)
        if data_args.streaming:
            # lazy tokenize + group_texts; no main_process_first: nothing is cached
            # (the reference's streaming maps run without num_proc / cache files, :484-489, :540-544)
            return (CLMStream(tr, col, tokenizer, block_size, shard=True, max_blocks=data_args.max_train_samples)
                    if tr is not None else None,
                    CLMStream(va, col, tokenizer, block_size, shard=False, max_blocks=data_args.max_eval_samples)
                    if va is not None else None)
        return (_cap(_blocks(column_texts(tr, col), tokenizer, block_size, data_args, train_args),
                     data_args.max_train_samples),
                _cap(_blocks(column_texts(va, col), tokenizer, block_size, data_args, train_args),
                     data_args.max_eval_samples))
    n_train = data_args.max_train_samples or data_args.synthetic_samples
    n_eval = data_args.max_eval_samples or max(8, n_train // 20)
    # disjoint by construction: the eval set is drawn from a different seed
    return (SyntheticCLMDataset(n_train, block_size, vocab_size, seed=train_args.seed),
            SyntheticCLMDataset(n_eval, block_size, vocab_size, seed=train_args.seed + 1))


def _n_samples(ds, cap):
    """len() of a map-style set; for a stream the cap (or -1: unknown)."""
    try:
        return len(ds)
    except TypeError:
        return cap if cap is not None else -1


def resize_embeddings_for(model, tokenizer) -> bool:
    """Grow the embedding (and tied LM head) when the tokenizer has more ids
    than the model (/root/reference/run_clm.py:446-450).  Returns True if resized."""
    emb = model.get_input_embeddings().weight.shape[0]
    if len(tokenizer) > emb:
        model.resize_token_embeddings(len(tokenizer))
        return True
    return False


def main(argv=None):
    parser = HfArgumentParser((ModelArguments, DataTrainingArguments, AsyncTrainingArguments))
    if argv is None and len(sys.argv) == 2 and sys.argv[1].endswith(".json"):
        model_args, data_args, training_args = parser.parse_json_file(json_file=os.path.abspath(sys.argv[1]))
    else:
        model_args, data_args, training_args = parser.parse_args_into_dataclasses(args=argv)

    if data_args.streaming and not (data_args.train_file or data_args.validation_file):
        # the reference streams hub datasets (run_clm.py:323); there is no hub here: streaming
        # covers local files (--train_file / --validation_file), refuse it for anything else
        raise ValueError("--streaming needs --train_file / --validation_file (local files; there is no hub "
                         "offline): synthetic data and saved datasets are map-style")
    if data_args.streaming and training_args.do_train and not (training_args.max_steps and training_args.max_steps > 0):
        raise ValueError("--streaming needs --max_steps (a stream has no length; reference run_clm.py:204)")

    logging.basicConfig(format="%(asctime)s - %(levelname)s - %(name)s - %(message)s", datefmt="%m/%d/%Y %H:%M:%S",
                        handlers=[logging.StreamHandler(sys.stdout)])
    log_level = training_args.get_process_log_level()
    logger.setLevel(log_level)
    transformers.utils.logging.set_verbosity(log_level)
    logger.warning(f"Process rank: {training_args.local_rank}, device: {training_args.device}, "
                   f"n_gpu: {training_args.n_gpu}, distributed: {training_args.parallel_mode.value}, "
                   f"bf16: {training_args.bf16}, lion: {training_args.lion}, async_grad: {training_args.async_grad}")

    last_checkpoint = None
    if os.path.isdir(training_args.output_dir) and training_args.do_train:
        last_checkpoint = get_last_checkpoint(training_args.output_dir)
        if last_checkpoint is not None and training_args.resume_from_checkpoint is None:
            logger.info(f"Checkpoint detected, resuming training at {last_checkpoint}.")
    set_seed(training_args.seed)

    config = load_config(model_args.config_name or model_args.model_name_or_path or model_args.model_type or "gpt2",
                         overrides=model_args.config_overrides)
    tokenizer = load_tokenizer(model_args.tokenizer_name or model_args.model_name_or_path)
    model = build_model(config, model_name_or_path=model_args.model_name_or_path, native=model_args.native_model,
                        torch_dtype=model_args.torch_dtype)
    if resize_embeddings_for(model, tokenizer):
        logger.warning(f"resized the token embeddings to the tokenizer's {len(tokenizer)} ids")
    n_params = sum({p.data_ptr(): p.numel() for p in model.parameters()}.values())
    logger.info(f"model {config.model_type}: {n_params / 2 ** 20:.2f}M params")

    max_pos = getattr(config, "n_positions", None) or getattr(config, "max_position_embeddings", 1024)
    block_size = min(data_args.block_size or 1024, max_pos)
    train_ds, eval_ds = build_datasets(data_args, training_args, tokenizer, model.config.vocab_size, block_size,
                                       cache_dir=model_args.cache_dir)

    def preprocess_logits_for_metrics(logits, labels):
        if isinstance(logits, tuple):
            logits = logits[0]
        return logits.argmax(dim=-1)

    def compute_metrics(eval_preds):  # token accuracy (evaluate.load("accuracy") offline-free)
        preds, labels = eval_preds
        labels = labels[:, 1:].reshape(-1)
        preds = preds[:, :-1].reshape(-1)
        mask = labels != -100
        return {"accuracy": float((preds[mask] == labels[mask]).mean())}

    optimizers = (None, None)
    if training_args.lion:
        optimizer = build_lion(model, training_args)
    else:
        logger.warning("AdamW fallback uses weight_decay=0.1 regardless of --weight_decay (reference parity, D17)")
        optimizer = torch.optim.AdamW(model.parameters(), lr=training_args.learning_rate, weight_decay=0.1)
    if training_args.max_steps and training_args.max_steps > 0:
        sched = transformers.get_cosine_schedule_with_warmup(optimizer, training_args.warmup_steps,
                                                             training_args.max_steps)
        optimizers = (optimizer, sched)
    else:  # D18: a cosine schedule over max_steps=-1 is broken; let HF derive the length
        optimizers = (optimizer, None)

    trainer_class = AsyncTrainer if training_args.async_grad else LocalTrainer
    trainer = trainer_class(
        model=model,
        args=training_args,
        train_dataset=train_ds if training_args.do_train else None,
        eval_dataset=eval_ds if training_args.do_eval else None,
        processing_class=None,
        data_collator=transformers.default_data_collator,
        compute_metrics=compute_metrics if training_args.do_eval else None,
        preprocess_logits_for_metrics=preprocess_logits_for_metrics if training_args.do_eval else None,
        optimizers=optimizers,
        callbacks=[JsonlMetricsCallback(training_args.output_dir, block_size)],
    )
    warn_unsynced(training_args)

    if training_args.do_train:
        checkpoint = training_args.resume_from_checkpoint or last_checkpoint
        train_result = trainer.train(resume_from_checkpoint=checkpoint)
        trainer.save_model()
        if hasattr(tokenizer, "save_pretrained") and trainer.is_world_process_zero():
            tokenizer.save_pretrained(training_args.output_dir)
        metrics = train_result.metrics
        metrics["train_samples"] = _n_samples(train_ds, data_args.max_train_samples)
        trainer.log_metrics("train", metrics)
        trainer.save_metrics("train", metrics)
        trainer.save_state()

    if training_args.do_eval:
        metrics = trainer.evaluate()
        metrics["eval_samples"] = _n_samples(eval_ds, data_args.max_eval_samples)
        try:
            metrics["perplexity"] = math.exp(metrics["eval_loss"])
        except OverflowError:
            metrics["perplexity"] = float("inf")
        trainer.log_metrics("eval", metrics)
        trainer.save_metrics("eval", metrics)

    # model card (reference run_clm.py:641-653); offline, so nothing is pushed
    kwargs = {"finetuned_from": model_args.model_name_or_path, "tasks": "text-generation"}
    if data_args.dataset_name:
        kwargs["dataset_tags"] = data_args.dataset_name
        kwargs["dataset"] = data_args.dataset_name if not data_args.dataset_config_name else \
            f"{data_args.dataset_name} {data_args.dataset_config_name}"
    if training_args.do_train and trainer.is_world_process_zero():
        try:
            trainer.create_model_card(**kwargs)
        except Exception as e:  # noqa: BLE001 - the card is documentation, never fail a run on it
            logger.warning("model card not written: %s", e)
    return trainer


if __name__ == "__main__":
    main()
