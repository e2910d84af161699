"""Direct Preference Optimization trainer (native replacement for trl's DPOTrainer).

Reference: /root/reference/dpo_llama2.py (does not parse) wires
``trl.DPOTrainer(model, model_ref, beta=0.1, max_prompt_length=512,
max_length=1024, peft_config=...)`` with the stack-exchange paired data
(prompt / chosen / rejected).  Implemented here on HF ``Trainer``:

* collator: prompt (left-truncated to ``max_prompt_length``) + response + EOS,
  truncated to ``max_length``; prompt tokens masked with -100 in the labels;
* loss (trl "sigmoid"): -log sigma(beta * [(log pi(c) - log pi(r)) -
  (log pi_ref(c) - log pi_ref(r))]), optional label smoothing (cDPO) and
  "ipo"; chosen and rejected go through the policy in ONE concatenated forward;
* reference model: frozen copy (or the explicit ``ref_model``).

``AsyncDPOTrainer`` adds the no-gradient-sync step (async_trainer.py:65-90).
"""
from __future__ import annotations

import copy
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F
from transformers import Trainer

from ..models.lora import LoraConfig, inject_lora
from .async_trainer import AsyncMixin


def sequence_logps(model, input_ids: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """Summed log p(label_t) per sequence; labels -100 ignored."""
    fn = getattr(model, "sequence_logps", None)
    if fn is not None:
        return fn(input_ids, labels)
    logits = model(input_ids=input_ids).logits[:, :-1].float()
    tgt = labels[:, 1:]
    mask = tgt != -100
    lp = torch.log_softmax(logits, -1).gather(-1, tgt.clamp_min(0).unsqueeze(-1)).squeeze(-1)
    return (lp * mask).sum(-1)


class DPOCollator:
    def __init__(self, tokenizer, max_length: int = 1024, max_prompt_length: int = 512):
        self.tok = tokenizer
        self.max_length = max_length
        self.max_prompt_length = max_prompt_length
        self.pad = tokenizer.pad_token_id if tokenizer.pad_token_id is not None else tokenizer.eos_token_id

    def _encode(self, prompt: str, response: str):
        p = self.tok(prompt, add_special_tokens=False)["input_ids"][-self.max_prompt_length:]
        r = self.tok(response, add_special_tokens=False)["input_ids"] + [self.tok.eos_token_id]
        ids = (p + r)[: self.max_length]
        labels = ([-100] * len(p) + r)[: self.max_length]
        return ids, labels

    def __call__(self, examples: List[Dict[str, str]]) -> Dict[str, torch.Tensor]:
        seqs = [self._encode(e["prompt"], e["chosen"]) for e in examples]
        seqs += [self._encode(e["prompt"], e["rejected"]) for e in examples]
        width = max(len(s[0]) for s in seqs)
        width = (width + 63) // 64 * 64  # kernel-friendly lengths (flash attention T % 64)
        ids = torch.full((len(seqs), width), self.pad, dtype=torch.long)
        labels = torch.full((len(seqs), width), -100, dtype=torch.long)
        for i, (a, b) in enumerate(seqs):
            ids[i, : len(a)] = torch.tensor(a)
            labels[i, : len(b)] = torch.tensor(b)
        return {"input_ids": ids, "labels": labels}


def dpo_loss(pc, pr, rc, rr, beta: float, loss_type: str = "sigmoid", label_smoothing: float = 0.0):
    logits = (pc - pr) - (rc - rr)
    if loss_type == "sigmoid":
        loss = -F.logsigmoid(beta * logits) * (1 - label_smoothing) - F.logsigmoid(-beta * logits) * label_smoothing
    elif loss_type == "ipo":
        loss = (logits - 1 / (2 * beta)) ** 2
    else:
        raise ValueError(f"unknown DPO loss_type {loss_type}")
    return loss.mean(), beta * (pc - rc).detach(), beta * (pr - rr).detach()


class DPOTrainer(Trainer):
    def __init__(self, model=None, ref_model=None, args=None, beta: float = 0.1, train_dataset=None,
                 eval_dataset=None, tokenizer=None, processing_class=None, max_prompt_length: int = 512,
                 max_length: int = 1024, peft_config: Optional[LoraConfig] = None, loss_type: str = "sigmoid",
                 label_smoothing: float = 0.0, **kwargs):
        tok = processing_class if processing_class is not None else tokenizer
        if ref_model is None:
            ref_model = copy.deepcopy(model)
        for p in ref_model.parameters():
            p.requires_grad_(False)
        ref_model.eval()
        if peft_config is not None:
            inject_lora(model, peft_config)
        self.ref_model = ref_model
        self.beta, self.loss_type, self.label_smoothing = beta, loss_type, label_smoothing
        args.remove_unused_columns = False
        super().__init__(model=model, args=args, train_dataset=train_dataset, eval_dataset=eval_dataset,
                         processing_class=tok, data_collator=DPOCollator(tok, max_length, max_prompt_length),
                         **kwargs)
        # device [chosen, rejected, accuracy, margin, micro-batches] since the last log, kept apart for
        # training and evaluation batches (trl reports them as rewards/* and eval_rewards/*)
        self._reward_acc = {"train": None, "eval": None}
        self.tokens_seen = 0  # training tokens through the policy (chosen + rejected, padded), host-side count

    _REWARD_KEYS = ("rewards/chosen", "rewards/rejected", "rewards/accuracies", "rewards/margins")

    def compute_loss(self, model, inputs, return_outputs=False, num_items_in_batch=None):
        ids, labels = inputs["input_ids"], inputs["labels"]
        n = ids.shape[0] // 2
        if model.training:
            self.tokens_seen += ids.numel()
        if next(self.ref_model.parameters()).device != ids.device:
            self.ref_model.to(ids.device)
        policy = self.accelerator.unwrap_model(model)
        logp = sequence_logps(policy, ids, labels)
        with torch.no_grad():
            ref_logp = sequence_logps(self.ref_model, ids, labels)
        loss, r_c, r_r = dpo_loss(logp[:n], logp[n:], ref_logp[:n], ref_logp[n:], self.beta, self.loss_type,
                                  self.label_smoothing)
        # reward statistics stay on the device (no .item() per micro-batch: each
        # one drained the queue, the host sync the HF nan filter fix removed);
        # log() reads the window's means with one transfer
        stats = torch.stack([r_c.float().mean(), r_r.float().mean(), (r_c > r_r).float().mean(),
                             (r_c - r_r).float().mean(), torch.ones((), device=r_c.device)])
        split = "train" if model.training else "eval"
        acc = self._reward_acc[split]
        self._reward_acc[split] = stats if acc is None else acc + stats
        return (loss, {"loss": loss}) if return_outputs else loss

    def reward_stats(self, reset: bool = True, split: str = "train") -> Dict[str, float]:
        """Means of the reward statistics of ``split`` ("train" / "eval") over
        the micro-batches since the last call (one device-to-host copy); eval
        keys carry trl's ``eval_`` prefix."""
        acc = self._reward_acc.get(split)
        if acc is None:
            return {}
        v = acc.tolist()
        if reset:
            self._reward_acc[split] = None
        n = max(v[4], 1.0)
        prefix = "eval_" if split == "eval" else ""
        return {prefix + k: x / n for k, x in zip(self._REWARD_KEYS, v[:4])}

    def log(self, logs, *args, **kwargs):
        # an evaluation log (eval_* keys) gets the evaluation batches' statistics,
        # a training log the training batches' -- never a mix of the two
        is_eval = any(k.startswith("eval_") for k in logs)
        logs.update(self.reward_stats(split="eval" if is_eval else "train"))
        return super().log(logs, *args, **kwargs)


class AsyncDPOTrainer(AsyncMixin, DPOTrainer):
    """DPO with per-worker gradients; replicas synchronised by Lion's vote."""
