"""Observability: JSONL metrics stream, HIP-event phase timers, wire-byte counters.

The reference only has HF logging + wandb (with a hard-coded key).
Here every logging step appends one JSON object to ``<output_dir>/metrics.jsonl``
on rank 0 with the HF logs (loss, lr, grad_norm, ...), tokens/s since the
previous record, and the Lion exchange counters (wire bytes sent/received,
collective count, vote agreement when telemetry is on).  No network service.
"""
from __future__ import annotations

import json
import os
import time
from typing import Optional

import torch

try:
    from transformers import TrainerCallback
except ImportError:  # pragma: no cover - the engine/bench path does not need HF
    TrainerCallback = object

from .timing import PhaseTimer, phase_of  # noqa: F401  (re-export)


def is_rank0() -> bool:
    import torch.distributed as dist

    return not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0


class JsonlMetricsCallback(TrainerCallback):
    def __init__(self, output_dir: str, seq_len: Optional[int] = None, filename: str = "metrics.jsonl",
                 token_count=None):
        """``token_count``: optional callable returning this rank's cumulative
        training tokens (variable-length batches, e.g. DPO); otherwise tokens
        = steps x batch x accumulation x world x ``seq_len``."""
        self.path = os.path.join(output_dir, filename)
        self.seq_len = seq_len
        self.token_count = token_count
        self._t = None
        self._step = 0
        self._tok = 0

    def on_train_begin(self, args, state, control, **kw):
        self._t = time.perf_counter()
        self._step = state.global_step
        self._tok = self.token_count() if self.token_count else 0

    def on_log(self, args, state, control, logs=None, optimizer=None, **kw):
        if not is_rank0():
            timer = getattr(getattr(optimizer, "optimizer", optimizer), "phase_timer", None)
            if timer is not None:
                timer.reset()  # only rank 0 reports; the others must not accumulate events
            return
        now = time.perf_counter()
        rec = {"step": state.global_step, "time": time.time()}
        rec.update(logs or {})
        world = max(1, args.world_size)
        if self._t is not None and state.global_step > self._step and self.token_count is not None:
            tok = self.token_count()
            rec["tokens_per_s"] = (tok - self._tok) * world / max(now - self._t, 1e-9)
            self._tok = tok
        elif self._t is not None and state.global_step > self._step and self.seq_len:
            steps = state.global_step - self._step
            toks = steps * args.per_device_train_batch_size * args.gradient_accumulation_steps * world * self.seq_len
            rec["tokens_per_s"] = toks / max(now - self._t, 1e-9)
        self._t, self._step = now, state.global_step
        opt = getattr(optimizer, "optimizer", optimizer)  # accelerate wraps it
        if opt is not None and hasattr(opt, "stats"):
            rec["lion"] = opt.stats(reset=True)
        timer = getattr(opt, "phase_timer", None)
        if timer is not None:
            # mean ms per optimizer step since the last record: fwd_bwd, clip and
            # the vote's encode / exchange (exposed comm) / apply, or local_update
            rec["phase_ms_per_step"] = {k: round(v, 3) for k, v in timer.summary(reset=True).items()}
        os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
        with open(self.path, "a") as f:
            f.write(json.dumps(rec, default=float) + "\n")
