"""Native training step: local forward/backward per rank, Lion vote sync.

This is the loop that ``bench.py`` and the native (non-HF) entrypoint paths
run.  It reproduces the HF ``Trainer`` inner loop the reference relies on
(SURVEY §3.2): gradient accumulation with loss/GA scaling, per-rank gradient
clipping (HF default ``max_grad_norm=1.0``, a *local* norm -- no collective),
``optimizer.step()``, LR scheduler, ``zero_grad`` -- and, like
``AsyncTrainer`` (/root/reference/async_trainer.py:13-34), it never
all-reduces gradients: replicas stay in sync only through the optimizer's
majority vote.
"""
from __future__ import annotations

import time
from typing import Callable, Iterable, Optional

import torch
import torch.distributed as dist

from ..parallel.elastic import fault_spec
from ..parallel.elastic import inject as inject_fault
from ..utils.timing import phase_of


def broadcast_parameters(model: torch.nn.Module, src: int = 0, group=None) -> None:
    """One-time replica initialisation (what DDP's constructor broadcast did
    for the reference, ACC:accelerator.py:1892).  Coalesced into one flat
    buffer per dtype so it is a handful of RCCL broadcasts, not one per tensor."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    by_dtype = {}
    seen = set()
    for t in list(model.parameters()) + list(model.buffers()):
        if t.data_ptr() in seen:
            continue
        seen.add(t.data_ptr())
        by_dtype.setdefault((t.dtype, t.device), []).append(t)
    for (dt, dev), ts in by_dtype.items():
        if dist.get_backend(group) == "nccl" and dev.type != "cuda":
            continue
        flat = torch.cat([t.detach().reshape(-1) for t in ts])
        dist.broadcast(flat, src=src, group=group)
        off = 0
        with torch.no_grad():
            for t in ts:
                n = t.numel()
                t.copy_(flat[off:off + n].view_as(t))
                off += n


class TrainStep:
    """One optimizer step = ``grad_accum`` micro-batches + clip + Lion step."""

    def __init__(self, model, optimizer, grad_accum: int = 1, max_grad_norm: Optional[float] = 1.0,
                 scheduler=None, loss_fn: Optional[Callable] = None, fuse_grad_accumulation: Optional[bool] = None):
        self.model = model
        self.optimizer = optimizer
        self.grad_accum = max(1, int(grad_accum))
        self.max_grad_norm = max_grad_norm
        self.scheduler = scheduler
        self.loss_fn = loss_fn or (lambda m, b: m(b["input_ids"], labels=b["labels"])["loss"])
        self.params = [p for p in model.parameters() if p.requires_grad]
        # weight gradients land straight in param.grad (ops/linear.py); off under
        # DDP, whose reducer relies on AccumulateGrad hooks
        if fuse_grad_accumulation is None:
            fuse_grad_accumulation = not isinstance(model, torch.nn.parallel.DistributedDataParallel)
        self.fuse_grad_accumulation = fuse_grad_accumulation

    def _fused_clip(self) -> bool:
        """Lion's fused clip covers exactly its own parameters: use it only when
        those are the parameters being trained (else the norm would differ)."""
        if not hasattr(self.optimizer, "clip_grad_norm_"):
            return False
        if not hasattr(self, "_fused_ok"):
            mine = {id(p) for g in self.optimizer.param_groups for p in g["params"]}
            self._fused_ok = mine == {id(p) for p in self.params}
        return self._fused_ok

    def set_timer(self, timer) -> None:
        """Attach a :class:`~..utils.timing.PhaseTimer` (``None`` detaches):
        phases ``fwd_bwd`` / ``clip`` / ``optimizer`` here, and the Lion
        step's own ``encode`` / ``exchange`` / ``apply`` (or ``local_update``)."""
        self.timer = timer
        if hasattr(self.optimizer, "phase_timer"):
            self.optimizer.phase_timer = timer

    def __call__(self, micro_batches: Iterable[dict]) -> torch.Tensor:
        from ..ops.linear import grad_accumulation_fusion

        t = getattr(self, "timer", None)
        self.model.train()
        total = None
        with phase_of(t, "fwd_bwd"):
            with grad_accumulation_fusion(self.fuse_grad_accumulation, micro_batches=self.grad_accum):
                for batch in micro_batches:
                    loss = self.loss_fn(self.model, batch) / self.grad_accum
                    if fault_spec() and loss.requires_grad:  # DLION_FAULT=rank:step:backward
                        n = getattr(self.optimizer, "_n_steps", 0)
                        loss.register_hook(lambda g, n=n: inject_fault("backward", n))
                    loss.backward()
                    total = loss.detach() if total is None else total + loss.detach()
        if self.max_grad_norm is not None and self.max_grad_norm > 0:
            with phase_of(t, "clip"):
                if self._fused_clip():
                    # norm on device, scale applied inside the Lion update kernels
                    self.optimizer.clip_grad_norm_(self.max_grad_norm)
                else:
                    torch.nn.utils.clip_grad_norm_(self.params, self.max_grad_norm, foreach=True)
        with phase_of(t, "optimizer"):
            self.optimizer.step()
        if self.scheduler is not None:
            self.scheduler.step()
        self.optimizer.zero_grad(set_to_none=True)
        if t is not None:
            t.step()
        from ..ops.fused import check_index_errors

        check_index_errors()  # out-of-range token ids / labels flagged by the kernels (one step late, no stall)
        return total


class StepTimer:
    """Wall-clock timing bracketed by barrier + device synchronize (bench contract)."""

    def __init__(self, device: torch.device):
        self.device = device

    def sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        if dist.is_available() and dist.is_initialized():
            dist.barrier()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def __enter__(self):
        self.sync()
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        self.sync()
        self.elapsed = time.perf_counter() - self.t0
        return False
