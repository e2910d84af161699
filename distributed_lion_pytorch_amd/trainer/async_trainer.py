"""HF ``Trainer`` integration: training with per-rank local gradients.

Reference: /root/reference/async_trainer.py:8-90 -- ``AsyncTrainer``,
``AsyncSFTTrainer``, ``AsyncDPOTrainer`` override ``training_step`` to run the
whole forward/backward under ``DDP.no_sync()`` so gradients are never
all-reduced; replicas are kept identical only by Lion's majority vote.

Re-designed for the installed transformers 5.x:
* ``training_step(model, inputs, num_items_in_batch=None)`` delegates to the
  stock implementation (GA loss scaling, loss-kwargs, CP buffers) and only
  adds the no-sync context -- no stale copy of HF internals;
* the no-sync context is a no-op when the model is not DDP-wrapped (W == 1,
  DataParallel), instead of an AttributeError;
* ``--lion`` builds the distributed Lion over the *trainable* parameters
  (LoRA-safe, D12) unless an optimizer is passed explicitly;
* every rank checkpoints its own momentum (``rank{r}-of-{W}-optimizer.pt``)
  next to HF's rank-0 ``optimizer.pt`` and reloads it on resume (D20);
* no DDP wrap at all: the reference wraps only to switch DDP off
  (/root/reference/async_trainer.py:15), but DDP's reducer still allocates a
  flat copy of every trainable gradient at wrap time (~16 GB of HBM per rank
  at Llama-3-8B full-parameter) and broadcasts the model; here the model is
  prepared without the wrap and the replicas are initialised by one coalesced
  broadcast (engine.broadcast_parameters).  ``--lion_ddp_wrap`` restores the
  reference's wrap.
"""
from __future__ import annotations

import contextlib
import logging
import os
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.distributed as dist
from transformers import Trainer, TrainingArguments

from ..optim.lion import Lion

logger = logging.getLogger(__name__)


@dataclass
class LionArguments:
    """The Lion knobs every entrypoint exposes: run_clm through
    :class:`AsyncTrainingArguments`, ``sft_llama2.py`` / ``dpo_llama2.py`` as
    their own argument group (:func:`apply_lion_args` copies them onto the
    TrainingArguments the trainer reads).  ``lion_bucket_mb`` None sizes the
    vote buckets automatically (>= 4 per step at W > 1 on RCCL, so encode of
    bucket i+1 overlaps the exchange of bucket i; optim/lion.py)."""

    lion_beta1: float = field(default=0.9, metadata={"help": "Lion beta1"})
    lion_beta2: float = field(default=0.99, metadata={"help": "Lion beta2"})
    lion_vote: str = field(default="majority", metadata={"help": "majority | average"})
    lion_tie_break: str = field(default="negative", metadata={"help": "negative (reference) | zero | positive"})
    lion_wire: str = field(default="a2a", metadata={"help": "allgather | a2a | ref_int64"})
    lion_bucket_mb: Optional[float] = field(default=None, metadata={
        "help": "packed-bit bucket size (MB); default: automatic (>= 4 pipelined buckets at W > 1)"})
    lion_stochastic_max_norm: Optional[float] = field(default=None, metadata={
        "help": "enable stochastic binarization with this max_grad_norm (reference max_grad_norm)"})
    lion_backend: str = field(default="auto", metadata={"help": "auto | hip | torch"})
    lion_dropout_schedule: Optional[str] = field(default=None, metadata={
        "help": "fault injection, e.g. '100:3' drops rank 3 from optimizer step 100 on"})
    lion_elastic_timeout: Optional[float] = field(default=None, metadata={
        "help": "real worker dropout: collective deadline (s); survivors regroup and continue "
                "(launch with python -m distributed_lion_pytorch_amd.launch for death notices)"})
    lion_ddp_wrap: bool = field(default=False, metadata={
        "help": "async trainers: let accelerate wrap the model in DDP as the reference does (its gradient "
                "buckets are never used under no_sync; default: no wrap, replicas initialised by one broadcast)"})


def apply_lion_args(training_args, lion_args: LionArguments):
    """Copy the Lion knobs onto ``training_args`` (what build_lion and the
    AsyncMixin read)."""
    import dataclasses

    for f in dataclasses.fields(LionArguments):
        setattr(training_args, f.name, getattr(lion_args, f.name))
    return training_args


@dataclass
class LegacyTrainingArguments:
    """TrainingArguments fields that the reference's command lines pass and the
    installed transformers dropped (``--group_by_length``, gone in transformers
    5; /root/reference/README.md's SFT command and sft_llama2.py:53 use it):
    accepted so those command lines still parse."""

    group_by_length: bool = field(default=False, metadata={"help": "TrainingArguments flag of transformers < 5"})


def legacy_training_arguments() -> tuple:
    """``(LegacyTrainingArguments,)`` when the installed TrainingArguments lacks
    one of its fields (add it to the HfArgumentParser), else ``()``."""
    import dataclasses

    names = {f.name for f in dataclasses.fields(TrainingArguments)}
    missing = [f.name for f in dataclasses.fields(LegacyTrainingArguments) if f.name not in names]
    return (LegacyTrainingArguments,) if missing else ()


@dataclass
class AsyncTrainingArguments(TrainingArguments, LionArguments):
    """HF TrainingArguments + the reference's flags (run_clm.py:73-86) + Lion knobs."""

    lion: bool = field(default=False, metadata={"help": "use the (distributed) Lion optimizer"})
    async_grad: bool = field(default=False, metadata={
        "help": "compute gradients per worker and never combine them (sync only via Lion's vote)"})
    synthetic_data: bool = field(default=False, metadata={"help": "train on synthetic token ids (offline)"})


def parse_dropout_schedule(spec: Optional[str]) -> dict:
    """'100:3,200:1' -> {100: [3], 200: [1]}"""
    out: dict = {}
    if not spec:
        return out
    for item in spec.split(","):
        step, rank = item.split(":")
        out.setdefault(int(step), []).append(int(rank))
    return out


def build_lion(model: torch.nn.Module, args, lr: Optional[float] = None, weight_decay: Optional[float] = None) -> Lion:
    params = [p for p in model.parameters() if p.requires_grad]
    opt = Lion(
        params,
        lr=args.learning_rate if lr is None else lr,
        betas=(getattr(args, "lion_beta1", 0.9), getattr(args, "lion_beta2", 0.99)),
        weight_decay=args.weight_decay if weight_decay is None else weight_decay,
        max_grad_norm=getattr(args, "lion_stochastic_max_norm", None),
        vote=getattr(args, "lion_vote", "majority"),
        tie_break=getattr(args, "lion_tie_break", "negative"),
        exchange=getattr(args, "lion_wire", "a2a"),
        bucket_mb=getattr(args, "lion_bucket_mb", None),
        backend=getattr(args, "lion_backend", "auto"),
        seed=getattr(args, "seed", 0),
        elastic_timeout=getattr(args, "lion_elastic_timeout", None),
    )
    sched = parse_dropout_schedule(getattr(args, "lion_dropout_schedule", None))
    if sched:
        opt.set_dropout_schedule(sched)
    return opt


def no_sync(model):
    """DDP.no_sync() when the model is DDP-wrapped, otherwise a no-op (D14)."""
    fn = getattr(model, "no_sync", None)
    return fn() if callable(fn) else contextlib.nullcontext()


def _lion_of(optimizer):
    opt = getattr(optimizer, "optimizer", optimizer)  # accelerate's AcceleratedOptimizer wraps it
    return opt if isinstance(opt, Lion) else None


class AsyncMixin:
    """Gradient-sync-free training step + Lion creation + per-rank optimizer state.

    Two engine features ride along on the HF loop (both off with
    ``DLION_HF_FUSION=0``): the micro-batches of one optimizer step form a
    gradient-accumulation fusion window (ops/linear.py: weight gradients go
    straight into ``param.grad``, split-K partials stay fp32 until the step's
    last micro-batch), and gradient clipping uses Lion's fused norm (the clip
    coefficient stays on the device and is applied inside the update kernels)
    when Lion owns exactly the model's trainable parameters."""

    def _engine_fusion(self, model) -> bool:
        if os.environ.get("DLION_HF_FUSION", "1") == "0":
            return False
        ok = getattr(self, "_dlion_fusion_ok", None)
        if ok is None:
            inner = getattr(model, "module", model)
            ok = any(p.is_cuda for p in inner.parameters()) and _lion_of(self.optimizer) is not None
            self._dlion_fusion_ok = ok
        return ok

    def _device_nan_filter(self) -> bool:
        """HF's ``logging_nan_inf_filter`` tests every micro-batch's loss with a
        Python ``or`` on two device tensors -- a host synchronisation per
        micro-batch that drains the GPU queue (measured: ~9 % of the GPT-2 step
        idle).  The same substitution is done on the device instead: the flag
        is switched off for HF's loop and a non-finite loss is replaced by the
        running average HF would have added."""
        if getattr(self, "_dlion_nan_filter", None) is None:
            self._dlion_nan_filter = bool(self.args.logging_nan_inf_filter) and self.args.device.type == "cuda"
            if self._dlion_nan_filter:
                self.args.logging_nan_inf_filter = False
        return self._dlion_nan_filter

    def training_step(self, model, inputs, num_items_in_batch=None):
        loss = self._training_step(model, inputs, num_items_in_batch)
        tr = getattr(self, "_tr_loss", None)
        if self._device_nan_filter() and isinstance(tr, torch.Tensor) and tr.device == loss.device:
            avg = tr / (1 + self.state.global_step - self._globalstep_last_logged)
            loss = torch.where(torch.isfinite(loss), loss, avg.to(loss.dtype))
        return loss

    # ------------------------------------------------------ worker dropout (HF path)
    def _elastic(self):
        """With ``--lion_elastic_timeout`` on a multi-rank run, the process-wide
        :class:`ElasticGroup`: Lion's vote is guarded by it, and so are the
        collectives HF / accelerate issue on their own -- the per-step
        ``num_items_in_batch`` gather, the logging loss gather, evaluation
        gathers, accelerate's ``wait_for_everyone`` -- so a worker dying in
        the training loop leaves the survivors a regrouped default group
        instead of a hang (parallel/elastic.py).  Not guarded: barriers outside
        the loop -- ``main_process_first`` in the entrypoints' data
        preparation (before training starts) and HF's ``dist.barrier()`` for
        ``load_best_model_at_end`` -- a death there still waits for the
        backend's timeout."""
        t = getattr(self.args, "lion_elastic_timeout", None)
        if t is None or not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
            return None
        from ..parallel.elastic import ElasticGroup

        el = ElasticGroup.active()
        if el is None or getattr(self, "_dlion_elastic", None) is not el:
            el = ElasticGroup.get(t)
            self._dlion_elastic = el
            el.on_regroup(self._on_regroup)
            _install_guarded_gathers(self, el)
        return el

    def _on_regroup(self, el) -> None:
        """accelerate caches the world in its shared state: point it at the
        survivors (new default group, dense ranks)."""
        from accelerate.state import AcceleratorState, PartialState

        for shared in (PartialState._shared_state, AcceleratorState._shared_state):
            if "num_processes" in shared:
                shared["num_processes"] = el.world
            if "process_index" in shared:
                shared["process_index"] = el.rank
        self.state.is_world_process_zero = el.rank == 0
        # the dead rank's data shard is simply not consumed any more; the
        # survivors keep their own shards (BatchSamplerShard is per process)

    def compute_loss(self, model, inputs, *a, **kw):
        loss = super().compute_loss(model, inputs, *a, **kw)
        from ..parallel.elastic import fault_spec, inject

        if fault_spec():  # DLION_FAULT=rank:step:backward -- die inside autograd
            t = loss[0] if isinstance(loss, tuple) else loss
            if isinstance(t, torch.Tensor) and t.requires_grad:
                n = self.state.global_step
                t.register_hook(lambda g, n=n: inject("backward", n))
        return loss

    def _prepare_without_ddp(self) -> None:
        """Route accelerate's model preparation through its ``evaluation_mode``
        (device placement, mixed-precision forward, no DDP wrap) and replace
        DDP's constructor broadcast by ``broadcast_parameters``."""
        if getattr(self.args, "lion_ddp_wrap", False) or getattr(self, "_dlion_noddp", False):
            return
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
            return
        acc = self.accelerator
        orig = acc.prepare_model

        def prepare_model(model, device_placement=None, evaluation_mode=False):
            out = orig(model, device_placement=device_placement, evaluation_mode=True)
            if not evaluation_mode and not getattr(out, "_dlion_broadcast", False):
                from .engine import broadcast_parameters

                broadcast_parameters(out)
                out._dlion_broadcast = True
            return out

        acc.prepare_model = prepare_model
        self._dlion_noddp = True

    def train(self, *a, **kw):
        _share_gpus_if_oversubscribed(self.args)
        self._prepare_without_ddp()
        if getattr(self.args, "lion_elastic_timeout", None) is not None:
            # no forward-time buffer broadcast on DDP's (possibly stale) group;
            # buffers are deterministic and every rank builds them identically
            self.args.ddp_broadcast_buffers = False
            self._elastic()
        out = super().train(*a, **kw)
        elastic = getattr(self, "_dlion_elastic", None)
        # also when a regroup left a single survivor: world_end records the shrink
        if dist.is_available() and dist.is_initialized() and (dist.get_world_size() > 1 or elastic is not None):
            same = replicas_identical(self.model, self._elastic())
            rec = {"replicas_identical": float(same), "world_end": float(dist.get_world_size()),
                   "ddp_wrapped": float(isinstance(self.model_wrapped, torch.nn.parallel.DistributedDataParallel))}
            rec["trainable_params"] = float(sum(p.numel() for p in self.model.parameters() if p.requires_grad))
            if self.args.device.type == "cuda":
                rec["max_memory_allocated_mb"] = torch.cuda.max_memory_allocated(self.args.device) / 2**20
            self.log(rec)
        return out

    def _phase_timer(self):
        """HIP-event phase times of the step (fwd_bwd, clip, and Lion's encode /
        exchange / apply) for metrics.jsonl; ``DLION_PHASE_TIMES=0`` disables."""
        lion = _lion_of(self.optimizer)
        if lion is None or os.environ.get("DLION_PHASE_TIMES", "1") == "0":
            return None
        if lion.phase_timer is None:
            from ..utils.timing import PhaseTimer

            lion.phase_timer = PhaseTimer(self.args.device)
        return lion.phase_timer

    def _training_step(self, model, inputs, num_items_in_batch=None):
        from ..ops.linear import begin_fusion_window, end_fusion_window
        from ..utils.timing import phase_of

        fuse = self._engine_fusion(model)
        if fuse:
            begin_fusion_window(getattr(self, "current_gradient_accumulation_steps", None))
        try:
            with no_sync(model), phase_of(self._phase_timer(), "fwd_bwd"):
                loss = super().training_step(model, inputs, num_items_in_batch)
        except BaseException:
            if fuse:
                end_fusion_window(flush=False)
            raise
        if fuse and self.accelerator.sync_gradients:
            end_fusion_window()  # last micro-batch of the step: every gradient is in param.grad now
        if self.accelerator.sync_gradients:
            from ..ops.fused import check_index_errors

            check_index_errors()  # out-of-range ids / labels flagged by the kernels (no stall)
            t = self._phase_timer()
            if t is not None:
                t.step()
        return loss

    def _prepare_input(self, data):
        # HF copies each batch with a blocking .to(device): for pinned host
        # memory that is a memcpy plus a stream synchronize, i.e. the host
        # waits for the previous micro-batch's whole backward before it can
        # launch the next forward.  A pinned tensor can go asynchronously (the
        # caching host allocator keeps its buffer until the copy has run).
        if (isinstance(data, torch.Tensor) and data.device.type == "cpu" and data.is_pinned()
                and self.args.device.type == "cuda"):
            return data.to(self.args.device, non_blocking=True)
        return super()._prepare_input(data)

    def get_batch_samples(self, epoch_iterator, num_batches, device):
        # HF fetches the whole accumulation window's batches up front; their
        # uploads are issued here back to back (pinned, non-blocking) instead of
        # one per micro-batch between the previous backward and the next forward,
        # where each copy waited on the stream with the GPU idle (~0.25 ms per
        # micro-batch in the run_clm trace).
        batch_samples, n = super().get_batch_samples(epoch_iterator, num_batches, device)
        if getattr(self.args.device, "type", None) == "cuda":
            for b in batch_samples:
                if isinstance(b, dict):
                    for k, v in b.items():
                        if isinstance(v, torch.Tensor) and v.device.type == "cpu" and v.is_pinned():
                            b[k] = v.to(self.args.device, non_blocking=True)
        return batch_samples, n

    def _get_num_items_in_batch(self, batch_samples, device):
        # HF counts the label tokens on the host and ships the count with a
        # blocking .to(device) -- a stream synchronise at every optimizer step.
        # Same count, pinned + non-blocking copy; the cross-rank sum (HF's
        # average_tokens_across_devices) stays a device collective.
        if getattr(device, "type", None) != "cuda" or self.args.n_gpu > 1:
            # (n_gpu > 1: single-process DataParallel -- HF's own branch order and normaliser)
            return super()._get_num_items_in_batch(batch_samples, device)
        avg = self.args.average_tokens_across_devices and self.args.world_size > 1
        prev = self.args.average_tokens_across_devices
        self.args.average_tokens_across_devices = False
        try:
            n = super()._get_num_items_in_batch(batch_samples, torch.device("cpu"))
        finally:
            self.args.average_tokens_across_devices = prev
        if not torch.is_tensor(n):
            return n
        n = n.pin_memory().to(device, non_blocking=True)
        if avg:
            n = self.accelerator.gather(n).sum()
        return n

    def _clip_grad_norm(self, model):
        from ..utils.timing import phase_of

        with phase_of(self._phase_timer(), "clip"):
            return self._clip_grad_norm_impl(model)

    def _clip_grad_norm_impl(self, model):
        lion = _lion_of(self.optimizer)
        if lion is not None and self._engine_fusion(model):
            mine = {id(p) for g in lion.param_groups for p in g["params"]}
            inner = getattr(model, "module", model)
            if mine == {id(p) for p in inner.parameters() if p.requires_grad}:
                return lion.clip_grad_norm_(self.args.max_grad_norm)
        return super()._clip_grad_norm(model)

    def create_optimizer(self, model=None):
        if self.optimizer is None and getattr(self.args, "lion", False):
            target = model if model is not None else self.model
            self.optimizer = build_lion(target, self.args)
            return self.optimizer
        return super().create_optimizer(model) if model is not None else super().create_optimizer()

    # ------------------------------------------------ per-rank optimizer state
    @staticmethod
    def _rank_file(output_dir: str) -> Optional[str]:
        if not (dist.is_available() and dist.is_initialized()):
            return None
        return os.path.join(output_dir, f"rank{dist.get_rank()}-of-{dist.get_world_size()}-optimizer.pt")

    def _save_optimizer_and_scheduler(self, output_dir):
        super()._save_optimizer_and_scheduler(output_dir)
        path = self._rank_file(output_dir)
        if path is not None and self.optimizer is not None:
            os.makedirs(output_dir, exist_ok=True)
            torch.save(self.optimizer.state_dict(), path)

    def _load_optimizer_and_scheduler(self, checkpoint):
        if checkpoint is None:
            return
        if self.args.device.type == "cpu" and self.args.world_size > 1:
            # HF maps to args.device ("cpu:0") in multi-process CPU runs, which
            # torch.load cannot restore; load on "cpu" instead
            opt_f, sch_f = os.path.join(checkpoint, "optimizer.pt"), os.path.join(checkpoint, "scheduler.pt")
            if os.path.isfile(opt_f) and os.path.isfile(sch_f):
                self.optimizer.load_state_dict(torch.load(opt_f, map_location="cpu", weights_only=True))
                self.lr_scheduler.load_state_dict(torch.load(sch_f, weights_only=True))
        else:
            super()._load_optimizer_and_scheduler(checkpoint)
        path = self._rank_file(checkpoint)
        if path is not None and os.path.isfile(path) and self.optimizer is not None:
            # optimizer.load_state_dict moves the state onto each parameter's device
            state = torch.load(path, map_location="cpu", weights_only=True)
            self.optimizer.load_state_dict(state)
            logger.info("restored per-rank optimizer state from %s", path)


def _share_gpus_if_oversubscribed(args) -> None:
    """More ranks than GPUs (rehearsals: W gloo ranks on one MI355X): accelerate
    places rank r on cuda:(r mod #GPUs) but builds DDP with device_ids=[r],
    which moves rank r's inputs to a device that does not exist.  Without
    device_ids DDP uses the module's device."""
    if not torch.cuda.is_available() or getattr(args, "world_size", 1) <= 1:
        return
    if getattr(args, "local_process_index", 0) >= torch.cuda.device_count():
        os.environ["ACCELERATE_BYPASS_DEVICE_MAP"] = "true"


def param_digest(model: torch.nn.Module, chunk: int = 1 << 24) -> torch.Tensor:
    """Order-dependent digest of every parameter's raw bits, computed ON the
    parameters' device (a 2-element int64 tensor).  Per tensor: the sum and the
    sum of squares of the bit patterns (integer view, int64 arithmetic,
    wrapping), mixed with the tensor's position.  Chunked, so the int64
    temporaries stay <= 128 MB even for 8B-parameter replicas (the host
    SHA-256 it replaces copied every parameter to the host as fp32: ~32 GB
    per rank at Llama-3-8B)."""
    inner = getattr(model, "module", model)
    acc = None
    for i, p in enumerate(inner.parameters()):
        x = p.detach().reshape(-1)
        x = x.view(torch.int16) if x.element_size() == 2 else (x.view(torch.int32) if x.element_size() == 4 else
                                                               x.view(torch.int64) if x.element_size() == 8 else
                                                               x.view(torch.uint8))
        s = torch.zeros(2, dtype=torch.int64, device=x.device)
        for c in range(0, x.numel(), chunk):
            v = x[c:c + chunk].to(torch.int64)
            s[0] += v.sum()
            s[1] += (v * v).sum()
        s = s * (2 * i + 1) + i
        acc = s if acc is None else acc * 31 + s
    return acc if acc is not None else torch.zeros(2, dtype=torch.int64)


def replicas_identical(model: torch.nn.Module, elastic=None) -> bool:
    """Do all ranks hold bit-identical parameters?  (:func:`param_digest` per
    rank, gathered -- guarded when ``elastic`` is given)."""
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    d = param_digest(model).to(dev)
    if elastic is not None:
        allv = elastic.all_gather(d)
    else:
        parts = [torch.empty_like(d) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, d)
        allv = torch.cat(parts)
    rows = allv.reshape(-1, 2).tolist()
    return all(r == rows[0] for r in rows)


def _install_guarded_gathers(trainer, el) -> None:
    """Route HF's own collectives through ``el``: ``transformers.trainer.nested_gather``
    (the logging loss gather) and this trainer's ``accelerator.gather`` (the
    ``num_items_in_batch`` sum, ``gather_for_metrics`` in evaluation)."""
    import transformers.trainer as hf_trainer
    from accelerate.utils import recursively_apply

    def gather_one(t):
        return el.all_gather(t.reshape(1) if t.dim() == 0 else t)

    def guarded_gather(tensor):
        return recursively_apply(gather_one, tensor, error_on_other_type=True)

    def guarded_nested_gather(tensors, parallel_mode=None, name=None):
        if tensors is None:
            return None
        return recursively_apply(gather_one, tensors, error_on_other_type=True)

    trainer.accelerator.gather = guarded_gather
    hf_trainer.nested_gather = guarded_nested_gather
    # accelerate's barrier (save_model / checkpoint paths) through the guard too
    trainer.accelerator.wait_for_everyone = el.barrier


class RankShardedLoaderMixin:
    """Training sets that shard themselves per rank (``rank_sharded``: the
    SFT :class:`~..utils.data.PackedStream`, run_clm's ``--streaming``
    :class:`~..utils.data.CLMStream`) get a plain DataLoader instead of
    accelerate's: accelerate would either read the stream on rank 0 and
    broadcast every batch (``dispatch_batches``, the reference's path for
    iterable data) or wrap it in an ``IterableDatasetShard`` that drops
    (W-1)/W of the already-sharded batches.  Batches are moved to the device by
    ``_prepare_inputs``."""

    def train(self, *a, **kw):
        _share_gpus_if_oversubscribed(self.args)
        return super().train(*a, **kw)

    def get_train_dataloader(self):
        ds = self.train_dataset
        if getattr(ds, "rank_sharded", False):
            from torch.utils.data import DataLoader

            return DataLoader(ds, batch_size=self._train_batch_size, collate_fn=self.data_collator,
                              num_workers=0, pin_memory=self.args.dataloader_pin_memory)
        return super().get_train_dataloader()


class AsyncTrainer(AsyncMixin, RankShardedLoaderMixin, Trainer):
    """HF Trainer without gradient all-reduce (reference async_trainer.py:8-34)."""


class LocalTrainer(RankShardedLoaderMixin, Trainer):
    """Stock HF Trainer (DDP gradient all-reduce, the reference's path without
    ``--async_grad``) that also takes rank-sharded streams."""


def warn_unsynced(args) -> None:
    """--async_grad without --lion leaves the replicas with no sync at all (D16)."""
    if getattr(args, "async_grad", False) and not getattr(args, "lion", False):
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            logger.warning("--async_grad without --lion: gradients are never synchronised and the replicas "
                           "will diverge (the reference silently does this, SURVEY D16)")
