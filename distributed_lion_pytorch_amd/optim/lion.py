"""Distributed Lion optimizer (majority-vote sign aggregation), MI355X-native.

API-compatible with the reference ``Lion`` (/root/reference/distributed_lion.py:140-200):

    Lion(params, lr=1e-4, betas=(0.9, 0.99), weight_decay=0.0, max_grad_norm=None)

with the same ``state_dict`` schema (``state[p] == {'exp_avg': Tensor}`` in the
parameter dtype; group keys ``lr``, ``betas``, ``weight_decay``) and the same
update semantics, but a different execution model:

* one fused gfx950 kernel per *bucket* instead of ~20+6W ATen ops per tensor;
* the sign votes travel as true 1-bit planes in a few large collectives
  (``exchange=`` ``"allgather"`` | ``"a2a"`` | ``"ref_int64"``) instead of one
  int64 ``all_gather`` per tensor;
* the world size is resolved at every step (no stale dispatch) and
  defects D2-D5 of the reference are fixed.

Keyword-only extensions (all optional):
  vote         "majority" (reference) | "average" (paper's server averaging)
  tie_break    "negative" (reference parity) | "zero" | "positive"
  exchange     vote exchange strategy, see parallel/exchange.py
  bucket_mb    packed-bit bucket size (MB) -- one collective per bucket
  group        torch.distributed process group (default: WORLD)
  backend      "auto" | "hip" | "torch"
  seed         base seed of the stochastic-binarization RNG
  telemetry    collect vote-agreement counts (see :meth:`stats`)
  elastic_timeout  seconds; enables real worker-dropout handling: a heartbeat
               before each step's vote detects dead ranks and the survivors
               continue in a shrunken group (parallel/elastic.py)
"""
from __future__ import annotations

import hashlib
from typing import Callable, Dict, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
from torch.optim.optimizer import Optimizer

from ..ops import reference as ref
from ..ops.linear import bump_weight_generation
from ..parallel.exchange import canonical_strategy, make_exchange, wire_bytes_per_step
from ..utils.timing import phase_of
from .executors import HParams, make_executor
from .plan import FlatPlan

# reference-compatible functional API re-exported from the oracle
update_fn = ref.update_fn
update_fn_distributed = ref.update_fn_distributed
update_fn_distributed_stoc = ref.update_fn_distributed_stoc
majority_vote = ref.majority_vote
flatten_and_pad = ref.flatten_and_pad
restore_flattened_tensor = ref.restore_flattened_tensor
exists = ref.exists


class Lion(Optimizer):
    def __init__(
        self,
        params,
        lr: float = 1e-4,
        betas: Tuple[float, float] = (0.9, 0.99),
        weight_decay: float = 0.0,
        max_grad_norm: Optional[float] = None,
        *,
        vote: str = "majority",
        tie_break: str = "negative",
        exchange: str = "a2a",
        bucket_mb: float = 32.0,
        group=None,
        backend: str = "auto",
        seed: int = 0,
        telemetry: bool = False,
        verify_consistency: bool = True,
        elastic_timeout: Optional[float] = None,
    ):
        if not lr > 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not all(0.0 <= b <= 1.0 for b in betas):
            raise ValueError(f"Invalid betas: {betas}")
        if max_grad_norm is not None and not max_grad_norm > 0:
            raise ValueError(f"Invalid max_grad_norm: {max_grad_norm}")
        if vote not in ref.VOTE_CODES:
            raise ValueError(f"vote must be one of {tuple(ref.VOTE_CODES)}")
        if tie_break not in ref.TIE_CODES:
            raise ValueError(f"tie_break must be one of {tuple(ref.TIE_CODES)}")
        defaults = dict(lr=lr, betas=betas, weight_decay=weight_decay)
        super().__init__(params, defaults)
        # stored (reference D2: it never was) but, like the reference, not part of state_dict
        self.max_grad_norm = max_grad_norm
        self.vote = vote
        self.tie_break = tie_break
        self.exchange_name = canonical_strategy(exchange)
        self.bucket_bytes = int(bucket_mb * (1 << 20))
        self.process_group = group
        self.backend = backend
        self.seed = int(seed)
        self.telemetry = telemetry
        self.verify_consistency = verify_consistency
        self._n_steps = 0
        self._plan: Optional[FlatPlan] = None
        self._executor = None
        self._exchange = None
        self._alive_host: Optional[Tuple[bool, ...]] = None
        self._alive_dev: Optional[torch.Tensor] = None
        self._dropped: set = set()
        self._dropout_schedule: Dict[int, Sequence[int]] = {}
        self._agree: Optional[torch.Tensor] = None
        self._agree_total = 0
        self.last_world = 1
        self.elastic_timeout = elastic_timeout
        self._elastic = None
        # optional utils.metrics.PhaseTimer: encode / exchange / apply (local_update at W=1)
        self.phase_timer = None
        # run the vote path (encode -> collectives -> apply) even on a 1-rank
        # group: exercises the RCCL calls on a single GPU (tests/test_nccl_gpu.py)
        self._force_vote = False

    # ------------------------------------------------------------ topology
    def _world(self):
        """(world, rank) resolved now -- never cached."""
        if not (dist.is_available() and dist.is_initialized()):
            return 1, 0
        g = self.process_group
        return dist.get_world_size(g), dist.get_rank(g)

    # ------------------------------------------------------ worker dropout
    def drop_workers(self, ranks: Sequence[int]) -> None:
        """Exclude ``ranks`` from every subsequent vote (simulated dropout /
        abstention).  Must be called identically on every rank; the dropped
        ranks keep running the collective so nothing hangs, but their planes
        are ignored and the majority is taken over the live voters only."""
        self._dropped |= {int(r) for r in ranks}

    def restore_workers(self, ranks: Optional[Sequence[int]] = None) -> None:
        if ranks is None:
            self._dropped.clear()
        else:
            self._dropped -= {int(r) for r in ranks}

    def set_dropout_schedule(self, schedule: Dict[int, Sequence[int]]) -> None:
        """{step: [ranks to drop from that optimizer step on]} (fault injection)."""
        self._dropout_schedule = {int(k): list(v) for k, v in schedule.items()}

    def _alive(self, world: int, device) -> torch.Tensor:
        if self._n_steps in self._dropout_schedule:
            self.drop_workers(self._dropout_schedule[self._n_steps])
        host = tuple(r not in self._dropped for r in range(world))
        if not any(host):
            # with no live voter the exchanges would disagree (allgather: delta 0,
            # a2a without a negative plane: delta -1), so this is refused outright
            raise ValueError(f"every worker of the {world}-rank vote is dropped ({sorted(self._dropped)}); "
                             "at least one rank must keep voting")
        if self._alive_dev is None or host != self._alive_host or self._alive_dev.device != device:
            t = torch.tensor([1 if a else 0 for a in host], dtype=torch.uint8)
            self._alive_dev = t.to(device)
            self._alive_host = host
        return self._alive_dev

    def _elastic_check(self) -> None:
        """Real dropout: heartbeat before the vote; on a drop, switch to the
        survivors' group (the plan is rebuilt below because the world changed)."""
        if self.elastic_timeout is None or not (dist.is_available() and dist.is_initialized()):
            return
        if self._elastic is None:
            from ..parallel.elastic import ElasticMembership

            self._elastic = ElasticMembership(self.elastic_timeout, group=self.process_group)
        grp = self._elastic.check(self._n_steps)
        if grp is not None:
            self.process_group = grp
            self._dropped.clear()  # simulated-dropout ranks were numbered in the old group
            self._alive_dev = None

    # --------------------------------------------------------------- plan
    def _get_plan(self, entries, world: int, rank: int):
        key = (FlatPlan.make_key(entries), world, self.exchange_name)
        if self._plan is not None and getattr(self._plan, "_full_key", None) == key:
            return self._plan
        plan = FlatPlan(entries, world=world, bucket_bytes=self.bucket_bytes)
        plan._full_key = key
        self._plan = plan
        self._executor = make_executor(plan, self.backend)
        if world > 1 or self._force_vote:
            if self.verify_consistency:
                self._check_consistency(plan)
            self._exchange = make_exchange(self.exchange_name, plan, self.process_group, rank, world,
                                           self._executor, ref.TIE_CODES[self.tie_break],
                                           ref.VOTE_CODES[self.vote])
        else:
            self._exchange = None
        return plan

    def _check_consistency(self, plan: FlatPlan) -> None:
        """All ranks must vote on the same tensors in the same order, or the
        collectives silently mismatch.  One tiny all-reduce per
        new plan compares a digest of the layout."""
        h = hashlib.sha256()
        for s in plan.segments:
            h.update(f"{s.numel}:{s.param.dtype}:{s.bit_off};".encode())
        for b in plan.buckets:
            h.update(f"B{b.nbytes}:{b.group};".encode())
        v = int.from_bytes(h.digest()[:7], "little")
        dev = plan.device if dist.get_backend(self.process_group) == "nccl" else torch.device("cpu")
        t = torch.tensor([v, -v], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.process_group)
        if int(t[0]) != v or int(t[1]) != -v:
            raise RuntimeError(
                "dlion Lion: parameter/gradient layout differs across ranks (different params have grads?); "
                "the vote collectives would mismatch")

    # --------------------------------------------------------------- step
    def _collect(self):
        entries, grads, moms = [], [], []
        for gi, group in enumerate(self.param_groups):
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("Lion does not support sparse gradients")
                state = self.state[p]
                if len(state) == 0:
                    state["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                entries.append((p, gi))
                grads.append(g)
                moms.append(state["exp_avg"])
        return entries, grads, moms

    @torch.no_grad()
    def clip_grad_norm_(self, max_norm: float) -> torch.Tensor:
        """Fused ``torch.nn.utils.clip_grad_norm_(params, max_norm)`` (L2) over
        this optimizer's gradients.  On the HIP path the norm is one read of
        every gradient through the update kernels' pointer table, the clip
        coefficient stays on the device (no host sync) and the NEXT ``step()``
        applies ``g * coef`` (rounded to the gradient dtype, exactly what the
        in-place ``_foreach_mul_`` would have stored) inside its kernels --
        instead of a separate read+write pass over all gradients (measured on
        Llama-3-8B: 19.5 ms of foreach norm+mul per step).  The coefficient is
        computed in fp32 (torch computes bf16 gradients' norms in bf16).  The
        gradients themselves are left unscaled; call ``step()`` next.
        Returns the total norm (0-dim device tensor)."""
        entries, grads, moms = self._collect()
        if not entries:
            return torch.zeros(())
        world, rank = self._world()
        plan = self._get_plan(entries, world, rank)
        ex = self._executor
        if ex.name != "hip":
            self._pending_gscale = None
            return torch.nn.utils.clip_grad_norm_([p for p, _ in entries], max_norm)
        meta = plan.meta(grads, moms)
        n = plan.total_chunks
        if getattr(self, "_clip_part", None) is None or self._clip_part.numel() < n or \
                self._clip_part.device != plan.device:
            self._clip_part = torch.empty(n, dtype=torch.float32, device=plan.device)
            self._clip_out = torch.empty(2, dtype=torch.float32, device=plan.device)
        for b in plan.buckets:
            ex.grad_sumsq(meta, b, self._clip_part)
        ex.clip_coef(self._clip_part, n, float(max_norm), self._clip_out)
        self._pending_gscale = self._clip_out
        return self._clip_out[0]

    @torch.no_grad()
    def step(self, closure: Optional[Callable] = None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()

        entries, grads, moms = self._collect()
        if not entries:
            return loss

        self._elastic_check()
        world, rank = self._world()
        self.last_world = world
        plan = self._get_plan(entries, world, rank)
        ex = self._executor
        meta = plan.meta(grads, moms) if ex.name == "hip" else None
        hps = [HParams(lr=g["lr"], wd=g["weight_decay"], beta1=g["betas"][0], beta2=g["betas"][1])
               for g in self.param_groups]

        gscale, self._pending_gscale = getattr(self, "_pending_gscale", None), None
        if world == 1 and not self._force_vote:
            with phase_of(self.phase_timer, "local_update"):
                for b in plan.buckets:
                    ex.local(meta, b, hps[b.group], grads=grads, moms=moms, gscale=gscale)
        else:
            self._distributed_step(plan, ex, meta, hps, grads, moms, world, rank, gscale)
        # the kernels wrote the weights through raw pointers (no autograd
        # version bump): invalidate derived per-step weight copies
        bump_weight_generation()
        self._n_steps += 1
        return loss

    def _distributed_step(self, plan, ex, meta, hps, grads, moms, world, rank, gscale=None):
        xch = self._exchange
        alive = self._alive(world, plan.device)
        stochastic = self.max_grad_norm is not None
        if self.telemetry and self._agree is None:
            self._agree = torch.zeros(1, dtype=torch.int64, device=plan.device)
        seed = (self.seed * 0x9E3779B1 + rank * 0x632BE59BD9B4E019 + 1) & 0x7FFFFFFFFFFFFFFF
        t = self.phase_timer
        states = []
        for b in plan.buckets:  # encode bucket i, then its collective overlaps encode of i+1
            hp = hps[b.group]
            rr = (1.0 + 1.0 / hp.beta1) * self.max_grad_norm if stochastic else 0.0
            with phase_of(t, "encode"):
                ex.encode(meta, b, xch.send_view(b), hp, update_m=True, stochastic=stochastic, rr=rr, seed=seed,
                          step=self._n_steps, grads=grads, moms=moms, gscale=gscale)
                states.append(xch.launch(b, alive))
        with phase_of(t, "exchange"):
            states = [xch.advance(b, s, alive) for b, s in zip(plan.buckets, states)]
        for b, s in zip(plan.buckets, states):
            with phase_of(t, "exchange"):
                a = xch.finish(b, s, alive)
            with phase_of(t, "apply"):
                ex.apply(meta, b, a.planes, a.stride, alive, a.mode, ref.TIE_CODES[self.tie_break], a.neg,
                         hps[b.group], own=xch.send_view(b) if self.telemetry else None,
                         agree=self._agree if self.telemetry else None)

    # ---------------------------------------------------------- telemetry
    def stats(self, reset: bool = True) -> dict:
        """Wire counters and (telemetry=True) vote agreement since last reset.
        Reading the agreement count synchronises with the device."""
        out = {"world": self.last_world, "exchange": self.exchange_name, "steps": self._n_steps}
        if self._exchange is not None:
            out.update(self._exchange.wire.snapshot())
            if reset:
                self._exchange.wire.reset()
        if self._plan is not None:
            out["numel"] = sum(s.numel for s in self._plan.segments)
            out["n_buckets"] = len(self._plan.buckets)
            out["wire_bytes_analytic"] = wire_bytes_per_step(out["numel"], self.last_world, self.exchange_name)
        if self._elastic is not None:
            out["live_ranks"] = list(self._elastic.members)
            out["dropout_events"] = list(self._elastic.events)
        if self._agree is not None:
            out["vote_agree"] = int(self._agree.item())
            if reset:
                self._agree.zero_()
        return out

    @property
    def plan(self) -> Optional[FlatPlan]:
        return self._plan
