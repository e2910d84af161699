"""Vote-exchange strategies over torch.distributed (RCCL on ROCm, gloo on CPU).

All strategies move the packed 1-bit sign planes produced by the encode
kernel; they differ in the collective pattern:

``allgather``  (wire "1bit_allgather")
    one ``all_gather_into_tensor`` per bucket; each rank receives the W planes
    and votes locally.  Receive bytes/rank: (W-1)·N/8.  Supports the paper's
    *average* server rule, since every rank sees every vote.
``a2a``  (wire "1bit_a2a", "vote-RS/AG")
    ``all_to_all_single`` sends shard j of the plane to rank j (all 7 xGMI
    links busy at once instead of one ring neighbour), each rank votes its
    shard (K4 kernel), then ``all_gather_into_tensor`` of the 1-bit result.
    Bytes/rank: 2(W-1)/W·N/8 -- 16x fewer than a bf16 ring all-reduce at W=8.
``ref_int64``  (reference wire format, A/B only)
    one blocking ``all_gather`` per *parameter tensor* with the packed bytes
    widened to int64, i.e. the reference's 1 byte/param and 148/291 calls per
    step (/root/reference/distributed_lion.py:76-81).

Every strategy is split into ``launch`` (issue async collectives right after
the bucket is encoded), ``advance`` (second phase for a2a) and ``finish``
(wait; return what the apply kernel consumes).  Collectives are async: on
RCCL they run on the process group's own HIP stream and overlap with the
encode of the next bucket on the compute stream.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from ..ops import reference as ref
from ..optim.plan import Bucket, FlatPlan

STRATEGIES = ("allgather", "a2a", "ref_int64")
_ALIASES = {"1bit_allgather": "allgather", "1bit_a2a": "a2a", "vote_rs_ag": "a2a", "ref": "ref_int64"}


def canonical_strategy(name: str) -> str:
    name = _ALIASES.get(name, name)
    if name not in STRATEGIES:
        raise ValueError(f"unknown vote exchange {name!r}; choose from {STRATEGIES}")
    return name


@dataclass
class ApplyArgs:
    planes: torch.Tensor
    stride: int
    mode: int  # VOTE_* code for the apply kernel
    neg: Optional[torch.Tensor] = None


class WireCounter:
    """Bytes this rank puts on / takes off the wire (payload only).  An
    all-gather delivers this rank's contribution to each of the W-1 peers, so
    it counts (W-1) x contribution sent -- ring or direct, the same bytes leave
    the rank -- and sent == recv for every collective used here."""

    def __init__(self):
        self.sent = 0
        self.recv = 0
        self.calls = 0

    def add(self, sent: int, recv: int, calls: int = 1):
        self.sent += int(sent)
        self.recv += int(recv)
        self.calls += calls

    def snapshot(self) -> dict:
        return {"wire_bytes_sent": self.sent, "wire_bytes_recv": self.recv, "collectives": self.calls}

    def reset(self):
        self.sent = self.recv = self.calls = 0


class VoteExchange:
    def __init__(self, plan: FlatPlan, group, rank: int, world: int, executor, tie: int, mode: int,
                 send: Optional[torch.Tensor] = None):
        self.plan, self.group, self.rank, self.world = plan, group, rank, world
        self.executor = executor
        self.tie, self.mode = tie, mode
        self.wire = WireCounter()
        self.ties: Optional[torch.Tensor] = None  # int64 tie counter (telemetry), set by the optimizer
        # ``send``: reuse already-encoded planes (the elastic re-vote after a regroup)
        self.send = send if send is not None else torch.zeros(plan.total_bytes, dtype=torch.uint8,
                                                              device=plan.device)

    def send_view(self, b: Bucket) -> torch.Tensor:
        return self.send[b.byte_off:b.byte_off + b.nbytes]

    # overridden ---------------------------------------------------------
    def launch(self, b: Bucket, alive: torch.Tensor):
        raise NotImplementedError

    def advance(self, b: Bucket, state, alive: torch.Tensor):
        return state

    def finish(self, b: Bucket, state, alive: torch.Tensor) -> ApplyArgs:
        raise NotImplementedError


class AllGatherExchange(VoteExchange):
    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.recv = torch.zeros(self.world * self.plan.total_bytes, dtype=torch.uint8, device=self.plan.device)

    def recv_view(self, b: Bucket) -> torch.Tensor:
        o = self.world * b.byte_off
        return self.recv[o:o + self.world * b.nbytes]

    def launch(self, b, alive):
        out = self.recv_view(b)
        work = dist.all_gather_into_tensor(out, self.send_view(b), group=self.group, async_op=True)
        self.wire.add((self.world - 1) * b.nbytes, (self.world - 1) * b.nbytes)
        return work

    def finish(self, b, work, alive):
        if work is not None:
            work.wait()
        return ApplyArgs(planes=self.recv_view(b), stride=b.nbytes, mode=self.mode)


class AllToAllExchange(VoteExchange):
    """vote-RS/AG: shard-wise vote after an all-to-all, then 1-bit all-gather."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        if self.mode == ref.VOTE_AVERAGE:
            raise ValueError("average voting needs every vote on every rank; use exchange='allgather'")
        dev, tb = self.plan.device, self.plan.total_bytes
        self.need_neg = self.tie == ref.TIE_ZERO
        self.recv = torch.zeros(tb, dtype=torch.uint8, device=dev)
        self.voted = torch.zeros(tb, dtype=torch.uint8, device=dev)
        self.shard_pos = torch.zeros(tb // self.world, dtype=torch.uint8, device=dev)
        if self.need_neg:
            self.voted_neg = torch.zeros(tb, dtype=torch.uint8, device=dev)
            self.shard_neg = torch.zeros(tb // self.world, dtype=torch.uint8, device=dev)

    def _v(self, buf, b, scale=1):
        o = b.byte_off // scale
        return buf[o:o + b.nbytes // scale]

    def launch(self, b, alive):
        out = self._v(self.recv, b)
        work = dist.all_to_all_single(out, self.send_view(b), group=self.group, async_op=True)
        shard = b.nbytes // self.world
        self.wire.add((self.world - 1) * shard, (self.world - 1) * shard)
        return work

    def advance(self, b, work, alive):
        work.wait()
        shard = b.nbytes // self.world
        pos = self._v(self.shard_pos, b, self.world)
        neg = self._v(self.shard_neg, b, self.world) if self.need_neg else None
        self.executor.vote_reduce(self._v(self.recv, b), shard, alive, self.tie, pos, neg, self.ties)
        works = [dist.all_gather_into_tensor(self._v(self.voted, b), pos, group=self.group, async_op=True)]
        if self.need_neg:
            works.append(dist.all_gather_into_tensor(self._v(self.voted_neg, b), neg, group=self.group,
                                                     async_op=True))
        n = len(works)
        self.wire.add(n * (self.world - 1) * shard, n * (self.world - 1) * shard, calls=n)
        return works

    def finish(self, b, works, alive):
        for w in works:
            w.wait()
        neg = self._v(self.voted_neg, b) if self.need_neg else None
        return ApplyArgs(planes=self._v(self.voted, b), stride=b.nbytes, mode=ref.VOTE_PREVOTED, neg=neg)


class RefInt64Exchange(AllGatherExchange):
    """Reference wire pattern: per-tensor blocking all_gather of int64 bytes."""

    def launch(self, b, alive):
        out = self.recv_view(b).view(self.world, b.nbytes)
        send = self.send_view(b)
        for s in b.segments:
            o = s.bit_off // 8
            nb = (s.numel + 7) // 8
            wide = send[o:o + nb].to(torch.int64).view(1, nb)
            bufs = [torch.empty_like(wide) for _ in range(self.world)]
            dist.all_gather(bufs, wide, group=self.group)
            for r, t in enumerate(bufs):
                out[r, o:o + nb] = t.view(-1).to(torch.uint8)
            self.wire.add(8 * nb * (self.world - 1), 8 * nb * (self.world - 1))
        return None

    def finish(self, b, _, alive):
        return ApplyArgs(planes=self.recv_view(b), stride=b.nbytes, mode=self.mode)


def make_exchange(strategy: str, plan: FlatPlan, group, rank: int, world: int, executor, tie: int,
                  mode: int) -> VoteExchange:
    strategy = canonical_strategy(strategy)
    cls = {"allgather": AllGatherExchange, "a2a": AllToAllExchange, "ref_int64": RefInt64Exchange}[strategy]
    if strategy == "a2a" and mode == ref.VOTE_AVERAGE:
        cls = AllGatherExchange
    return cls(plan, group, rank, world, executor, tie, mode)


def wire_bytes_per_step(numel: int, world: int, strategy: str) -> int:
    """Analytic per-rank receive bytes for reporting."""
    strategy = canonical_strategy(strategy)
    nb = (numel + 7) // 8
    if world <= 1:
        return 0
    if strategy == "allgather":
        return (world - 1) * nb
    if strategy == "a2a":
        return 2 * (world - 1) * nb // world
    return (world - 1) * numel  # ref int64: 1 byte per param per peer


