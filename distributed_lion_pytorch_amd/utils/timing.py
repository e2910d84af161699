"""HIP-event phase timers for the training step (no HF import: the optimizer
uses them on its hot path)."""
from __future__ import annotations

import time
from collections import defaultdict
from contextlib import contextmanager, nullcontext
from typing import Dict, Optional

import torch


class PhaseTimer:
    """Per-phase time of the training step, summed per phase name.

    On a GPU each phase is a pair of HIP events recorded on the current
    (compute) stream, so nothing synchronises the host until :meth:`summary`;
    a phase's time is what the compute stream spent between the two events,
    i.e. for the vote exchange the *exposed* communication (the stream waits
    on the RCCL stream) plus the shard-vote kernel.  On the CPU the phases are
    wall-clock intervals.  Phases may repeat (once per bucket / micro-batch);
    their times add up.  ``count`` tells how many optimizer steps the sums
    span (:meth:`step`), so :meth:`summary` can report per-step means."""

    def __init__(self, device=None, enabled: bool = True):
        dev = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self.device = dev
        self.enabled = enabled
        self.cuda = dev.type == "cuda"
        self._events = defaultdict(list)
        self._wall = defaultdict(float)
        self.count = 0

    @contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        if self.cuda:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            try:
                yield
            finally:
                e.record()
                self._events[name].append((s, e))
        else:
            t0 = time.perf_counter()
            try:
                yield
            finally:
                self._wall[name] += 1000.0 * (time.perf_counter() - t0)

    # event pairs kept before step() folds them into host sums: a timer that
    # nobody drains (library use of the HF path without the metrics callback)
    # must not grow without bound over a long run
    MAX_PENDING = 4096

    def step(self) -> None:
        self.count += 1
        if self.cuda and sum(len(v) for v in self._events.values()) > self.MAX_PENDING:
            self._fold()

    def _fold(self) -> None:
        """Move the event pairs whose end event has completed into the
        millisecond sums -- no device synchronisation on the training path
        (``query()`` only asks); pairs still in flight stay pending.  Events
        complete in stream order, so the completed pairs are a prefix of each
        list."""
        for k, v in self._events.items():
            done = 0
            while done < len(v) and v[done][1].query():
                done += 1
            if done:
                self._wall[k] += sum(s.elapsed_time(e) for s, e in v[:done])
                del v[:done]

    def totals_ms(self) -> Dict[str, float]:
        """Summed milliseconds per phase (synchronises the device)."""
        if self.cuda and self._events:
            torch.cuda.synchronize(self.device)
        out = dict(self._wall)
        for k, v in self._events.items():
            out[k] = out.get(k, 0.0) + sum(s.elapsed_time(e) for s, e in v)
        return out

    def summary(self, reset: bool = True) -> Dict[str, float]:
        """Per-step mean milliseconds per phase (sums when no step was counted)."""
        if not self.enabled:
            return {}
        n = max(1, self.count)
        out = {k: v / n for k, v in self.totals_ms().items()}
        if reset:
            self.reset()
        return out

    def reset(self) -> None:
        self._events.clear()
        self._wall.clear()
        self.count = 0


def phase_of(timer: Optional[PhaseTimer], name: str):
    """``timer.phase(name)``, or a no-op context when there is no timer."""
    return timer.phase(name) if timer is not None else nullcontext()
