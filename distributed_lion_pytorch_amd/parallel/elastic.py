"""Worker dropout at any instant: bounded-time collectives, a store-arbitrated
commit per collective, and regrouping of the survivors into a fresh default
process group.

The reference claims robustness to worker drop-out (/root/reference/README.md:2)
but its blocking per-tensor ``dist.all_gather`` (distributed_lion.py:81) hangs
every survivor until the c10d watchdog kills the job.  Majority
vote over the *live* voters is still a valid Distributed Lion step, so a dead
worker only has to be detected and cut out -- wherever it died: in backward,
between the launch of the vote all-to-all and its completion, inside the
1-bit all-gather, or between steps.

Protocol (all ranks run the same sequence of *guarded* collectives):

1. **Bounded wait.**  A guarded collective is issued asynchronously and its
   works are polled on the host (``is_completed``) against a deadline of
   ``timeout_s``.  Nothing on the compute stream ever waits on a work that has
   not completed, so a collective stuck on a dead peer can be abandoned (gloo
   reports a closed peer at once; RCCL kernels spin until aborted).
2. **Commit.**  Completing locally does not mean every peer completed (a ring
   or all-to-all can finish on some ranks only).  So no rank *uses* a result
   before the rendezvous store -- which outlives the workers: torchrun's agent
   or :mod:`..launch` hosts it -- has recorded the outcome: each rank adds
   itself to ``<gen>/<seq>/ok`` or proposes ``fail``; the last of the W adders
   writes ``all``.  ``compare_set`` makes the first written decision final, so
   every survivor acts on the same outcome (apply the step, or regroup).
3. **Membership.**  After a ``fail`` every live rank checks in under
   ``<gen>/members``; once every member has checked in or is known dead (the
   launcher posts a death notice when a rank's process exits with an error),
   or after ``grace_s``, the first proposal of the ranks seen is the new
   member list for everybody.  Death notices also end the bounded wait of
   step 1 and the commit wait of step 2 at once.  A rank left out (it was only late)
   raises :class:`WorkerExcluded`.
4. **Regroup.**  Every process group of the process is aborted
   (``ncclCommAbort`` under RCCL -- it stops the spinning kernels; gloo's abort
   runs off-thread because it waits for a hung, not dead, peer) and the
   survivors initialise a *new default* group over the same store with dense
   ranks.  Everything that resolves the group at call time -- Lion, HF /
   accelerate collectives (their cached process counts are updated by a
   listener, trainer/async_trainer.py) -- then runs on the survivors.  The
   failed collective is re-issued on the new group; Lion re-votes the step
   from its intact encoded sign planes (optim/lion.py).

Cost while nobody fails: one host wait for the collective plus three store
round trips per guarded collective (one per optimizer step); measured in
profiles/stress.  A rank's identity across regroups is its *original* global
rank (``ElasticGroup.me``).
"""
from __future__ import annotations

import atexit
import datetime
import json
import logging
import os
import threading
import time
from typing import Callable, List, Optional

import torch
import torch.distributed as dist

log = logging.getLogger(__name__)

DEFAULT_GRACE_S = 5.0
DECISION_WAIT_S = 0.25  # slice of the blocking decision read between death-notice checks
GLOO_DRAIN_S = 2.0  # after a failure signal: time gloo works get to fail on their own before being abandoned
DEATH_KEY = "dlion/dead"  # + "/<rank>", in the root rendezvous store (written by ..launch)
DEATH_COUNT_KEY = "dlion/dead_count"


class WorkerExcluded(RuntimeError):
    """This rank was voted out of the group (it checked in after the deadline)."""


def _default_store():
    from torch.distributed import distributed_c10d as c10d

    return c10d._get_default_store()


_GRAVEYARD: list = []  # aborted gloo groups: keep them referenced so no destructor blocks the caller
_ABORTS: List[threading.Thread] = []


def _quiet_abort(pg) -> None:
    for fn in (pg.abort, pg.shutdown):  # shutdown also closes the pairs' sockets
        try:
            fn()
        except Exception:  # noqa: BLE001 - best effort on a broken group
            pass


@atexit.register
def _drain_graveyard() -> None:
    """At exit: let the off-thread aborts of the old gloo groups finish."""
    for t in _ABORTS:
        t.join(timeout=10.0)


def discard_process_groups(backend: str) -> None:
    """Abort and forget every process group of this process so a new default
    group can be initialised.  RCCL: ``_abort_process_group()`` (all
    communicators aborted inside one group call, kernels stop spinning).
    gloo: its ``abort()`` blocks until a hung peer's pending op ends, so it runs
    on a daemon thread and the bookkeeping that ``_abort_process_group`` would
    do is done here directly."""
    from torch.distributed import distributed_c10d as c10d

    if not dist.is_initialized():
        return
    if backend == "nccl":
        c10d._abort_process_group()
        return
    w = c10d._world
    for pg in list(w.pg_names):
        _GRAVEYARD.append(pg)
        t = threading.Thread(target=_quiet_abort, args=(pg,), daemon=True)
        t.start()
        _ABORTS.append(t)
    c10d._update_default_pg(None)
    for m in (w.pg_map, w.pg_names, w.pg_group_ranks, w.pg_backend_config, w.pg_to_tag, w.tags_to_pg,
              w.pg_coalesce_state):
        m.clear()
    c10d._unregister_all_process_groups()
    w.group_count = 0


class ElasticGroup:
    """Process-wide membership of the data-parallel group, and guarded
    collectives on it (see module docstring).  One instance per process
    (:meth:`get`); it always works on the *default* process group."""

    _current: Optional["ElasticGroup"] = None

    def __init__(self, timeout_s: float = 60.0, grace_s: Optional[float] = None, store=None,
                 poll_s: float = 2e-4):
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("ElasticGroup needs an initialised torch.distributed default group")
        from torch.distributed import PrefixStore

        self.backend = dist.get_backend()
        self.timeout = float(timeout_s)
        self._grace_fixed = float(grace_s) if grace_s is not None else None
        self.store = PrefixStore("dlion/elastic", store if store is not None else _default_store())
        self.me = dist.get_rank()  # stable identity: the original global rank
        self.members: List[int] = list(range(dist.get_world_size()))
        self.gen = 0
        self.seq = 0
        self.events: List[dict] = []
        self.stall_s = 0.0
        self.commits = 0
        self._poll = float(poll_s)
        self._last_commit_t: Optional[float] = None
        self._intervals: List[float] = []  # recent times between commits (~ the step time)
        self._listeners: List[Callable[["ElasticGroup"], None]] = []
        # the backend's own timeout must never fire before ours (RCCL's watchdog
        # would tear the process down)
        self.pg_timeout = datetime.timedelta(seconds=max(600.0, 10.0 * self.timeout))
        self.device = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else None
        self._pg = dist.group.WORLD
        # death notices: the failure-tolerant launcher (..launch) writes
        # ``dlion/dead/<rank>`` into the root store when a rank's process exits
        # with an error, so a dead peer is cut out at once instead of after the
        # deadline (an RCCL collective on a dead peer spins until aborted)
        root = self.store
        while isinstance(root, PrefixStore):
            root = root.underlying_store
        self._root = root
        self._dead: set = set()
        self._dead_count = 0
        self._trash: List[str] = []  # commit keys every member has read: deleted while the host idles

    @classmethod
    def get(cls, timeout_s: float = 60.0, **kw) -> "ElasticGroup":
        cur = cls._current
        if cur is None or not dist.is_initialized() or (dist.group.WORLD is not cur._pg):
            cur = cls._current = cls(timeout_s, **kw)
        return cur

    @classmethod
    def active(cls) -> Optional["ElasticGroup"]:
        cur = cls._current
        if cur is not None and dist.is_initialized() and dist.group.WORLD is cur._pg:
            return cur
        return None

    # ------------------------------------------------------------- topology
    @property
    def world(self) -> int:
        return len(self.members)

    @property
    def rank(self) -> int:
        return self.members.index(self.me)

    @property
    def grace(self) -> float:
        """Membership check-in window after a failure.  Live ranks arrive within
        the skew between ranks (a fraction of a step), so by default it is 3x
        the longest of the last 8 intervals between commits, at least 1 s and at
        most ``timeout`` (5 s before any history)."""
        if self._grace_fixed is not None:
            return self._grace_fixed
        if not self._intervals:
            return min(self.timeout, DEFAULT_GRACE_S)
        # a gloo survivor may spend GLOO_DRAIN_S draining its works before it checks in
        floor = 1.0 + (GLOO_DRAIN_S if self.backend == "gloo" else 0.0)
        return min(self.timeout, max(floor, 3.0 * max(self._intervals)))

    def dead_members(self) -> List[int]:
        """Members the launcher reported dead (one store round trip when
        nothing new died)."""
        try:
            n = self._root.add(DEATH_COUNT_KEY, 0)
        except Exception:  # noqa: BLE001 - no store, no notices
            return []
        if n != self._dead_count:
            self._dead_count = n
            for r in self.members:
                if r not in self._dead and self._root.check([f"{DEATH_KEY}/{r}"]):
                    self._dead.add(r)
        return [r for r in self.members if r in self._dead]

    def on_regroup(self, fn: Callable[["ElasticGroup"], None]) -> None:
        if fn not in self._listeners:
            self._listeners.append(fn)

    # ------------------------------------------------------ bounded waiting
    def wait_works(self, works) -> bool:
        """True when every work completed without error before the deadline.
        Only then is ``work.wait()`` called (it is what makes the compute
        stream depend on the collective).

        The launcher's death notices are consulted on EVERY backend: RCCL
        kernels spin on a dead peer until aborted, and gloo does not reliably
        fail a pending collective either -- with CUDA tensors a survivor whose
        peers had already pushed their bytes sat in the bounded wait for the
        whole ``elastic_timeout`` (round 3's 3-rank Llama-3-8B rehearsal:
        ``regroup_s`` 120.1 s = the deadline), so a death notice ends the wait
        within one 20 ms poll instead.  Under gloo the pending works then get
        a short drain (``GLOO_DRAIN_S``) to fail on the closed sockets by
        themselves: a gloo work abandoned while still running leaves a worker
        thread that ``terminate()``s the process at exit."""
        start = time.monotonic()
        deadline = start + self.timeout
        next_check = start + 0.02
        dec = f"{self.gen}/{self.seq}/decision"
        drain_until = None
        for w in works:
            if w is None:
                continue
            try:
                while not w.is_completed():
                    now = time.monotonic()
                    if now > deadline or (drain_until is not None and now > drain_until):
                        return False
                    if drain_until is None and now > next_check:  # a peer declared this collective failed, or died
                        next_check = now + 0.02
                        if self.store.check([dec]) or self.dead_members():
                            if self.backend != "gloo":
                                return False
                            drain_until = now + GLOO_DRAIN_S
                    if self._trash:  # store housekeeping while the host would sleep anyway
                        self._delete_keys(self._trash.pop())
                    else:
                        time.sleep(self._poll)
                if drain_until is not None:  # completed after a death: do not use it
                    try:
                        w.wait()
                    except Exception:  # noqa: BLE001 - expected on a closed peer
                        pass
                    continue
                w.wait()
            except Exception as e:  # noqa: BLE001 - a failed collective is what this detects
                log.warning("dlion elastic: collective failed on rank %d: %s", self.me, str(e)[:200])
                if drain_until is None and self.backend == "gloo":
                    drain_until = time.monotonic() + GLOO_DRAIN_S  # let the other works fail too
                    continue
                return False
        return drain_until is None

    # --------------------------------------------------------------- commit
    def commit(self, ok: bool) -> bool:
        """Store-arbitrated outcome of the current guarded collective: True
        when every member completed it (the result may be used), False when
        the survivors must regroup.  Identical on every surviving rank.

        Steady state costs two store round trips on every rank and no polling
        sleep: each member ``add``s itself to the commit's ok counter; the
        member that completes the count writes the decision (``compare_set``:
        the first decision written is final, so a concurrent "fail" wins or
        loses atomically), and the others block in one ``get`` of the decision
        key, which the store answers the moment it is written.  (Round 4 polled
        the key every 5 ms and had the deciding rank delete old keys inline:
        3-5 round trips plus up to 5 ms of sleep per commit.)"""
        key = f"{self.gen}/{self.seq}"
        self.seq += 1
        self.commits += 1
        dec = key + "/decision"
        now = time.monotonic()
        if self._last_commit_t is not None:
            self._intervals = (self._intervals + [now - self._last_commit_t])[-8:]
        self._last_commit_t = now
        if ok:
            if self.store.add(key + "/ok", 1) == self.world:
                val = self.store.compare_set(dec, "", "all")
                if val == b"all" and self.seq > 2:  # every member is past seq-2: its keys can go
                    self._trash.append(f"{self.gen}/{self.seq - 3}")
                return val == b"all"
        else:
            self.store.compare_set(dec, "", "fail")
        return self._await_decision(dec) == b"all"

    def _await_decision(self, dec: str) -> bytes:
        """Block until the decision of ``dec`` is written (one ``get``), in
        slices of DECISION_WAIT_S so that a member that died before adding
        itself -- it never will -- is noticed through the death notices or
        the deadline; then decide "fail" (first write wins)."""
        deadline = time.monotonic() + self.timeout + self.grace
        first = True
        while True:
            left = deadline - time.monotonic()
            if left <= 0 or (not first and self.dead_members()):
                break
            first = False
            # a per-call deadline (Store.wait): the client-wide timeout, shared
            # with the process groups' store operations on other threads, stays
            # as it is (set_timeout on the PrefixStore changed the
            # root TCPStore client's)
            try:
                self.store.wait([dec], datetime.timedelta(seconds=min(left, DECISION_WAIT_S)))
            except RuntimeError:  # DistStoreError: not decided yet
                continue
            return self.store.get(dec)
        return self.store.compare_set(dec, "", "fail")

    def _delete_keys(self, key: str) -> None:
        for k in ("/ok", "/decision"):
            try:
                self.store.delete_key(key + k)
            except Exception:  # noqa: BLE001 - best effort
                pass

    # --------------------------------------------------------------- regroup
    def regroup(self, tag: Optional[dict] = None) -> None:
        """Agree on the survivors, abort every group, initialise the new default
        group over them, notify listeners."""
        t0 = time.monotonic()
        ns = f"{self.gen}/members"
        self.store.set(f"{ns}/alive/{self.me}", "1")
        # wait until every member checked in or is known dead, at most ``grace``
        deadline = time.monotonic() + self.grace
        seen: List[int] = []
        while True:
            seen = [r for r in self.members if self.store.check([f"{ns}/alive/{r}"])]
            dead = set(self.dead_members())
            if all(r in dead or r in seen for r in self.members) or time.monotonic() > deadline:
                break
            time.sleep(0.01)
        seen = [r for r in seen if r not in dead]
        survivors = sorted(json.loads(self.store.compare_set(f"{ns}/decision", "", json.dumps(seen))))
        discard_process_groups(self.backend)
        if self.me not in survivors:
            raise WorkerExcluded(f"rank {self.me} was excluded from the group in generation {self.gen} "
                                 f"(survivors {survivors})")
        dropped = sorted(set(self.members) - set(survivors))
        self.gen += 1
        self.seq = 0
        self.members = survivors
        self._last_commit_t = None
        from torch.distributed import PrefixStore

        kw = dict(backend=self.backend, store=PrefixStore(f"pg/{self.gen}", self.store), rank=self.rank,
                  world_size=self.world, timeout=self.pg_timeout)
        if self.device is not None:
            kw["device_id"] = self.device
        dist.init_process_group(**kw)
        self._pg = dist.group.WORLD
        stall = time.monotonic() - t0
        self.stall_s += stall
        ev = dict(tag or {})
        ev.update({"generation": self.gen, "dropped": dropped, "survivors": survivors,
                   "regroup_s": round(stall, 3)})
        self.events.append(ev)
        log.warning("dlion elastic: ranks %s dropped; continuing on %s (new rank %d of %d)", dropped, survivors,
                    self.rank, self.world)
        for fn in list(self._listeners):
            fn(self)

    # ----------------------------------------------------- guarded execution
    def run(self, issue: Callable[[], tuple], tag: Optional[dict] = None):
        """``issue()`` launches async collectives on the *current* default
        group and returns ``(works, result)``.  Returns ``result`` once every
        member completed; on failure regroups and issues again."""
        while True:
            t0 = time.monotonic()
            try:
                works, result = issue()
                ok = self.wait_works(works)
            except WorkerExcluded:
                raise
            except Exception as e:  # noqa: BLE001 - issuing on a broken group
                log.warning("dlion elastic: issuing a collective failed: %s", str(e)[:200])
                ok = False
            if self.commit(ok):
                return result
            self.stall_s += time.monotonic() - t0
            self.regroup(tag)

    # ---------------------------------------------- guarded collective helpers
    def _dev(self, t: torch.Tensor) -> torch.Tensor:
        return t.to(self.device) if self.device is not None and t.device != self.device else t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """Concatenation along dim 0 of every member's ``t`` (``t`` 0-dim ->
        1-element rows), on ``t``'s device."""
        src = self._dev(t.reshape(1) if t.dim() == 0 else t).contiguous()

        def issue():
            outs = [torch.empty_like(src) for _ in range(self.world)]
            return [dist.all_gather(outs, src, async_op=True)], outs

        outs = self.run(issue, {"where": "all_gather"})
        return torch.cat(outs, dim=0).to(t.device)

    def all_reduce(self, t: torch.Tensor, op=dist.ReduceOp.SUM) -> torch.Tensor:
        """In-place all-reduce of ``t`` over the members (re-done from ``t``'s
        value at the call after a regroup)."""
        orig = t.detach().clone()
        buf = self._dev(t)

        def issue():
            buf.copy_(self._dev(orig))
            return [dist.all_reduce(buf, op=op, async_op=True)], buf

        self.run(issue, {"where": "all_reduce"})
        if buf is not t:
            t.copy_(buf)
        return t

    def barrier(self) -> None:
        self.all_reduce(torch.zeros(1, device=self.device or "cpu"))

    def stats(self) -> dict:
        return {"live_ranks": list(self.members), "dropout_events": list(self.events),
                "elastic_generation": self.gen, "elastic_commits": self.commits,
                "elastic_stall_s": round(self.stall_s, 3)}


def flatten_works(states) -> list:
    """Works out of the exchange's per-bucket states (a work, a list, or None)."""
    out = []
    for s in states:
        if isinstance(s, (list, tuple)):
            out.extend(x for x in s if x is not None)
        elif s is not None:
            out.append(s)
    return out


# ---------------------------------------------------------------- fault injection
_FAULT_PHASES = ("before_step", "backward", "after_launch", "in_allgather", "after_vote", "raise_in_launch")


class InjectedLaunchError(RuntimeError):
    """``raise_in_launch``: issuing bucket 1's vote collective failed (the rank lives on)."""


def parse_fault(spec: Optional[str]) -> list:
    """``"rank:step:phase[,rank:step:phase...]"`` (``DLION_FAULT``): the process
    of original global rank ``rank`` kills itself (SIGKILL: no teardown,
    sockets just close) at optimizer step ``step`` in ``phase`` -- one of
    before_step, backward (inside autograd), after_launch (vote all-to-all
    issued, not completed), in_allgather (vote all-gather issued), after_vote
    (step applied) -- or, for ``raise_in_launch``, raises
    :class:`InjectedLaunchError` where bucket 1's vote collective is issued
    (a broken group reporting at issue time; nobody dies)."""
    out = []
    for item in (spec or "").split(","):
        if not item.strip():
            continue
        r, s, ph = item.strip().split(":")
        if ph not in _FAULT_PHASES:
            raise ValueError(f"DLION_FAULT phase must be one of {_FAULT_PHASES}, got {ph!r}")
        out.append((int(r), int(s), ph))
    return out


_FAULT_CACHE: list = []


def fault_spec() -> list:
    if not _FAULT_CACHE:
        _FAULT_CACHE.append(parse_fault(os.environ.get("DLION_FAULT")))
    return _FAULT_CACHE[0]


def inject(phase: str, step: int) -> None:
    """Die here if ``DLION_FAULT`` names this rank, step and phase."""
    faults = fault_spec()
    if not faults or not (dist.is_available() and dist.is_initialized()):
        return
    eg = ElasticGroup.active()
    me = eg.me if eg is not None else dist.get_rank()
    if (me, step, phase) in faults:
        if phase == "raise_in_launch":
            raise InjectedLaunchError(f"injected launch failure on rank {me} at step {step}")
        import signal
        import sys

        print(json.dumps({"rank": me, "event": "fault", "step": step, "phase": phase}), file=sys.stderr, flush=True)
        os.kill(os.getpid(), signal.SIGKILL)
