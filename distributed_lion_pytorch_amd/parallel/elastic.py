"""Real worker dropout: detect dead ranks between optimizer steps and keep
training on the survivors.

The reference claims robustness to worker drop-out (/root/reference/README.md:2)
but its blocking per-tensor ``dist.all_gather`` (distributed_lion.py:81) hangs
every survivor until the c10d watchdog kills the job.  Majority
vote over the *live* voters is still a valid Distributed Lion step, so a dead
rank only has to be detected and cut out of the vote group:

1. **Heartbeat.**  Before its vote collectives, every member publishes
   ``<prefix>/<gen>/<step>/hb/<rank>`` to the rendezvous store and waits (with
   ``timeout_s``) for all members' keys.  No collective is entered with a
   rank that has not checked in, so nothing can hang on it.
2. **Agreement.**  On timeout each survivor proposes the members whose keys it
   sees; the first proposal written with ``compare_set`` is the decision for
   everybody, so all survivors adopt the identical member list even when a
   slow rank checks in during the race.  A rank left out of the decision
   (it was only late) raises :class:`WorkerExcluded` instead of voting on.
3. **Regroup.**  Survivors build a new process group over themselves only
   (``new_group(..., use_local_synchronization=True)``: the dead rank never has
   to call it) and the optimizer re-plans for the new world size on the same
   step.  Parameters stay identical on the survivors because they were
   identical before and every survivor applies the same vote.

Granularity is one optimizer step: a rank that dies *inside* a collective is
still caught by the backend's own timeout.  The store must outlive the dead
rank -- torchrun's agent-hosted store does; with a rank-0-hosted TCPStore,
rank 0 cannot be the one that drops.
"""
from __future__ import annotations

import datetime
import json
import logging
from typing import List, Optional

import torch.distributed as dist

log = logging.getLogger(__name__)


class WorkerExcluded(RuntimeError):
    """This rank was voted out of the group (it checked in after the deadline)."""


def _default_store():
    from torch.distributed import distributed_c10d as c10d

    return c10d._get_default_store()


class ElasticMembership:
    """Tracks the live members of a vote group across optimizer steps.

    ``check(step)`` returns ``None`` while everybody is alive, or the new
    process group over the survivors after a drop (also kept in ``.group``).
    """

    def __init__(self, timeout_s: float = 60.0, group=None, store=None, prefix: str = "dlion/elastic"):
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("ElasticMembership needs an initialised torch.distributed process group")
        self.timeout = datetime.timedelta(seconds=float(timeout_s))
        self.group = group
        self.store = store if store is not None else _default_store()
        self.prefix = prefix
        self.me = dist.get_rank()
        self.members: List[int] = sorted(dist.get_process_group_ranks(group)) if group is not None else list(
            range(dist.get_world_size()))
        self.gen = 0
        self.events: List[dict] = []
        self._last_step: Optional[int] = None

    # ------------------------------------------------------------------ keys
    def _hb(self, step: int, r: int) -> str:
        return f"{self.prefix}/{self.gen}/{step}/hb/{r}"

    def _decision(self, step: int) -> str:
        return f"{self.prefix}/{self.gen}/{step}/decision"

    def _cleanup(self, step: int) -> None:
        # keys of two steps ago can go: every member has passed that heartbeat
        for r in self.members:
            try:
                self.store.delete_key(self._hb(step - 2, r))
            except Exception:  # noqa: BLE001 - best effort (older stores lack delete_key)
                return

    # ----------------------------------------------------------------- check
    def check(self, step: int):
        if len(self.members) <= 1:
            return None
        self.store.set(self._hb(step, self.me), "1")
        keys = [self._hb(step, r) for r in self.members]
        try:
            self.store.wait(keys, self.timeout)
            self._cleanup(step)
            return None
        except Exception:  # noqa: BLE001 - DistStoreError / RuntimeError on timeout
            pass
        seen = [r for r in self.members if self.store.check([self._hb(step, r)])]
        decided = self.store.compare_set(self._decision(step), "", json.dumps(seen))
        survivors = sorted(json.loads(decided))
        dropped = sorted(set(self.members) - set(survivors))
        if self.me not in survivors:
            raise WorkerExcluded(f"rank {self.me} was excluded from the vote group at step {step} "
                                 f"(survivors {survivors})")
        if not dropped:  # everybody made it in the end
            return None
        log.warning("dlion elastic: step %d: ranks %s dropped; continuing on %s", step, dropped, survivors)
        self.events.append({"step": step, "dropped": dropped, "survivors": survivors})
        self.members = survivors
        self.gen += 1
        self.group = dist.new_group(ranks=survivors, use_local_synchronization=True)
        return self.group

    @property
    def world(self) -> int:
        return len(self.members)
