"""Failure-tolerant single-node launcher: one process per rank, the rendezvous
store hosted HERE (not in rank 0), survivors keep running when a rank dies.

    python -m distributed_lion_pytorch_amd.launch --nproc 8 [--max_failures 1] script.py [args...]

Why not torchrun: its agent stops the whole worker group as soon as one
worker exits with an error, which turns a single worker's death into a job
failure -- the opposite of the worker-dropout robustness the reference claims
(/root/reference/README.md:2).  This launcher

* starts a ``TCPStore`` server in the launcher process and exports
  ``TORCHELASTIC_USE_AGENT_STORE=True`` so every rank's ``env://`` rendezvous
  connects as a client (the store survives any rank, rank 0 included -- it is
  what parallel/elastic.py arbitrates membership through);
* exports RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR /
  MASTER_PORT (127.0.0.1) like torchrun;
* tolerates up to ``--max_failures`` ranks dying (any exit status, signals
  included) and posts a death notice (``dlion/dead/<rank>``) in the store for
  each, so the survivors regroup without waiting out a deadline; beyond that
  it terminates the remaining ranks.  Exit status: 0
  when every other rank exited 0, else the first non-tolerated failure's.

It never touches the GPU (children are fresh interpreters; nothing is forked
or exec'd from a process with a HIP context).  ``bench.py --gpus N`` uses
:func:`run` with ``max_failures=0``.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import signal
import socket
import subprocess
import sys
import time
from typing import List, Optional, Sequence


DEATH_KEY = "dlion/dead"  # parallel/elastic.py reads these (kept in sync by test_elastic_cpu)
DEATH_COUNT_KEY = "dlion/dead_count"
# seconds the ranks get to exit on their own after a forwarded SIGTERM / SIGINT
SIGNAL_GRACE_S = float(os.environ.get("DLION_LAUNCH_GRACE_S", "10"))


def _free_port(host: str) -> int:
    with socket.socket() as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def run(cmd: Sequence[str], nproc: int, max_failures: int = 0, host: str = "127.0.0.1", port: Optional[int] = None,
        quiet_ranks: bool = False, env: Optional[dict] = None, report: Optional[str] = None) -> int:
    """Run ``cmd`` (argv list) as ``nproc`` ranks; see module docstring.
    ``quiet_ranks``: only rank 0's stdout reaches ours.  ``report``: path of a
    JSON summary (per-rank exit status, tolerated failures)."""
    from torch.distributed import TCPStore

    port = port or _free_port(host)
    store = TCPStore(host, port, nproc + 1, is_master=True, wait_for_workers=False,
                     timeout=datetime.timedelta(seconds=300))
    procs: List[subprocess.Popen] = []
    base = dict(os.environ if env is None else env)
    for r in range(nproc):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_WORLD_SIZE=str(nproc),
                 GROUP_RANK="0", MASTER_ADDR=host, MASTER_PORT=str(port), TORCHELASTIC_USE_AGENT_STORE="True",
                 DLION_LAUNCHER="distributed_lion_pytorch_amd.launch")
        out = subprocess.DEVNULL if (quiet_ranks and r > 0) else None
        procs.append(subprocess.Popen(list(cmd), env=e, stdout=out))
    codes: List[Optional[int]] = [None] * nproc
    failed: List[int] = []
    rc = 0
    # a launcher that is itself signalled (scheduler SIGTERM, Ctrl-C) or fails
    # must not orphan rank processes holding GPUs: forward the signal, then
    # terminate / kill whatever is left (finally block)
    prev = {}
    signalled = []

    def _foreground_sigint() -> bool:
        # Ctrl-C at a terminal already reached every process of the foreground
        # group, the ranks included (they inherit the launcher's group)
        try:
            return os.tcgetpgrp(sys.stdin.fileno()) == os.getpgrp()
        except (OSError, ValueError, AttributeError):
            return False

    def _forward(signum, _frame):
        signalled.append(signum)
        if not (signum == signal.SIGINT and _foreground_sigint()):
            for q in procs:
                if q.poll() is None:
                    try:
                        q.send_signal(signum)
                    except OSError:
                        pass
        raise KeyboardInterrupt if signum == signal.SIGINT else SystemExit(128 + signum)

    for sig in (signal.SIGTERM, signal.SIGINT):
        try:
            prev[sig] = signal.signal(sig, _forward)
        except ValueError:  # not the main thread: no handler, the finally block still cleans up
            pass
    try:
        while any(c is None for c in codes):
            for r, p in enumerate(procs):
                if codes[r] is not None:
                    continue
                c = p.poll()
                if c is None:
                    continue
                codes[r] = c
                if c != 0:
                    failed.append(r)
                    # death notice for parallel/elastic.py: survivors stop waiting for r at once
                    store.set(f"{DEATH_KEY}/{r}", str(c))
                    store.add(DEATH_COUNT_KEY, 1)
                    if len(failed) > max_failures and rc == 0:
                        rc = c if c > 0 else 128 - c
                        print(f"launch: rank {r} exited with {c} ({len(failed)} failures > {max_failures} "
                              "tolerated); stopping the other ranks", file=sys.stderr, flush=True)
                        for q in procs:
                            if q.poll() is None:
                                q.terminate()
                    else:
                        print(f"launch: rank {r} exited with {c}; tolerated ({len(failed)}/{max_failures}), the "
                              "other ranks continue", file=sys.stderr, flush=True)
            time.sleep(0.05)
    finally:
        for sig, h in prev.items():
            signal.signal(sig, h)
        live = [q for q in procs if q.poll() is None]
        if signalled:
            # the ranks got the signal: let them shut down on their own first
            # (flush a checkpoint, abort their process groups) before SIGTERM
            grace = time.monotonic() + SIGNAL_GRACE_S
            while live and time.monotonic() < grace:
                time.sleep(0.05)
                live = [q for q in live if q.poll() is None]
        for q in live:
            q.terminate()
        deadline = time.monotonic() + 10.0
        for q in live:
            try:
                q.wait(timeout=max(0.1, deadline - time.monotonic()))
            except subprocess.TimeoutExpired:
                q.kill()
                q.wait()
    del store
    if report:
        with open(report, "w") as f:
            json.dump({"nproc": nproc, "exit_codes": codes, "failed_ranks": failed, "max_failures": max_failures,
                       "rc": rc}, f)
    return rc


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--nproc", "--nproc-per-node", "--nproc_per_node", dest="nproc", type=int, required=True)
    ap.add_argument("--max_failures", type=int, default=0, help="ranks allowed to die without failing the job")
    ap.add_argument("--master_addr", "--master-addr", dest="host", default="127.0.0.1")
    ap.add_argument("--master_port", "--master-port", dest="port", type=int, default=None)
    ap.add_argument("--report", default=None, help="write a JSON summary of the ranks' exit codes here")
    ap.add_argument("-m", dest="module", default=None, help="run a module (python -m) instead of a script")
    ap.add_argument("script", nargs="?")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    if a.module:
        cmd = [sys.executable, "-u", "-m", a.module] + ([a.script] if a.script else []) + a.args
    else:
        if not a.script:
            ap.error("a script (or -m module) is required")
        cmd = [sys.executable, "-u", a.script] + a.args
    return run(cmd, a.nproc, a.max_failures, a.host, a.port, report=a.report)


if __name__ == "__main__":
    sys.exit(main())
