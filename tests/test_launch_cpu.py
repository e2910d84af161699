"""The failure-tolerant launcher (distributed_lion_pytorch_amd.launch) never
orphans its ranks: a SIGTERM to the launcher reaches every rank process and
the launcher reaps them before it exits."""
import os
import signal
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    # a zombie still answers kill(0); check its state
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().split()[2] != "Z"
    except FileNotFoundError:
        return False


def test_sigterm_to_launcher_stops_every_rank(tmp_path):
    script = tmp_path / "sleeper.py"
    script.write_text("import os, time\n"
                      f"open(os.path.join({str(tmp_path)!r}, 'pid' + os.environ['RANK']), 'w').write(str(os.getpid()))\n"
                      "time.sleep(120)\n")
    p = subprocess.Popen([sys.executable, "-m", "distributed_lion_pytorch_amd.launch", "--nproc", "2", str(script)],
                         cwd=ROOT)
    pids = []
    deadline = time.monotonic() + 60
    while time.monotonic() < deadline and len(pids) < 2:
        pids = [int((tmp_path / f"pid{r}").read_text()) for r in range(2)
                if (tmp_path / f"pid{r}").exists() and (tmp_path / f"pid{r}").read_text()]
        time.sleep(0.1)
    assert len(pids) == 2
    p.send_signal(signal.SIGTERM)
    rc = p.wait(timeout=30)
    assert rc != 0
    time.sleep(0.2)
    assert not any(_alive(x) for x in pids), pids


def test_ranks_get_one_signal_and_a_grace_period(tmp_path):
    """after forwarding SIGTERM the launcher gives the ranks time
    to shut down on their own (here: a 1 s "checkpoint flush" in the
    handler) instead of SIGTERMing them again at once."""
    script = tmp_path / "flusher.py"
    script.write_text(
        "import os, signal, time\n"
        f"d = {str(tmp_path)!r}\n"
        "n = [0]\n"
        "def h(signum, frame):\n"
        "    n[0] += 1\n"
        "    if n[0] == 1:\n"
        "        time.sleep(1.0)\n"
        "        open(os.path.join(d, 'flushed' + os.environ['RANK']), 'w').write(str(n[0]))\n"
        "        os._exit(0)\n"
        "signal.signal(signal.SIGTERM, h)\n"
        "open(os.path.join(d, 'pid' + os.environ['RANK']), 'w').write(str(os.getpid()))\n"
        "time.sleep(120)\n")
    p = subprocess.Popen([sys.executable, "-m", "distributed_lion_pytorch_amd.launch", "--nproc", "2", str(script)],
                         cwd=ROOT)
    deadline = time.monotonic() + 60
    while time.monotonic() < deadline and not all((tmp_path / f"pid{r}").exists() for r in range(2)):
        time.sleep(0.1)
    time.sleep(0.3)
    p.send_signal(signal.SIGTERM)
    p.wait(timeout=30)
    # each rank saw exactly one SIGTERM (n == 1 when it flushed) and finished its flush
    assert [(tmp_path / f"flushed{r}").read_text() for r in range(2)] == ["1", "1"]
