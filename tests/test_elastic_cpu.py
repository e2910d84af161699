"""Real worker dropout (gloo, CPU): a rank process exits mid-run, the survivors
detect it at the next step's heartbeat, regroup and keep identical replicas."""
import hashlib
import os

import torch
import torch.distributed as dist

from distributed_lion_pytorch_amd import Lion
from tests.dist_utils import run_world


def _digest(t):
    return hashlib.sha256(t.detach().float().numpy().tobytes()).hexdigest()


def _train(rank, world, exchange, drop_rank, drop_step, steps):
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Tanh(), torch.nn.Linear(32, 4))
    opt = Lion(model.parameters(), lr=1e-2, weight_decay=0.1, exchange=exchange, elastic_timeout=3.0,
               backend="torch")
    gen = torch.Generator().manual_seed(100 + rank)
    for step in range(steps):
        if rank == drop_rank and step == drop_step:
            # the worker dies: no goodbye, no collective, no process-group teardown
            os._exit(0)
        x = torch.randn(8, 16, generator=gen)
        loss = model(x).pow(2).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
    st = opt.stats()
    params = torch.cat([p.detach().flatten() for p in model.parameters()])
    # survivors can still talk to each other in the shrunken group
    t = torch.tensor([float(rank)])
    dist.all_reduce(t, group=opt.process_group)
    return {"digest": _digest(params), "world": st["world"], "live": st.get("live_ranks"),
            "events": st.get("dropout_events"), "sum": float(t)}


def _run(world, exchange, drop_rank, drop_step, steps=5):
    import torch.multiprocessing as mp

    from tests import dist_utils

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = dist_utils.free_port()
    procs = [ctx.Process(target=dist_utils._entry,
                         args=(r, world, port, _train, (exchange, drop_rank, drop_step, steps), q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world - 1):
            r, status, res = q.get(timeout=180)
            assert status == "ok", res
            out[r] = res
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return out


def test_real_dropout_allgather():
    out = _run(3, "allgather", drop_rank=2, drop_step=2)
    assert sorted(out) == [0, 1]
    assert out[0]["digest"] == out[1]["digest"]
    assert out[0]["world"] == 2 and out[0]["live"] == [0, 1]
    assert out[0]["events"] == [{"step": 2, "dropped": [2], "survivors": [0, 1]}]
    assert out[0]["sum"] == 1.0


def test_real_dropout_a2a_w4():
    out = _run(4, "a2a", drop_rank=1, drop_step=3)
    assert sorted(out) == [0, 2, 3]
    assert len({o["digest"] for o in out.values()}) == 1
    assert all(o["world"] == 3 and o["live"] == [0, 2, 3] for o in out.values())
    assert out[2]["sum"] == 5.0


def test_no_dropout_heartbeat_is_transparent():
    res = run_world(_train, 2, "allgather", -1, -1, 4)
    assert res[0]["digest"] == res[1]["digest"]
    assert res[0]["events"] == [] and res[0]["world"] == 2


def test_dropout_stress_entrypoint_torchrun():
    """dropout_stress.py (BASELINE config #5 harness) under torchrun, 3 gloo ranks."""
    import json
    import subprocess
    import sys

    from tests.dist_utils import free_port

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "3",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(root, "dropout_stress.py"),
           "--model", "gpt2-tiny", "--device", "cpu", "--seq_len", "32", "--micro_batch", "2", "--steps", "5",
           "--drop_rank", "1", "--drop_step", "2", "--elastic_timeout", "5"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith('{"metric"')][-1]
    res = json.loads(line)
    assert res["world_start"] == 3 and res["world_end"] == 2 and res["replicas_identical"]
    assert res["dropout_events"] == [{"step": 2, "dropped": [1], "survivors": [0, 2]}]
