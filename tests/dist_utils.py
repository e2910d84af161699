"""Multi-process helpers: spawn W gloo ranks on 127.0.0.1 and collect results."""
import io
import os
import socket
import traceback

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, world, port, fn, args, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(world)
    os.environ["LOCAL_RANK"] = str(rank)
    torch.set_num_threads(1)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        out = fn(rank, world, *args)
        # by value: a tensor put on the queue travels as a shared-memory fd that the
        # parent fetches from THIS process, which may already have exited
        # (ConnectionResetError in rebuild_storage_fd on a loaded box)
        buf = io.BytesIO()
        torch.save(out, buf)
        q.put((rank, "ok", buf.getvalue()))
    except Exception:  # pragma: no cover - reported to the parent
        q.put((rank, "err", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def run_world(fn, world, *args, timeout=240):
    """Run fn(rank, world, *args) on `world` gloo ranks; return results by rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            rank, status, out = q.get(timeout=timeout)
            if status != "ok":
                raise RuntimeError(f"rank {rank} failed:\n{out}")
            results[rank] = torch.load(io.BytesIO(out), weights_only=True)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return [results[r] for r in range(world)]
