"""Steady-state cost of elastic mode's guarded collectives, without a model:
W gloo ranks on the CPU time (a) a plain 1-element all_reduce, (b) the same
through ElasticGroup (host poll + store-arbitrated commit), with the round-4
commit protocol (5 ms decision polling, inline key deletes) and the current
one.  The difference (b) - (a) is what elastic mode adds per guarded
collective.  python tools/elastic_overhead.py [world] [iters]"""
import datetime
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def commit_r4(self, ok):  # round 4's protocol, kept here for the A/B only
    key = f"{self.gen}/{self.seq}"
    self.seq += 1
    self.commits += 1
    dec = key + "/decision"
    if ok:
        if self.store.add(key + "/ok", 1) == self.world:
            val = self.store.compare_set(dec, "", "all")
            if val == b"all" and self.seq > 2:
                old = f"{self.gen}/{self.seq - 3}"
                for k in ("/ok", "/decision"):
                    try:
                        self.store.delete_key(old + k)
                    except Exception:  # noqa: BLE001
                        pass
            return val == b"all"
    else:
        self.store.compare_set(dec, "", "fail")
    deadline = time.monotonic() + self.timeout + self.grace
    while not self.store.check([dec]):
        if time.monotonic() > deadline or self.dead_members():
            break
        time.sleep(0.005)
    return self.store.compare_set(dec, "", "fail") == b"all"


def worker(rank, world, port, iters, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=120))
    from distributed_lion_pytorch_amd.parallel import elastic

    el = elastic.ElasticGroup(timeout_s=60.0)
    t = torch.zeros(1)
    res = {}
    for rnd in range(3):  # interleaved rounds
        for name in ("plain", "elastic_r4", "elastic"):
            dist.barrier()
            if name == "elastic_r4":
                el.commit = commit_r4.__get__(el)
            elif name == "elastic":
                el.commit = elastic.ElasticGroup.commit.__get__(el)
            t0 = time.perf_counter()
            for _ in range(iters):
                if name == "plain":
                    dist.all_reduce(t)
                else:
                    el.all_reduce(t)
            res.setdefault(name, []).append((time.perf_counter() - t0) / iters * 1e6)
    q.put((rank, res))
    dist.destroy_process_group()


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + os.getpid() % 200
    ps = [ctx.Process(target=worker, args=(r, world, port, iters, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=600) for _ in ps)
    for p in ps:
        p.join()
    r0 = out[0]
    for k, v in r0.items():
        print(f"W={world} {k:11s} us/collective per round: " + " ".join(f"{x:8.1f}" for x in v))
    base = min(r0["plain"])
    for k in ("elastic_r4", "elastic"):
        print(f"W={world} {k:11s} added per guarded collective: {min(r0[k]) - base:8.1f} us (best round)")


if __name__ == "__main__":
    main()
