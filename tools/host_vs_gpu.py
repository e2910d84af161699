"""Is the training step host-bound?  Times how long the host takes to ENQUEUE
each step (step() returning, no synchronisation) against the step's wall time
after a synchronise, for the bench.py GPT-2 config.  A host time close to the
wall time means the GPU queue runs dry between launches (host-bound); the
margin is what CPU contention (8 ranks per node) can eat before the GPU waits.
usage: python tools/host_vs_gpu.py [--task clm|sft|llama3] [--steps N]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from distributed_lion_pytorch_amd.trainer.engine import TrainStep  # noqa: E402


def main():
    sys.argv = [sys.argv[0]] + sys.argv[1:]
    args = bench.parse()
    world, rank, dev = bench.setup_dist(args)
    model, opt, cfg = bench.build_native(args, dev)
    step = TrainStep(model, opt, grad_accum=args.grad_accum, max_grad_norm=args.max_grad_norm,
                     fuse_grad_accumulation=bool(args.fuse_accum))
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234)

    def batches():
        for _ in range(args.grad_accum):
            ids = torch.randint(0, cfg.vocab_size, (args.micro_batch, args.seq_len), device=dev, generator=gen)
            yield {"input_ids": ids, "labels": ids}

    for _ in range(args.warmup):
        step(batches())
    torch.cuda.synchronize()
    host, wall = [], []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        step(batches())
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host.append((t1 - t0) * 1e3)
        wall.append((t2 - t0) * 1e3)
    print(json.dumps({"task": args.task, "host_enqueue_ms": [round(h, 2) for h in host],
                      "wall_ms": [round(w, 2) for w in wall],
                      "host_fraction": round(sum(host) / sum(wall), 3)}), flush=True)


if __name__ == "__main__":
    main()
