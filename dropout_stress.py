#!/usr/bin/env python
"""Worker-dropout stress run (BASELINE config #5: "Llama-3 8B bf16 Distributed
Lion async worker-dropout stress, 1 rank drops mid-run").

Every rank trains its own replica on its own synthetic data through the
native engine (no gradient all-reduce, Lion vote sync).  At optimizer step
``--drop_step`` the process of rank ``--drop_rank`` kills itself (SIGKILL: no
teardown, no goodbye) at ``--drop_phase``:

  before_step   between steps
  backward      inside autograd (the survivors are already in their vote)
  after_launch  after issuing the vote all-to-all, before it completed
  in_allgather  after issuing the vote's 1-bit all-gather
  after_vote    right after applying the step

With ``--elastic_timeout`` the survivors detect it (bounded wait on the vote
collectives), agree on the outcome through the rendezvous store, regroup,
re-vote that step among themselves and carry on (parallel/elastic.py); the run
then checks that the survivors' parameters are bit-identical and reports
tokens/s before and after the drop plus the regroup stall.

Launch it with the failure-tolerant launcher (torchrun stops every worker
when one dies; this launcher hosts the store itself, so even rank 0 may drop):

  python -m distributed_lion_pytorch_amd.launch --nproc 8 --max_failures 1 dropout_stress.py \
      --model llama-3-8b --micro_batch 1 --seq_len 2048 --steps 20 --drop_rank 5 --drop_step 8
  # CPU rehearsal (gloo): --model llama-tiny / gpt2-tiny --device cpu
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_lion_pytorch_amd import Lion  # noqa: E402
from distributed_lion_pytorch_amd.models.registry import build_model, load_config  # noqa: E402
from distributed_lion_pytorch_amd.parallel.elastic import ElasticGroup  # noqa: E402
from distributed_lion_pytorch_amd.trainer.engine import TrainStep, broadcast_parameters  # noqa: E402


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--micro_batch", type=int, default=1)
    ap.add_argument("--seq_len", type=int, default=2048)
    ap.add_argument("--grad_accum", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--drop_rank", type=int, default=1)
    ap.add_argument("--drop_step", type=int, default=8)
    ap.add_argument("--drop_phase", default="backward",
                    choices=["before_step", "backward", "after_launch", "in_allgather", "after_vote"])
    ap.add_argument("--elastic_timeout", type=float, default=30.0)
    ap.add_argument("--elastic_grace", type=float, default=None,
                    help="membership check-in window after a failure (default min(timeout, 5 s))")
    ap.add_argument("--exchange", default="a2a")
    ap.add_argument("--lr", type=float, default=1e-5)
    ap.add_argument("--weight_decay", type=float, default=0.0)
    ap.add_argument("--gradient_checkpointing", action="store_true")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo on cuda: rehearse N ranks on fewer GPUs (ranks share cuda:local%%ngpu)")
    return ap.parse_args()


def main():
    a = parse()
    if a.drop_rank >= 0:
        os.environ["DLION_FAULT"] = f"{a.drop_rank}:{a.drop_step}:{a.drop_phase}"
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.device == "cuda":
        if a.backend == "gloo":
            local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if a.backend == "nccl":
            # the elastic path aborts communicators itself; the watchdog must not kill the process first
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "0")
            os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        dtype = torch.bfloat16
    else:
        dev = torch.device("cpu")
        dist.init_process_group("gloo")
        dtype = torch.float32
    if a.drop_rank == 0 and os.environ.get("TORCHELASTIC_USE_AGENT_STORE") != "True":
        raise SystemExit("--drop_rank 0 needs a launcher-hosted store (python -m distributed_lion_pytorch_amd.launch "
                         "or torchrun); with a rank-0-hosted store drop another rank")
    cfg = load_config(a.model)
    torch.manual_seed(0)
    with torch.device(dev):  # materialise on the device (8B: no 32 GB host copy per rank)
        model = build_model(cfg, native=True).to(dtype=dtype)
    if a.gradient_checkpointing:
        model.gradient_checkpointing_enable()
    broadcast_parameters(model)
    el = ElasticGroup.get(a.elastic_timeout, grace_s=a.elastic_grace)
    opt = Lion([p for p in model.parameters() if p.requires_grad], lr=a.lr, weight_decay=a.weight_decay,
               exchange=a.exchange, elastic_timeout=a.elastic_timeout)
    step_fn = TrainStep(model, opt, grad_accum=a.grad_accum, max_grad_norm=1.0)
    gen = torch.Generator(device=dev).manual_seed(1000 + rank)

    def batches():
        for _ in range(a.grad_accum):
            ids = torch.randint(0, cfg.vocab_size, (a.micro_batch, a.seq_len), device=dev, generator=gen)
            yield {"input_ids": ids, "labels": ids}

    log = []
    for s in range(a.steps):
        t0 = time.perf_counter()
        loss = step_fn(batches())
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        w = el.world
        log.append({"step": s, "world": w, "loss": float(loss), "s": round(dt, 4),
                    "tokens_per_s": w * a.grad_accum * a.micro_batch * a.seq_len / dt})
        if el.rank == 0:
            print(json.dumps({"progress": log[-1]}), file=sys.stderr, flush=True)
    # survivors: compare replicas over the (possibly regrouped) default group
    h = hashlib.sha256()
    for p in model.parameters():
        h.update(p.detach().float().cpu().numpy().tobytes())
    d = torch.tensor([int.from_bytes(h.digest()[:7], "little")], dtype=torch.int64, device=dev)
    digests = el.all_gather(d).tolist()
    st = opt.stats()
    if el.rank == 0:
        ev = st.get("dropout_events") or []
        first = ev[0]["step"] if ev else a.steps
        pre = [r["tokens_per_s"] for r in log if 0 < r["step"] < first]
        post = [r["tokens_per_s"] for r in log if r["step"] > first + 1]
        print(json.dumps({
            "metric": "worker-dropout stress", "model": a.model, "world_start": world, "world_end": el.world,
            "fault": os.environ.get("DLION_FAULT"), "dropout_events": ev, "survivors": el.members,
            "replicas_identical": len(set(digests)) == 1, "elastic_stall_s": st.get("elastic_stall_s"),
            "elastic_commits": st.get("elastic_commits"),
            "tokens_per_s_before": sum(pre) / max(1, len(pre)), "tokens_per_s_after": sum(post) / max(1, len(post)),
            "final_loss": log[-1]["loss"], "steps": log}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
