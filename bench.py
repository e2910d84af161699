#!/usr/bin/env python
"""Headline benchmark: GPT-2 small CLM training with Distributed Lion.

Metric (BASELINE.json): tokens/sec (whole job) + vote wire bytes per step,
GPT-2 CLM at 1/2/4/8 MI355X.  Config = the reference's README run
(/root/reference/README.md:20-37): GPT-2 small (124M, `--config_name gpt2`,
random init), bf16 weights (`--torch_dtype bfloat16`), per-device batch 20,
block size 1024, gradient accumulation 8, Lion lr 1e-4 / wd 0.1, async grads
(no gradient all-reduce), HF-default local grad clipping at 1.0, dropout 0.1.
Data is synthetic (random token ids of that shape; no network).

  python bench.py --gpus N --steps K --warmup W
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Every step is a full training step (8 micro-batches fwd+bwd, clip, vote
exchange over RCCL, Lion update).  Rank 0 prints one JSON line.
`--impl reference` runs the reference algorithm on the same hardware (HF
GPT2LMHeadModel + per-tensor int64 all_gather Lion) for an A/B comparison.
`--task sft` measures BASELINE config #3 instead: Llama-2-7B, LoRA r=8 on
q_proj/v_proj (bf16 base instead of the reference's 4-bit NF4), per-device
batch 4 x seq 1024, grad-accum 2, Lion lr 1e-4 / wd 0.05; `--task dpo`
BASELINE config #4: Llama-2-7B LoRA DPO, policy fwd+bwd plus frozen
reference fwd on 4 chosen/rejected pairs x 1024 tokens, grad-accum 4,
gradient checkpointing (dpo_llama2.py defaults); `--task llama3` BASELINE
config #5's model: Llama-3-8B full-parameter bf16 Lion, 4 x 2048 tokens per
step (the worker-dropout stress itself is dropout_stress.py).
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from distributed_lion_pytorch_amd import Lion  # noqa: E402
from distributed_lion_pytorch_amd.models.gpt2 import gpt2_config  # noqa: E402
from distributed_lion_pytorch_amd.parallel.exchange import wire_bytes_per_step  # noqa: E402
from distributed_lion_pytorch_amd.trainer.engine import StepTimer, TrainStep, broadcast_parameters  # noqa: E402
from distributed_lion_pytorch_amd.utils.timing import PhaseTimer  # noqa: E402


# reference configs: run_clm README (/root/reference/README.md:20-37) and
# sft_llama2 README + defaults (README.md:41-62, sft_llama2.py:29-51)
PRESETS = {
    "clm": dict(model="gpt2", micro_batch=20, seq_len=1024, grad_accum=8, lr=1e-4, weight_decay=0.1, lora=None,
                metric="tokens/sec + all-reduce bytes/step, GPT-2 CLM at 1/2/4/8 MI355X"),
    "sft": dict(model="llama-2-7b", micro_batch=4, seq_len=1024, grad_accum=2, lr=1e-4, weight_decay=0.05,
                lora=dict(r=8, lora_alpha=16, lora_dropout=0.05, target_modules=["q_proj", "v_proj"]),
                metric="tokens/sec + all-reduce bytes/step, Llama-2-7B LoRA SFT (sft_llama2 config)"),
    # dpo_llama2.py:25-52 defaults: batch 4 pairs, grad-accum 4, max_length 1024 (prompt 512), beta 0.1,
    # lr 5e-4, wd 0.05, gradient checkpointing on, LoRA r=8 (its target list's Llama names: q/k/v_proj);
    # frozen reference model = a copy of the base weights.  Tokens counted = chosen + rejected sequences.
    "dpo": dict(model="llama-2-7b", micro_batch=4, seq_len=1024, grad_accum=4, lr=5e-4, weight_decay=0.05,
                lora=dict(r=8, lora_alpha=16, lora_dropout=0.05, target_modules=["q_proj", "v_proj", "k_proj"]),
                grad_ckpt=True, dpo_beta=0.1,
                metric="tokens/sec + all-reduce bytes/step, Llama-2-7B LoRA DPO (dpo_llama2 config)"),
    # BASELINE config #5's model: Llama-3-8B, FULL-parameter bf16 Distributed Lion
    # (8.03B trainable: the optimizer hot path at scale -- 1-bit vote planes of
    # 1 GB per rank, encode/apply over 48 GB of weights+grads+momentum), the
    # dropout_stress.py shape (seq 2048) with 4 sequences per micro-batch.
    "llama3": dict(model="llama-3-8b", micro_batch=4, seq_len=2048, grad_accum=1, lr=1e-5, weight_decay=0.0,
                   lora=None,
                   metric="tokens/sec + all-reduce bytes/step, Llama-3-8B full-parameter bf16 Distributed Lion"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--task", default="clm", choices=sorted(PRESETS),
                    help="clm: GPT-2 pretraining (headline); sft: Llama-2-7B LoRA SFT (sft_llama2 config)")
    ap.add_argument("--model", default=None)
    ap.add_argument("--micro_batch", type=int, default=None)
    ap.add_argument("--seq_len", type=int, default=None)
    ap.add_argument("--grad_accum", type=int, default=None)
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--weight_decay", type=float, default=None)
    ap.add_argument("--gradient_checkpointing", action="store_true")
    ap.add_argument("--checkpointing_policy", default="auto", choices=["auto", "reference"],
                    help="auto: checkpoint only when the activations would not fit in HBM (dpo_llama2.py default)")
    ap.add_argument("--no_gradient_checkpointing", action="store_true",
                    help="override a preset's checkpointing (the DPO preset's replicas fit 288 GB without it)")
    ap.add_argument("--fuse_accum", type=int, default=1, help="gradient-accumulation fusion (ops/linear.py)")
    ap.add_argument("--max_grad_norm", type=float, default=1.0)
    ap.add_argument("--exchange", default="a2a", help="allgather | a2a | ref_int64")
    ap.add_argument("--bucket_mb", type=float, default=None,
                    help="vote bucket size in MB (default: automatic, >= 4 buckets of 1-32 MB at W > 1)")
    ap.add_argument("--impl", default="native", choices=["native", "reference"])
    ap.add_argument("--fused", default="auto", choices=["auto", "torch", "hip"])
    ap.add_argument("--dropout", type=float, default=None, help="override GPT-2 dropout (default 0.1)")
    ap.add_argument("--load_in_4bit", action="store_true",
                    help="frozen base weights in 4-bit NF4 (the reference's bitsandbytes base, models/quant.py)")
    ap.add_argument("--profile_dir", default=None)
    ap.add_argument("--rocm_fa", default=None, help="PyTorch SDPA flash library on ROCm: ck | aotriton")
    ap.add_argument("--device", default="auto", choices=["auto", "cuda", "cpu"],
                    help="auto: cuda when a GPU is visible (cpu + gloo: plumbing rehearsal of the multi-rank path)")
    ap.add_argument("--no_phase_times", action="store_true", help="do not record per-phase HIP events")
    ap.add_argument("--elastic_timeout", type=float, default=None,
                    help="run the vote as guarded, store-committed collectives (worker-dropout mode) to measure its cost")
    ap.add_argument("--data", default="random", choices=["random", "markov"],
                    help="random token ids (throughput) | a learnable Markov-chain corpus (learning curves)")
    ap.add_argument("--loss_log", default=None,
                    help="learning-curve mode: run --steps steps untimed, rank 0 writes one JSON line per step here")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend; gloo (with ranks sharing GPUs) only to rehearse the multi-rank "
                         "path on a 1-GPU box -- RCCL refuses two ranks on one device")
    a = ap.parse_args()
    for k, v in PRESETS[a.task].items():
        if getattr(a, k, None) is None:
            setattr(a, k, v)
    # an explicit --gradient_checkpointing is honoured; a preset's (DPO) goes through --checkpointing_policy
    a.ckpt_explicit = bool(a.gradient_checkpointing)
    a.gradient_checkpointing = (a.gradient_checkpointing or bool(getattr(a, "grad_ckpt", False))) and \
        not a.no_gradient_checkpointing
    return a


RCCL_ENV_DEFAULTS = {
    # the host driver only supports dmabuf IPC (RCCL / cross-process CUDA tensors fail without it)
    "HSA_ENABLE_IPC_MODE_LEGACY": "0",
    # RCCL's streams at high priority: the vote collectives are issued while the
    # compute stream still has the next bucket's encode / apply queued
    "TORCH_NCCL_HIGH_PRIORITY": "1",
}
_ENV_PREFIXES = ("NCCL_", "RCCL_", "TORCH_NCCL_", "HSA_", "HIP_", "GPU_MAX_HW_QUEUES", "OMP_NUM_THREADS")


def comm_env() -> dict:
    """The collective-relevant environment this rank ran with (reported in the JSON)."""
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith(_ENV_PREFIXES)}


def _rccl_version():
    try:
        v = torch.cuda.nccl.version()
        return ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
    except Exception:  # noqa: BLE001
        return None


def resolve_device(args) -> str:
    if args.device != "auto":
        return args.device
    return "cuda" if torch.cuda.device_count() > 0 else "cpu"


def launch_local(args) -> int:
    """``--gpus N`` without a launcher: start N rank processes (one per GPU,
    127.0.0.1 rendezvous, store hosted by this parent) and relay rank 0's JSON
    line; any rank failing fails the run.  This parent makes no HIP call at
    all: GPUs are counted through amdsmi or the KFD sysfs topology
    (utils/devices.py), never ``hipGetDeviceCount`` -- so no HIP context is
    ever forked or exec'd over; the children are fresh interpreters and
    validate their own device (``setup_dist``)."""
    from distributed_lion_pytorch_amd.launch import run
    from distributed_lion_pytorch_amd.utils.devices import visible_gpu_count

    device = args.device
    if device != "cpu":
        n = visible_gpu_count()
        if n is None and os.path.exists("/dev/kfd"):
            print("bench.py: cannot count the GPUs without a HIP call (amdsmi and /sys/class/kfd both failed); "
                  "run under torchrun, or pass --device cpu", file=sys.stderr)
            return 2
        n = n or 0
        if device == "auto":
            device = "cuda" if n > 0 else "cpu"
        if device == "cuda" and args.backend == "nccl" and n < args.gpus:
            print(f"bench.py: --gpus {args.gpus} but only {n} GPU(s) visible; refusing to report a smaller run",
                  file=sys.stderr)
            return 2
    argv = list(sys.argv[1:])
    if args.device == "auto":  # the children use the parent's answer (no second detection)
        argv += ["--device", device]
    env = dict(os.environ, DLION_BENCH_LAUNCHER="bench.py")
    return run([sys.executable, os.path.abspath(__file__)] + argv, args.gpus, max_failures=0,
               quiet_ranks=True, env=env)


def setup_dist(args):
    env_world = os.environ.get("WORLD_SIZE")
    world = int(env_world) if env_world is not None else 1
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a dp{world} run "
                         f"as {args.gpus} GPUs")
    device = resolve_device(args)
    if device == "cuda":
        n_dev = torch.cuda.device_count()
        if args.backend == "gloo":
            local = local % max(1, n_dev)  # gloo rehearsal: ranks may share a GPU
        elif local >= n_dev:
            raise SystemExit(f"bench.py: rank {rank} wants cuda:{local} but only {n_dev} GPU(s) are visible")
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        if args.backend == "nccl" and world > 1:
            raise SystemExit("bench.py: --device cpu needs --backend gloo")
        dev = torch.device("cpu")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.backend == "nccl":
            for k, v in RCCL_ENV_DEFAULTS.items():
                os.environ.setdefault(k, v)
            if args.elastic_timeout is not None:  # the elastic path aborts communicators itself
                os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "0")
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
    return world, rank, dev


def build_native(args, dev):
    from distributed_lion_pytorch_amd.models.registry import build_model, load_config
    from distributed_lion_pytorch_amd.ops import fused

    fused.set_impl(args.fused)
    cfg = load_config(args.model)
    if args.dropout is not None and cfg.model_type == "gpt2":
        cfg.resid_pdrop = cfg.embd_pdrop = cfg.attn_pdrop = args.dropout
    torch.manual_seed(0)
    with torch.device(dev):  # materialise weights on the GPU directly (7B: no host round trip)
        model = build_model(cfg, native=True).to(dtype=torch.bfloat16)
    ref_model = None
    if args.task == "dpo":
        import copy

        ref_model = copy.deepcopy(model).eval()
        for p in ref_model.parameters():
            p.requires_grad_(False)
    if args.load_in_4bit:
        from distributed_lion_pytorch_amd.models.quant import QuantConfig, quantize_model

        quantize_model(model, QuantConfig(bnb_4bit_compute_dtype=torch.bfloat16))
        if ref_model is not None:
            quantize_model(ref_model, QuantConfig(bnb_4bit_compute_dtype=torch.bfloat16))
        torch.cuda.empty_cache()
    if args.lora:
        from distributed_lion_pytorch_amd.models.lora import LoraConfig, inject_lora

        inject_lora(model, LoraConfig(**args.lora))
        model.to(device=dev, dtype=torch.bfloat16)
    if args.gradient_checkpointing:
        # the DPO preset's reference setting; "auto" (dpo_llama2.py's default policy) keeps the
        # activations when they fit in HBM (trainer/memory.py)
        from distributed_lion_pytorch_amd.trainer.memory import should_checkpoint

        tokens = args.micro_batch * (2 if args.task == "dpo" else 1) * args.seq_len
        policy = "reference" if args.ckpt_explicit else args.checkpointing_policy
        args.gradient_checkpointing = should_checkpoint(True, policy, cfg, tokens, model, ref_model)
    if args.gradient_checkpointing:
        model.gradient_checkpointing_enable()
    broadcast_parameters(model)
    opt = Lion([p for p in model.parameters() if p.requires_grad], lr=args.lr, weight_decay=args.weight_decay,
               exchange=args.exchange, bucket_mb=args.bucket_mb, elastic_timeout=args.elastic_timeout)
    args.ref_model = ref_model  # not a submodule: stays out of the parameter counts
    return model, opt, cfg


def build_reference(args, dev):
    """HF GPT2LMHeadModel + the reference optimizer algorithm (per-tensor
    int64 all_gather, ATen ops) -- the reference's behaviour on MI355X."""
    import transformers

    from distributed_lion_pytorch_amd.ops import reference as ref

    cfg = gpt2_config(args.model)
    if args.dropout is not None:
        cfg.resid_pdrop = cfg.embd_pdrop = cfg.attn_pdrop = args.dropout
    # the same initial weights as the native run (same seed, same builder; HF checkpoint layout)
    from distributed_lion_pytorch_amd.models.registry import build_model

    torch.manual_seed(0)
    with torch.device(dev):
        # from a copy: building the native model sets the config's attention
        # implementation to "eager", which would send HF's model to eager
        # attention instead of its default SDPA (what the reference's run_clm gets)
        init = build_model(copy.deepcopy(cfg), native=True).to(dtype=torch.bfloat16).state_dict()
    model = transformers.GPT2LMHeadModel(cfg).to(device=dev, dtype=torch.bfloat16)
    missing = model.load_state_dict(init, strict=False)
    assert not [k for k in missing.missing_keys if "attn.bias" not in k and "masked_bias" not in k], missing
    del init
    broadcast_parameters(model)

    class RefLion(torch.optim.Optimizer):
        def __init__(self, params, lr, weight_decay):
            super().__init__(params, dict(lr=lr, betas=(0.9, 0.99), weight_decay=weight_decay))

        @torch.no_grad()
        def step(self):
            distributed = dist.is_initialized() and dist.get_world_size() > 1
            for g in self.param_groups:
                for p in g["params"]:
                    if p.grad is None:
                        continue
                    st = self.state[p]
                    if not st:
                        st["exp_avg"] = torch.zeros_like(p)
                    args_ = (p, p.grad, st["exp_avg"], g["lr"], g["weight_decay"], *g["betas"])
                    if distributed:
                        ref.update_fn_distributed(*args_, wire_dtype=torch.int64)
                    else:
                        ref.update_fn(*args_)

    opt = RefLion(model.parameters(), args.lr, args.weight_decay)
    return model, opt, cfg


def main():
    args = parse()
    if os.environ.get("WORLD_SIZE") is None and args.gpus > 1:
        sys.exit(launch_local(args))  # one process per GPU, started here (no torchrun needed)
    if resolve_device(args) == "cpu" and args.backend == "nccl":
        args.backend = "gloo"
    world, rank, dev = setup_dist(args)
    if args.rocm_fa:
        torch.backends.cuda.preferred_rocm_fa_library(args.rocm_fa)
    build = build_native if args.impl == "native" else build_reference
    model, opt, cfg = build(args, dev)
    n_params = sum({p.data_ptr(): p.numel() for p in model.parameters()}.values())
    n_params += sum(m.in_features * m.out_features for m in model.modules() if hasattr(m, "qweight"))  # 4-bit bases
    n_train = sum({p.data_ptr(): p.numel() for p in model.parameters() if p.requires_grad}.values())

    if args.task == "dpo":
        from distributed_lion_pytorch_amd.trainer.dpo import dpo_loss, sequence_logps

        ref = args.ref_model

        def loss_fn(m, b):
            ids, labels = b["input_ids"], b["labels"]
            n = ids.shape[0] // 2
            logp = sequence_logps(m, ids, labels)
            with torch.no_grad():
                ref_logp = sequence_logps(ref, ids, labels)
            return dpo_loss(logp[:n], logp[n:], ref_logp[:n], ref_logp[n:], args.dpo_beta)[0]
    elif args.impl == "native":
        loss_fn = None
    else:
        def loss_fn(m, b):
            return m(input_ids=b["input_ids"], labels=b["labels"]).loss

    step = TrainStep(model, opt, grad_accum=args.grad_accum, max_grad_norm=args.max_grad_norm, loss_fn=loss_fn,
                     fuse_grad_accumulation=bool(args.fuse_accum))
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + rank)

    seqs_per_mb = args.micro_batch * (2 if args.task == "dpo" else 1)  # DPO: chosen + rejected

    if args.data == "markov":
        # learnable synthetic corpus (the loss can fall well below ln V): every
        # token is followed by succ[token] with probability 0.75, else by a
        # uniformly random token; the table is the same on every rank
        mk = torch.Generator(device=dev).manual_seed(99)
        succ = torch.randperm(cfg.vocab_size, device=dev, generator=mk)

    def sample_ids():
        if args.data != "markov":
            return torch.randint(0, cfg.vocab_size, (seqs_per_mb, args.seq_len), device=dev, generator=gen)
        rnd = torch.randint(0, cfg.vocab_size, (seqs_per_mb, args.seq_len), device=dev, generator=gen)
        follow = torch.rand(seqs_per_mb, args.seq_len, device=dev, generator=gen) < 0.75
        out = rnd.clone()
        for t in range(1, args.seq_len):
            out[:, t] = torch.where(follow[:, t], succ[out[:, t - 1]], rnd[:, t])
        return out

    def batches():
        for _ in range(args.grad_accum):
            ids = sample_ids()
            labels = ids
            if args.task == "dpo":  # prompt half masked out of the log-likelihood, as the DPO collator does
                labels = ids.clone()
                labels[:, : args.seq_len // 2] = -100
            yield {"input_ids": ids, "labels": labels}

    loss_log = open(args.loss_log, "w") if args.loss_log and rank == 0 else None
    if loss_log is not None:  # learning-curve mode: data is generated before timing
        for i in range(args.steps):
            data = list(batches())
            loss = step(iter(data))
            loss_log.write(json.dumps({"step": i, "loss": float(loss), "world": world, "impl": args.impl}) + "\n")
            loss_log.flush()
        loss_log.close()
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    if args.loss_log:  # other ranks in learning-curve mode: same steps, no log
        for _ in range(args.steps):
            step(iter(list(batches())))
        dist.barrier()
        dist.destroy_process_group()
        return
    for _ in range(args.warmup):
        step(batches())
    if hasattr(opt, "stats"):
        opt.stats(reset=True)  # wire counters cover the timed steps only
    phases = None if args.no_phase_times else PhaseTimer(dev)
    step.set_timer(phases)
    timer = StepTimer(dev)
    prof = None
    if args.profile_dir and rank == 0:
        prof = torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU,
                                                  torch.profiler.ProfilerActivity.CUDA], record_shapes=True)
        prof.__enter__()
    with timer:
        for _ in range(args.steps):
            loss = step(batches())
    if prof is not None:
        prof.__exit__(None, None, None)
        os.makedirs(args.profile_dir, exist_ok=True)
        prof.export_chrome_trace(os.path.join(args.profile_dir, "trace.json"))
        with open(os.path.join(args.profile_dir, "top_kernels.txt"), "w") as f:
            f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=40))
        with open(os.path.join(args.profile_dir, "top_ops_by_shape.txt"), "w") as f:
            f.write(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=80,
                                                                          max_name_column_width=40,
                                                                          max_shapes_column_width=90))
    step.set_timer(None)
    from distributed_lion_pytorch_amd.ops.fused import check_index_errors

    check_index_errors(blocking=True)
    phase_ms = phases.summary() if phases is not None else {}
    names = sorted(phase_ms)
    vec = torch.tensor([timer.elapsed] + [phase_ms[k] for k in names], dtype=torch.float64, device=dev)
    if world > 1:  # slowest rank (the contract's MAX over ranks), and its phase times
        allv = [torch.zeros_like(vec) for _ in range(world)]
        dist.all_gather(allv, vec)
        vec = max(allv, key=lambda v: float(v[0]))
        per_rank_ms = [round(1000.0 * float(v[0]) / args.steps, 3) for v in allv]
    else:
        per_rank_ms = [round(1000.0 * timer.elapsed / args.steps, 3)]
    elapsed = float(vec[0])
    phase_ms = {k: round(float(vec[i + 1]), 3) for i, k in enumerate(names)}
    tokens = world * args.grad_accum * seqs_per_mb * args.seq_len * args.steps
    tps = tokens / elapsed
    ms = 1000.0 * elapsed / args.steps
    stats = opt.stats() if hasattr(opt, "stats") else {}
    exchange = args.exchange if args.impl == "native" else "ref_int64"
    wire = wire_bytes_per_step(n_train, world, exchange)
    wire_meas = {k: stats.get(k, 0) // max(1, args.steps) for k in ("wire_bytes_sent", "wire_bytes_recv",
                                                                       "collectives")}
    if rank == 0:
        out = {
            "metric": args.metric,
            "value": round(tps, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": f"synthetic (random token ids of the {args.model} vocab), random-init weights",
            "config": {
                "model": f"{args.model} ({n_params / 1e6:.1f}M params)",
                "trainable_params": n_train,
                "lora": args.lora,
                "base_weights": "nf4 (4-bit, frozen)" if args.load_in_4bit else "bf16",
                "global_batch": world * args.grad_accum * args.micro_batch,
                "task": args.task,
                "gradient_checkpointing": bool(args.gradient_checkpointing),
                "micro_batch": args.micro_batch,
                "grad_accum": args.grad_accum,
                "seq_len": args.seq_len,
                "parallelism": f"dp{world}",
                "optimizer": f"distributed Lion (majority vote), lr {args.lr:g}, wd {args.weight_decay:g}",
                "exchange": exchange,
                "impl": args.impl,
                "elastic_timeout": args.elastic_timeout,
            },
            "wire_bytes_per_step_per_rank": wire_meas["wire_bytes_sent"] if world > 1 else 0,
            "wire_bytes_per_step_per_rank_measured": wire_meas,
            "wire_bytes_per_step_per_rank_analytic": wire,
            "phase_ms_per_step": phase_ms,
            "ms_per_step_per_rank": per_rank_ms,
            "device": str(dev),
            "backend": args.backend if world > 1 else None,
            "launcher": os.environ.get("DLION_BENCH_LAUNCHER", "torchrun" if world > 1 else "none"),
            "comm_env": comm_env() if world > 1 else {},
            "rccl_version": _rccl_version() if world > 1 and args.backend == "nccl" else None,
            "bf16_allreduce_bytes_per_step_per_rank": 0 if world == 1 else int(2 * (world - 1) / world * 2 * n_train),
            "loss": round(float(loss.item()), 4),
            "optimizer_stats": stats,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
