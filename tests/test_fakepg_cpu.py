"""API-level tests of the vote exchange at the production world sizes (W = 4, 8)
without any transport: torch's fake process group ("Fake PG").
Collectives complete instantly and move no data, so these tests pin what does
not depend on the peers' votes -- strategy selection, bucket/shard alignment
for W ranks, collective counts and wire-byte accounting per step -- for the
world sizes the 8-GPU scaling run uses, on CPU."""
import multiprocessing as mp
import traceback

import pytest
import torch


def _fake_world(q, world, rank, exchange, bucket_mb, steps):
    try:
        import torch.distributed as dist
        from torch.testing._internal.distributed.fake_pg import FakeStore

        from distributed_lion_pytorch_amd import Lion
        from distributed_lion_pytorch_amd.models.gpt2 import GPT2LMHeadModel, gpt2_config
        from distributed_lion_pytorch_amd.parallel.exchange import wire_bytes_per_step

        torch.set_num_threads(1)
        dist.init_process_group("fake", store=FakeStore(), rank=rank, world_size=world)
        cfg = gpt2_config("gpt2-tiny")
        torch.manual_seed(0)
        model = GPT2LMHeadModel(cfg)
        kw = {} if exchange is None else {"exchange": exchange}  # None: the constructor default
        opt = Lion(model.parameters(), lr=1e-3, weight_decay=0.1, bucket_mb=bucket_mb, backend="torch",
                   verify_consistency=False, **kw)
        ids = torch.randint(0, cfg.vocab_size, (2, 16))
        per_step = []
        for _ in range(steps):
            opt.zero_grad()
            model(ids, labels=ids)["loss"].backward()
            opt.step()
            per_step.append(opt.stats())
        plan = opt.plan
        out = {
            "stats": per_step,
            "bucket_bytes": [b.nbytes for b in plan.buckets],
            "total_bytes": plan.total_bytes,
            "numel": sum(s.numel for s in plan.segments),
            "analytic": wire_bytes_per_step(sum(s.numel for s in plan.segments), world, opt.exchange_name),
            "finite": all(torch.isfinite(p).all().item() for p in model.parameters()),
            "exchange_cls": type(opt._exchange).__name__,
        }
        dist.destroy_process_group()
        q.put(("ok", out))
    except Exception:  # pragma: no cover - reported to the parent
        q.put(("err", traceback.format_exc()))


def run_fake(world, rank, exchange, bucket_mb=32.0, steps=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_fake_world, args=(q, world, rank, exchange, bucket_mb, steps))
    p.start()
    try:
        status, out = q.get(timeout=240)
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    if status != "ok":
        raise RuntimeError(out)
    return out


@pytest.mark.parametrize("world,rank", [(8, 0), (8, 7), (4, 2)])
def test_a2a_shards_align_and_wire_bytes(world, rank):
    out = run_fake(world, rank, "a2a", bucket_mb=0.005)
    assert out["exchange_cls"] == "AllToAllExchange"
    assert out["finite"]
    assert len(out["bucket_bytes"]) > 1  # small buckets: several collectives per step
    for nb in out["bucket_bytes"]:
        assert nb % world == 0, "a2a shard must split evenly over the ranks"
        assert (nb // world) % 4 == 0, "shards stay dword-aligned for the vote kernels"
    assert sum(out["bucket_bytes"]) == out["total_bytes"] >= (out["numel"] + 7) // 8
    nbk = len(out["bucket_bytes"])
    for s in out["stats"]:
        # one all_to_all + one 1-bit all_gather per bucket (tie rule 'negative')
        assert s["collectives"] == 2 * nbk
        assert s["wire_bytes_recv"] == 2 * (world - 1) * out["total_bytes"] // world
        assert s["wire_bytes_sent"] == s["wire_bytes_recv"]
        # padding to the 2048-bit regions is the only difference from the analytic count
        assert out["analytic"] <= s["wire_bytes_recv"] <= out["analytic"] + 2 * (world - 1) * 256 * nbk
        # reference wire: 1 byte per parameter per peer; here >= 4x less even with a
        # tiny model's per-tensor padding
        assert 4 * s["wire_bytes_recv"] < (world - 1) * out["numel"]


def test_reference_signature_defaults_to_a2a():
    """``Lion(model.parameters(), lr=...)`` -- exactly the reference usage
    (/root/reference/README.md:8-15) -- gets the vote-RS/AG exchange, not the
    4x-more-bytes all-gather."""
    out = run_fake(4, 1, None, steps=1)
    assert out["exchange_cls"] == "AllToAllExchange"
    assert out["stats"][0]["wire_bytes_recv"] == 2 * 3 * out["total_bytes"] // 4


@pytest.mark.parametrize("exchange", ["allgather", "ref_int64"])
def test_allgather_family_wire_bytes_w8(exchange):
    world = 8
    out = run_fake(world, 3, exchange, bucket_mb=32.0, steps=1)
    s = out["stats"][0]
    if exchange == "allgather":
        assert out["exchange_cls"] == "AllGatherExchange"
        assert s["wire_bytes_recv"] == (world - 1) * out["total_bytes"]
        assert s["collectives"] == len(out["bucket_bytes"])
    else:
        # reference wire: one int64 per packed byte, one blocking all_gather per tensor
        assert out["exchange_cls"] == "RefInt64Exchange"
        assert s["wire_bytes_recv"] >= (world - 1) * out["numel"]
        assert s["collectives"] > len(out["bucket_bytes"])
    assert out["finite"]


def _fake_all_dropped(q, world):
    try:
        import torch.distributed as dist
        from torch.testing._internal.distributed.fake_pg import FakeStore

        from distributed_lion_pytorch_amd import Lion

        torch.set_num_threads(1)
        dist.init_process_group("fake", store=FakeStore(), rank=0, world_size=world)
        p = torch.nn.Parameter(torch.randn(64, 64))
        opt = Lion([p], lr=1e-3, exchange="a2a", backend="torch", verify_consistency=False)
        p.grad = torch.randn_like(p)
        opt.drop_workers(range(world))
        try:
            opt.step()
            q.put(("err", "step with every worker dropped did not raise"))
        except ValueError as e:
            q.put(("ok", str(e)))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        q.put(("err", traceback.format_exc()))


def test_dropping_every_worker_is_refused():
    """With no live voter the allgather and a2a exchanges would disagree (0 vs
    -1 delta), so the optimizer refuses the configuration instead."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    proc = ctx.Process(target=_fake_all_dropped, args=(q, 4))
    proc.start()
    try:
        status, out = q.get(timeout=240)
    finally:
        proc.join(timeout=30)
        if proc.is_alive():
            proc.kill()
    assert status == "ok", out
    assert "dropped" in out


def test_auto_buckets_pipeline_gpt2_at_w_gt_1():
    """bucket_mb=None: GPT-2 small's 15.6 MB of sign planes become >= 4
    buckets of >= 1 MB at W > 1 (encode i+1 overlaps exchange i); one bucket
    at W = 1; Llama-3-8B-sized planes are capped at 32 MB per bucket."""
    from distributed_lion_pytorch_amd import Lion
    from distributed_lion_pytorch_amd.models.registry import build_model, load_config
    from distributed_lion_pytorch_amd.optim.plan import FlatPlan

    with torch.device("meta"):
        model = build_model(load_config("gpt2"), native=True)
    ps = list(model.parameters())
    opt = Lion(ps)
    entries = [(p, 0) for p in ps]
    for w, lo, hi in ((1, 1, 1), (2, 4, 8), (8, 4, 8)):
        plan = FlatPlan(entries, world=w, bucket_bytes=opt._bucket_bytes(entries, w), device=torch.device("cpu"))
        assert lo <= len(plan.buckets) <= hi, (w, [b.nbytes for b in plan.buckets])
        if w > 1:
            assert min(b.nbytes for b in plan.buckets) >= 1 << 20
    big = [(torch.empty(128256 * 4096 // 8, device="meta"), 0)] * 64  # 4.2B params: 525 MB of bits
    assert opt._bucket_bytes(big, 8) == 32 << 20
    assert Lion(ps, bucket_mb=2.0)._bucket_bytes(entries, 8) == 2 << 20
    # host-side collectives (gloo): the fewest buckets; an explicit size still wins
    assert opt._bucket_bytes(entries, 8, backend="gloo") == 32 << 20
    assert Lion(ps, bucket_mb=2.0)._bucket_bytes(entries, 8, backend="gloo") == 2 << 20


def _clm_buckets(q, world):
    """run_clm's own argument parsing + build_lion on a 2-rank fake group:
    the default (automatic) bucket size at GPT-2 small."""
    try:
        import os
        import sys

        import torch.distributed as dist
        from torch.testing._internal.distributed.fake_pg import FakeStore

        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import run_clm
        from distributed_lion_pytorch_amd.models.gpt2 import GPT2LMHeadModel, gpt2_config
        from transformers import HfArgumentParser

        torch.set_num_threads(2)
        dist.init_process_group("fake", store=FakeStore(), rank=1, world_size=world)
        parser = HfArgumentParser((run_clm.ModelArguments, run_clm.DataTrainingArguments,
                                   run_clm.AsyncTrainingArguments))
        _, _, targs = parser.parse_args_into_dataclasses(
            args=["--output_dir", "/tmp/unused", "--use_cpu", "--lion", "--async_grad", "--report_to", "none"])
        model = GPT2LMHeadModel(gpt2_config("gpt2")).to(torch.bfloat16)
        opt = run_clm.build_lion(model, targs)
        opt.backend = "torch"
        opt.verify_consistency = False
        for p in model.parameters():
            p.grad = torch.zeros_like(p)
        opt.step()
        plan = opt.plan
        q.put(("ok", {"default_bucket_mb": targs.lion_bucket_mb, "buckets": [b.nbytes for b in plan.buckets],
                      "backend": dist.get_backend()}))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover - reported to the parent
        q.put(("err", traceback.format_exc()))


def test_run_clm_default_buckets_pipeline_at_w2():
    """the HF entrypoints used to pin 32 MB buckets (GPT-2
    went out as ONE bucket and never pipelined at W > 1).  With the default
    (automatic) size, run_clm's Lion splits GPT-2 small into >= 4 buckets on a
    non-gloo backend."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_clm_buckets, args=(q, 2))
    p.start()
    try:
        status, out = q.get(timeout=300)
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert status == "ok", out
    assert out["default_bucket_mb"] is None and out["backend"] != "gloo"
    assert len(out["buckets"]) >= 4, out["buckets"]
    assert max(out["buckets"]) <= 32 << 20
