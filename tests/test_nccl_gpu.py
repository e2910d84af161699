"""The RCCL-only code paths on ONE GPU (a 1-rank ``nccl`` group is legal).

Every multi-rank test elsewhere runs over gloo (RCCL refuses two ranks on one
device), so the calls the 8-GPU run makes under ``nccl`` are exercised here on
the single GPU a gpurun box has:

* ``init_process_group("nccl", device_id=...)`` (bench.py / dropout_stress.py);
* uint8 ``all_to_all_single`` / ``all_gather_into_tensor`` on *slices* of the
  flat send/recv buffers, sync and async (parallel/exchange.py);
* the layout-digest all-reduce on the device (Lion._check_consistency);
* the coalesced parameter broadcast (trainer/engine.py broadcast_parameters);
* a full Lion vote step through every exchange strategy, HIP kernels vs the
  PyTorch executor (identical parameters);
* ``new_group(..., use_local_synchronization=True)``, collectives on it, and
  destroying the subgroup before the default group (parallel/elastic.py).

What a 1-rank group cannot show (peers' data, link bandwidth, a peer dying
inside a collective) is listed in docs/DESIGN.md "RCCL audit".
Each scenario runs in a fresh interpreter (a process group per process)."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PRELUDE = textwrap.dedent("""
    import json, os, sys
    import torch, torch.distributed as dist
    sys.path.insert(0, sys.argv[1])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"
    out = {}
""")
EPILOGUE = textwrap.dedent("""
    torch.cuda.synchronize()
    dist.destroy_process_group()
    print("RESULT " + json.dumps(out), flush=True)
""")


def _run(body: str, timeout: int = 150) -> dict:
    from dist_utils import free_port

    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()),
               RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    code = PRELUDE + textwrap.dedent(body) + EPILOGUE
    r = subprocess.run([sys.executable, "-c", code, ROOT], capture_output=True, text=True, timeout=timeout, env=env,
                       cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")]
    assert line, r.stdout[-2000:]
    return json.loads(line[-1][len("RESULT "):])


def test_uint8_collectives_on_buffer_slices():
    out = _run("""
        src = (torch.arange(8192, device=dev) * 7 % 251).to(torch.uint8)
        big = torch.zeros(8192, dtype=torch.uint8, device=dev)
        # all_to_all_single between slices at non-zero offsets (the exchange's bucket views)
        dist.all_to_all_single(big[256:256 + 2048], src[1024:1024 + 2048])
        out["a2a"] = torch.equal(big[256:256 + 2048], src[1024:1024 + 2048])
        w = dist.all_to_all_single(big[4096:4096 + 1024], src[0:1024], async_op=True)
        w.wait()
        out["a2a_async"] = torch.equal(big[4096:4096 + 1024], src[0:1024])
        g = torch.zeros(4096, dtype=torch.uint8, device=dev)
        w = dist.all_gather_into_tensor(g[512:512 + 1536], src[2048:2048 + 1536], async_op=True)
        w.wait()
        out["ag_async"] = torch.equal(g[512:512 + 1536], src[2048:2048 + 1536])
        t = torch.tensor([5, -5], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        out["allreduce_max"] = t.tolist()
    """)
    assert out == {"a2a": True, "a2a_async": True, "ag_async": True, "allreduce_max": [5, -5]}


def test_broadcast_and_consistency_digest_on_device():
    out = _run("""
        from distributed_lion_pytorch_amd import Lion
        from distributed_lion_pytorch_amd.optim.plan import FlatPlan
        from distributed_lion_pytorch_amd.trainer.engine import broadcast_parameters
        from distributed_lion_pytorch_amd.models.gpt2 import GPT2LMHeadModel, gpt2_config
        torch.manual_seed(0)
        model = GPT2LMHeadModel(gpt2_config("gpt2-tiny")).to(device=dev, dtype=torch.bfloat16)
        before = [p.detach().clone() for p in model.parameters()]
        broadcast_parameters(model)  # returns early at W=1: run its collective by hand as well
        flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
        dist.broadcast(flat, src=0)
        out["broadcast_equal"] = torch.equal(flat, torch.cat([b.reshape(-1) for b in before]))
        opt = Lion(model.parameters(), lr=1e-3)
        plan = FlatPlan([(p, 0) for p in model.parameters()], world=1)
        opt._check_consistency(plan)  # device all-reduce under nccl
        out["digest_ok"] = True
    """)
    assert out == {"broadcast_equal": True, "digest_ok": True}


@pytest.mark.parametrize("exchange", ["a2a", "allgather", "ref_int64"])
def test_lion_vote_step_over_rccl_hip_equals_torch(exchange):
    out = _run(f"""
        from distributed_lion_pytorch_amd import Lion
        from distributed_lion_pytorch_amd.models.gpt2 import GPT2LMHeadModel, gpt2_config
        res = {{}}
        for backend in ("hip", "torch"):
            torch.manual_seed(0)
            cfg = gpt2_config("gpt2-tiny")
            model = GPT2LMHeadModel(cfg).to(device=dev, dtype=torch.bfloat16)
            opt = Lion(model.parameters(), lr=1e-3, weight_decay=0.1, exchange="{exchange}", backend=backend,
                       bucket_mb=0.004)
            opt._force_vote = True
            g = torch.Generator(device=dev).manual_seed(3)
            for _ in range(3):
                ids = torch.randint(0, cfg.vocab_size, (2, 64), device=dev, generator=g)
                model(ids, labels=ids)["loss"].backward()
                opt.step()
                opt.zero_grad()
            torch.cuda.synchronize()
            res[backend] = torch.cat([p.detach().float().reshape(-1) for p in model.parameters()])
            st = opt.stats()
            out[backend + "_collectives"] = st["collectives"]
            out[backend + "_exchange"] = type(opt._exchange).__name__
        out["equal"] = torch.equal(res["hip"], res["torch"])
        out["n_buckets"] = len(opt.plan.buckets)
    """)
    assert out["equal"], out
    assert out["hip_collectives"] == out["torch_collectives"] > 0
    assert out["n_buckets"] > 1


def test_subgroup_local_sync_then_destroy():
    out = _run("""
        sub = dist.new_group(ranks=[0], use_local_synchronization=True)
        t = torch.ones(4, device=dev)
        dist.all_reduce(t, group=sub)
        x = torch.zeros(2048, dtype=torch.uint8, device=dev)
        dist.all_to_all_single(x, torch.full((2048,), 3, dtype=torch.uint8, device=dev), group=sub)
        out["sub_ok"] = bool(t.sum().item() == 4 and int(x.sum().item()) == 3 * 2048)
        dist.destroy_process_group(sub)
        t2 = torch.ones(2, device=dev)
        dist.all_reduce(t2)  # default group still works after the subgroup is gone
        out["default_ok"] = bool(t2.sum().item() == 2)
    """)
    assert out == {"sub_ok": True, "default_ok": True}


def test_elastic_abort_and_reinit_under_rccl():
    """The regroup path of parallel/elastic.py under RCCL: guarded collectives,
    then ``_abort_process_group`` (ncclCommAbort of every communicator) and a
    fresh default ``nccl`` group over the survivors' store prefix, then the
    Lion vote (guarded, store-committed) on the new group."""
    out = _run("""
        os.environ["TORCH_NCCL_ASYNC_ERROR_HANDLING"] = "0"
        from distributed_lion_pytorch_amd import Lion
        from distributed_lion_pytorch_amd.models.gpt2 import GPT2LMHeadModel, gpt2_config
        from distributed_lion_pytorch_amd.parallel.elastic import ElasticGroup
        el = ElasticGroup.get(30.0, grace_s=0.5)
        out["gather"] = el.all_gather(torch.arange(4, device=dev, dtype=torch.float32)).tolist()
        torch.manual_seed(0)
        cfg = gpt2_config("gpt2-tiny")
        model = GPT2LMHeadModel(cfg).to(device=dev, dtype=torch.bfloat16)
        opt = Lion(model.parameters(), lr=1e-3, weight_decay=0.1, elastic_timeout=30.0, bucket_mb=0.004)
        opt._force_vote = True
        ids = torch.randint(0, cfg.vocab_size, (2, 64), device=dev)
        for i in range(3):
            model(ids, labels=ids)["loss"].backward()
            opt.step()
            opt.zero_grad()
            if i == 0:
                old = dist.group.WORLD
                el.regroup({"where": "test"})  # abort every communicator, re-init the default group
                out["new_group"] = dist.group.WORLD is not old
                out["after"] = [dist.get_world_size(), dist.get_rank(), dist.get_backend()]
        x = torch.ones(3, device=dev)
        el.all_reduce(x)
        out["allreduce"] = x.tolist()
        torch.cuda.synchronize()
        out["finite"] = all(bool(torch.isfinite(p).all()) for p in model.parameters())
        st = opt.stats()
        out["events"] = len(st["dropout_events"])
        out["commits"] = st["elastic_commits"] >= 3
        out["executor"] = type(opt._executor).__name__
    """)
    assert out["gather"] == [0.0, 1.0, 2.0, 3.0]
    assert out["new_group"] and out["after"] == [1, 0, "nccl"]
    assert out["allreduce"] == [1.0, 1.0, 1.0] and out["finite"]
    assert out["events"] == 1 and out["commits"] and out["executor"] == "HipExecutor"
