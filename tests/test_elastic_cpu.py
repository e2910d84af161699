"""Real worker dropout at any instant (gloo, CPU).

A rank process SIGKILLs itself at a chosen optimizer step and phase
(DLION_FAULT=rank:step:phase, parallel/elastic.py): inside backward, after
the vote all-to-all was issued but before it completed, inside the 1-bit
all-gather, after the step was applied, or between steps.  The survivors must
detect it within the bounded wait, agree on the outcome through the store,
regroup into a new default group, re-vote the interrupted step among
themselves and keep bit-identical replicas -- in the native loop
(dropout_stress.py) and in the HF path (run_clm.py --lion_elastic_timeout).
Runs go through the failure-tolerant launcher (distributed_lion_pytorch_amd.launch),
whose store outlives any rank, rank 0 included."""
import json
import os
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist

from distributed_lion_pytorch_amd import Lion
from tests.dist_utils import run_world

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _launch(nproc, script_args, max_failures=1, env_extra=None, timeout=300):
    cmd = [sys.executable, "-m", "distributed_lion_pytorch_amd.launch", "--nproc", str(nproc), "--max_failures",
           str(max_failures)] + script_args
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.update(env_extra or {})
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)


def _stress(nproc, fault_args, steps=5):
    r = _launch(nproc, ["dropout_stress.py", "--model", "gpt2-tiny", "--device", "cpu", "--seq_len", "32",
                        "--micro_batch", "2", "--steps", str(steps), "--elastic_timeout", "120"] + fault_args,
                max_failures=2)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-2000:] + r.stderr[-3000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("phase,victim,nproc", [
    ("backward", 1, 3),
    ("after_launch", 2, 3),
    ("in_allgather", 1, 4),
    ("after_vote", 0, 3),  # rank 0 too: the store lives in the launcher
    ("before_step", 3, 4),
])
def test_dropout_at_phase(phase, victim, nproc):
    res = _stress(nproc, ["--drop_rank", str(victim), "--drop_step", "2", "--drop_phase", phase])
    survivors = [r for r in range(nproc) if r != victim]
    assert res["world_start"] == nproc and res["world_end"] == nproc - 1
    assert res["survivors"] == survivors and res["replicas_identical"], res
    ev = res["dropout_events"]
    assert len(ev) == 1 and ev[0]["dropped"] == [victim] and ev[0]["survivors"] == survivors
    # a death after the step-2 vote is applied is noticed in step 3's vote
    assert ev[0]["step"] == (3 if phase == "after_vote" else 2)
    assert [s["world"] for s in res["steps"]][-1] == nproc - 1 and len(res["steps"]) == 5
    # bounded by the launcher's death notice, not by the 120 s collective deadline
    # (round 3's GPU rehearsal stalled for the whole deadline: gloo never failed the wait)
    assert res["elastic_stall_s"] < 5.0, ev


def test_two_workers_drop_at_different_steps():
    r = _launch(4, ["dropout_stress.py", "--model", "gpt2-tiny", "--device", "cpu", "--seq_len", "32",
                    "--micro_batch", "2", "--steps", "6", "--elastic_timeout", "20", "--drop_rank", "-1",
                    "--elastic_grace", "60"],
                max_failures=2, env_extra={"DLION_FAULT": "1:2:after_launch,3:4:backward"})
    assert r.returncode == 0, r.stderr[-4000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')][0])
    assert res["world_end"] == 2 and res["survivors"] == [0, 2] and res["replicas_identical"]
    assert [e["dropped"] for e in res["dropout_events"]] == [[1], [3]]
    assert [e["step"] for e in res["dropout_events"]] == [2, 4]
    # the launcher's death notices end the membership wait at once: nowhere
    # near the 60 s check-in grace
    assert res["elastic_stall_s"] < 10.0, res["dropout_events"]


def test_death_notice_keys_agree():
    from distributed_lion_pytorch_amd import launch
    from distributed_lion_pytorch_amd.parallel import elastic

    assert (launch.DEATH_KEY, launch.DEATH_COUNT_KEY) == (elastic.DEATH_KEY, elastic.DEATH_COUNT_KEY)


def test_run_clm_survives_a_dropout(tmp_path):
    """HF path: the AsyncTrainer guards HF's own collectives (num_items gather,
    logging loss gather) and Lion's vote; a rank dying in backward leaves the
    survivors training, checkpointing and evaluating on the regrouped group."""
    out = str(tmp_path / "clm")
    args = ["run_clm.py", "--synthetic_data", "--synthetic_samples", "96", "--block_size", "32",
            "--per_device_train_batch_size", "2", "--gradient_accumulation_steps", "2", "--warmup_steps", "1",
            "--learning_rate", "1e-3", "--report_to", "none", "--use_cpu", "--logging_steps", "1",
            "--config_name", "gpt2-tiny", "--lion", "--async_grad", "--do_train", "--max_steps", "5",
            "--output_dir", out, "--ddp_backend", "gloo", "--lion_elastic_timeout", "20", "--save_steps", "4"]
    r = _launch(3, args, env_extra={"DLION_FAULT": "1:2:backward"})
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-4000:]
    recs = [json.loads(x) for x in open(os.path.join(out, "metrics.jsonl"))]
    last = [x for x in recs if "replicas_identical" in x]
    assert last and last[-1]["replicas_identical"] == 1.0 and last[-1]["world_end"] == 2.0
    steps = [x["step"] for x in recs if "loss" in x]
    assert max(steps) == 5
    lion = [x["lion"] for x in recs if "lion" in x]
    assert lion[-1]["world"] == 2 and lion[-1]["dropout_events"][0]["dropped"] == [1]
    ck = os.path.join(out, "checkpoint-4")
    files = set(os.listdir(ck))
    # per-rank momentum files are named in the regrouped world (dense ranks 0, 1 of 2)
    assert {"rank0-of-2-optimizer.pt", "rank1-of-2-optimizer.pt", "model.safetensors"} <= files
    assert os.path.isfile(os.path.join(out, "model.safetensors"))


# ------------------------------------------------------- no failure: transparent
def _train(rank, world, exchange, steps):
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Tanh(), torch.nn.Linear(32, 4))
    opt = Lion(model.parameters(), lr=1e-2, weight_decay=0.1, exchange=exchange, elastic_timeout=10.0,
               backend="torch")
    gen = torch.Generator().manual_seed(100 + rank)
    m2 = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Tanh(), torch.nn.Linear(32, 4))
    m2.load_state_dict(model.state_dict())
    ref = Lion(m2.parameters(), lr=1e-2, weight_decay=0.1, exchange=exchange, backend="torch")
    for _ in range(steps):
        x = torch.randn(8, 16, generator=gen)
        for m, o in ((model, opt), (m2, ref)):
            o.zero_grad()
            m(x).pow(2).mean().backward()
            o.step()
    st = opt.stats()
    same = all(torch.equal(a, b) for a, b in zip(model.parameters(), m2.parameters()))
    t = torch.tensor([float(rank)])
    dist.all_reduce(t)
    return {"same_as_plain": same, "events": st["dropout_events"], "world": st["world"], "commits": st["elastic_commits"],
            "sum": float(t)}


def _train_multibucket(rank, world, fault, steps):
    """4 tensors, one bucket each (256-byte buckets); ``fault`` set: rank 1's
    launch of bucket 1 raises at step 2 (nobody dies: all three regroup and
    re-vote that step from their send buffers)."""
    if fault:
        os.environ["DLION_FAULT"] = "1:2:raise_in_launch"
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Tanh(), torch.nn.Linear(32, 4))
    opt = Lion(model.parameters(), lr=1e-2, weight_decay=0.1, exchange="a2a", elastic_timeout=20.0,
               backend="torch", bucket_mb=256 / (1 << 20))
    gen = torch.Generator().manual_seed(100 + rank)
    for _ in range(steps):
        x = torch.randn(8, 16, generator=gen)
        opt.zero_grad()
        model(x).pow(2).mean().backward()
        opt.step()
    st = opt.stats()
    return {"params": [p.detach().clone() for p in model.parameters()],
            "moms": [opt.state[p]["exp_avg"].clone() for p in model.parameters()],
            "events": st["dropout_events"], "n_buckets": st["n_buckets"]}


def test_launch_error_at_later_bucket_encodes_every_bucket():
    """a launch failing at bucket i>0 must not leave buckets i+1..
    unencoded on that rank (stale sign planes in the survivors' re-vote, a
    momentum that skips the step).  The regrouped re-vote must equal the plain
    vote bit for bit, parameters and momenta."""
    plain = run_world(_train_multibucket, 3, False, 4)
    faulty = run_world(_train_multibucket, 3, True, 4)
    assert faulty[0]["n_buckets"] >= 3, faulty[0]["n_buckets"]
    for r in range(3):
        assert len(faulty[r]["events"]) == 1 and faulty[r]["events"][0]["step"] == 2
        assert faulty[r]["events"][0]["survivors"] == [0, 1, 2]
        for a, b in zip(plain[r]["params"] + plain[r]["moms"], faulty[r]["params"] + faulty[r]["moms"]):
            assert torch.equal(a, b)


@pytest.mark.parametrize("exchange", ["a2a", "allgather"])
def test_no_dropout_elastic_equals_plain(exchange):
    res = run_world(_train, 3, exchange, 4)
    for r in res:
        assert r["same_as_plain"], "guarded vote must give the plain vote's result bit for bit"
        assert r["events"] == [] and r["world"] == 3 and r["commits"] >= 4
    assert res[0]["sum"] == 3.0


def _sft_corpus(tmp_path, n):
    rows = [{"question": f"q{i:04d} " + "what is this " * 3, "response_j": "an answer " * 8,
             "response_k": "other " * 8} for i in range(n)]
    path = tmp_path / "sft.jsonl"
    path.write_text("\n".join(json.dumps(r) for r in rows) + "\n")
    return str(path)


@pytest.mark.parametrize("script", ["sft", "dpo"])
def test_sft_and_dpo_survive_a_dropout(tmp_path, script):
    """the SFT / DPO entrypoints take the full --lion_*
    flag set, --lion_elastic_timeout included; a 2-rank gloo run under the
    launcher loses rank 1 inside backward and the survivor finishes, saves and
    logs world_end = 1."""
    out = str(tmp_path / script)
    common = ["--lion", "--async_grad", "--lion_elastic_timeout", "20", "--lion_beta1", "0.95",
              "--lion_tie_break", "negative", "--lion_wire", "a2a", "--output_dir", out, "--max_steps", "4",
              "--logging_steps", "1", "--per_device_train_batch_size", "2", "--report_to", "none", "--use_cpu",
              "--ddp_backend", "gloo"]
    if script == "sft":
        args = ["sft_llama2.py", "--model_name", "llama-tiny", "--dataset_name", _sft_corpus(tmp_path, 200),
                "--seq_length", "64", "--size_valid_set", "10", "--shuffle_buffer", "50",
                "--save_strategy", "no", "--gradient_accumulation_steps", "1"] + common
    else:
        args = ["dpo_llama2.py", "--model_name_or_path", "llama-tiny", "--synthetic_data", "--synthetic_samples", "64",
                "--max_length", "400", "--max_prompt_length", "200", "--gradient_accumulation_steps", "1",
                "--eval_steps", "0", "--save_steps", "100", "--warmup_steps", "1",
                "--checkpointing_policy", "reference", "--gradient_checkpointing", "false"] + common
    r = _launch(2, args, env_extra={"DLION_FAULT": "1:2:backward"})
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-4000:]
    recs = [json.loads(x) for x in open(os.path.join(out, "metrics.jsonl"))]
    last = [x for x in recs if "world_end" in x]
    assert last and last[-1]["world_end"] == 1.0, recs[-3:]
    lion = [x["lion"] for x in recs if "lion" in x]
    assert lion[-1]["world"] == 1 and lion[-1]["dropout_events"][0]["dropped"] == [1]
    assert max(x["step"] for x in recs if "loss" in x) == 4
    assert os.path.isdir(os.path.join(out, "final_checkpoint"))
