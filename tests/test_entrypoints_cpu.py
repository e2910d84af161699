"""End-to-end entrypoints on CPU: run_clm (1 rank and 2 gloo ranks via torchrun,
per-rank optimizer checkpoints, resume), sft_llama2, dpo_llama2, and the
drop-in ``distributed_lion`` / ``async_trainer`` module names."""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

COMMON = ["--synthetic_data", "--synthetic_samples", "64", "--block_size", "64", "--per_device_train_batch_size",
          "4", "--gradient_accumulation_steps", "2", "--warmup_steps", "1", "--learning_rate", "1e-3",
          "--report_to", "none", "--use_cpu", "--logging_steps", "1",
          "--config_name", "gpt2-tiny", "--config_overrides", "resid_pdrop=0.0,embd_pdrop=0.0,attn_pdrop=0.0"]


def test_dropin_module_names():
    import async_trainer
    import distributed_lion

    assert distributed_lion.Lion.__module__.endswith("optim.lion")
    for name in ("AsyncTrainer", "AsyncSFTTrainer", "AsyncDPOTrainer"):
        assert hasattr(async_trainer, name)
    for name in ("update_fn", "update_fn_distributed", "update_fn_distributed_stoc", "majority_vote",
                 "flatten_and_pad", "restore_flattened_tensor"):
        assert callable(getattr(distributed_lion, name))


def test_run_clm_single_process(tmp_path):
    import run_clm

    out = str(tmp_path / "clm")
    trainer = run_clm.main(COMMON + ["--max_steps", "3", "--lion", "--async_grad", "--do_train", "--do_eval",
                                     "--output_dir", out])
    assert os.path.isfile(os.path.join(out, "model.safetensors"))
    recs = [json.loads(x) for x in open(os.path.join(out, "metrics.jsonl"))]
    assert any("loss" in r for r in recs) and any("lion" in r for r in recs)
    assert type(trainer.optimizer.optimizer if hasattr(trainer.optimizer, "optimizer") else trainer.optimizer
                ).__name__ == "Lion"
    ev = json.load(open(os.path.join(out, "eval_results.json")))
    assert "perplexity" in ev and "eval_accuracy" in ev


def _torchrun(args, port):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc_per_node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.join(ROOT, "run_clm.py")] + args
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r


@pytest.mark.slow
def test_run_clm_two_ranks_resume(tmp_path):
    from dist_utils import free_port

    out = str(tmp_path / "clm2")
    args = COMMON + ["--lion", "--async_grad", "--do_train", "--output_dir", out, "--ddp_backend", "gloo",
                     "--save_steps", "2"]
    _torchrun(args + ["--max_steps", "4"], free_port())
    ck = os.path.join(out, "checkpoint-2")
    files = set(os.listdir(ck))
    assert {"rank0-of-2-optimizer.pt", "rank1-of-2-optimizer.pt", "optimizer.pt"} <= files
    m0 = torch.load(os.path.join(ck, "rank0-of-2-optimizer.pt"), weights_only=True)["state"]
    m1 = torch.load(os.path.join(ck, "rank1-of-2-optimizer.pt"), weights_only=True)["state"]
    assert any(not torch.equal(m0[k]["exp_avg"], m1[k]["exp_avg"]) for k in m0), "momenta must be per worker"
    from safetensors.torch import load_file

    final = load_file(os.path.join(out, "model.safetensors"))
    # resume from checkpoint-2 in a fresh directory copy and finish the same 4 steps
    out2 = str(tmp_path / "clm2b")
    import shutil

    shutil.copytree(ck, os.path.join(out2, "checkpoint-2"))
    _torchrun(COMMON + ["--lion", "--async_grad", "--do_train", "--output_dir", out2, "--ddp_backend", "gloo",
                        "--save_steps", "2", "--max_steps", "4"], free_port())
    resumed = load_file(os.path.join(out2, "model.safetensors"))
    for k in final:
        assert torch.equal(final[k], resumed[k]), k


def test_sft_and_dpo_entrypoints(tmp_path):
    import dpo_llama2
    import sft_llama2

    sft_out = str(tmp_path / "sft")
    sft_llama2.main(["--model_name", "llama-tiny", "--synthetic_data", "--synthetic_samples", "100", "--seq_length", "64",
                     "--output_dir", sft_out, "--max_steps", "2", "--per_device_train_batch_size", "2",
                     "--learning_rate", "1e-3", "--lion", "--async_grad", "--report_to", "none", "--use_cpu",
                     "--torch_dtype", "float32"])
    assert os.path.isfile(os.path.join(sft_out, "final_checkpoint", "adapter_model.safetensors"))
    merged = os.path.join(sft_out, "final_merged_checkpoint")
    assert os.path.isfile(os.path.join(merged, "model.safetensors"))
    dpo_out = str(tmp_path / "dpo")
    tr = dpo_llama2.main(["--model_name_or_path", merged, "--synthetic_data", "--synthetic_samples", "60", "--max_length", "1024",
                          "--max_prompt_length", "256", "--output_dir", dpo_out, "--max_steps", "2",
                          "--per_device_train_batch_size", "2", "--gradient_accumulation_steps", "1", "--lion",
                          "--async_grad", "--use_cpu", "--torch_dtype", "float32", "--eval_steps", "0",
                          "--warmup_steps", "1", "--logging_steps", "1"])
    assert tr.state.global_step == 2
    assert os.path.isfile(os.path.join(dpo_out, "final_checkpoint", "adapter_config.json"))


def test_sft_4bit_merge_uses_original_weights(tmp_path):
    """--load_in_4bit: the merged checkpoint is W + B@A*scaling on the ORIGINAL
    compute-dtype base (reference sft_llama2.py:195-196 reloads it), not
    dequant(quant(W)) + delta."""
    from safetensors.torch import load_file

    import sft_llama2
    from distributed_lion_pytorch_amd.models.quant import QuantConfig, quantize_model

    out = str(tmp_path / "qsft")
    args = ["--model_name", "llama-tiny", "--synthetic_data", "--synthetic_samples", "60", "--seq_length", "64", "--output_dir", out,
            "--max_steps", "2", "--per_device_train_batch_size", "2", "--learning_rate", "1e-2", "--lion",
            "--async_grad", "--report_to", "none", "--use_cpu", "--torch_dtype", "float32", "--load_in_4bit"]
    sft_llama2.main(args)
    merged = load_file(os.path.join(out, "final_merged_checkpoint", "model.safetensors"))
    adapter = load_file(os.path.join(out, "final_checkpoint", "adapter_model.safetensors"))
    sa = sft_llama2.HfArgumentParser((sft_llama2.ScriptArguments, sft_llama2.TrainingArguments)) \
        .parse_args_into_dataclasses(args=args)[0]
    base = sft_llama2.build_base(sa, 42).state_dict()  # HF TrainingArguments default seed
    key = "model.layers.0.self_attn.q_proj.weight"
    a = adapter["base_model.model.model.layers.0.self_attn.q_proj.lora_A.weight"]
    b = adapter["base_model.model.model.layers.0.self_attn.q_proj.lora_B.weight"]
    assert b.abs().max() > 0, "the adapter must have trained"
    expect = base[key] + (b @ a) * (16 / 8)
    assert torch.allclose(merged[key], expect, atol=1e-6, rtol=0)
    # and it is NOT the 4-bit-rounded base
    q = quantize_model(sft_llama2.build_base(sa, 42), QuantConfig(bnb_4bit_compute_dtype=torch.float32))
    deq = q.model.layers[0].self_attn.q_proj.dequantize(torch.float32)
    assert not torch.allclose(merged[key], deq + (b @ a) * 2.0, atol=1e-4)


def test_dpo_checkpointing_decision_sees_lora_and_frozen_reference(tmp_path, monkeypatch):
    """dpo_llama2 decides activation checkpointing after LoRA injection with the
    reference frozen: the memory estimate then counts a gradient + momentum only
    for the adapters (the all-trainable count checkpointed a batch that fits)."""
    import dpo_llama2
    from distributed_lion_pytorch_amd.trainer import memory

    seen = {}

    def spy(requested, policy, config, tokens, *models, **kw):
        seen["trainable"] = [sum(p.numel() for p in m.parameters() if p.requires_grad) for m in models]
        seen["total"] = [sum(p.numel() for p in m.parameters()) for m in models]
        return False

    monkeypatch.setattr(memory, "should_checkpoint", spy)
    tr = dpo_llama2.main(["--model_name_or_path", "llama-tiny", "--synthetic_data", "--synthetic_samples", "60", "--max_length", "1024",
                          "--max_prompt_length", "256", "--output_dir", str(tmp_path / "dpo"), "--max_steps", "1",
                          "--per_device_train_batch_size", "2", "--gradient_accumulation_steps", "1", "--lion",
                          "--async_grad", "--use_cpu", "--torch_dtype", "float32", "--eval_steps", "0",
                          "--warmup_steps", "1", "--final_save", "false"])
    assert tr.state.global_step == 1
    policy, ref = seen["trainable"]
    assert ref == 0  # the reference is frozen before the estimate
    assert 0 < policy < seen["total"][0] // 10  # only the LoRA adapters train


def test_dpo_reward_stats_keep_train_and_eval_apart(tmp_path):
    """evaluation batches must not be averaged into the training
    log's rewards/* (trl logs them separately as eval_rewards/*)."""
    import dpo_llama2

    tr = dpo_llama2.main(["--model_name_or_path", "llama-tiny", "--synthetic_data", "--synthetic_samples", "60", "--max_length", "512",
                          "--max_prompt_length", "256", "--output_dir", str(tmp_path / "dpo"), "--max_steps", "2",
                          "--per_device_train_batch_size", "2", "--gradient_accumulation_steps", "1", "--lion",
                          "--async_grad", "--use_cpu", "--torch_dtype", "float32", "--eval_steps", "1",
                          "--warmup_steps", "1", "--logging_steps", "1", "--final_save", "false"])
    hist = tr.state.log_history
    evals = [h for h in hist if "eval_loss" in h]
    trains = [h for h in hist if "loss" in h and "eval_loss" not in h]
    assert evals and trains
    assert all("eval_rewards/accuracies" in h and "rewards/accuracies" not in h for h in evals), evals
    assert all("rewards/accuracies" in h and "eval_rewards/accuracies" not in h for h in trains), trains


def test_reference_readme_command_lines(tmp_path):
    """The three launch commands of /root/reference/README.md:16-66 parse
    unchanged (wandb reporting aside), including ``--group_by_length``, which
    transformers 5 dropped from TrainingArguments; the SFT one also trains
    two steps on a tiny model, and group_by_length + packing is refused as in
    /root/reference/sft_llama2.py:53."""
    from transformers import HfArgumentParser

    import dpo_llama2
    import run_clm
    import sft_llama2
    from distributed_lion_pytorch_amd.trainer.async_trainer import AsyncTrainingArguments

    clm = ["--config_name", "gpt2", "--tokenizer_name", "gpt2", "--dataset_name", "openwebtext",
           "--per_device_train_batch_size", "20", "--per_device_eval_batch_size", "24", "--do_train", "--do_eval",
           "--output_dir", str(tmp_path / "gpt2_lion_wd_0.1"), "--report_to", "none", "--torch_dtype", "bfloat16",
           "--gradient_accumulation_steps", "8", "--max_steps", "100000", "--warmup_steps", "2000", "--lion",
           "--save_total_limit", "2", "--learning_rate", "0.0001", "--weight_decay", "0.1", "--async_grad"]
    m, d, t = HfArgumentParser((run_clm.ModelArguments, run_clm.DataTrainingArguments, AsyncTrainingArguments)) \
        .parse_args_into_dataclasses(args=clm)
    assert t.lion and t.async_grad and t.gradient_accumulation_steps == 8 and d.dataset_name == "openwebtext"

    sft = ["--output_dir", str(tmp_path / "sft"), "--max_steps", "2", "--logging_steps", "10", "--save_steps", "10",
           "--per_device_train_batch_size", "4", "--per_device_eval_batch_size", "1",
           "--gradient_accumulation_steps", "2", "--gradient_checkpointing", "False", "--group_by_length", "False",
           "--learning_rate", "1e-4", "--lr_scheduler_type", "cosine", "--warmup_steps", "100",
           "--weight_decay", "0.05", "--optim", "paged_adamw_32bit", "--bf16", "True",
           "--remove_unused_columns", "False", "--run_name", "sft_llama2", "--report_to", "none", "--lion",
           "--async_grad"]
    tiny = ["--model_name", "llama-tiny", "--synthetic_data", "--synthetic_samples", "100", "--seq_length", "64",
            "--use_cpu"]
    sft_llama2.main(sft + tiny)
    assert os.path.isfile(os.path.join(tmp_path, "sft", "final_checkpoint", "adapter_model.safetensors"))
    with pytest.raises(ValueError, match="packing"):
        sft_llama2.main([a if a != "False" or sft[i - 1] != "--group_by_length" else "True"
                         for i, a in enumerate(sft)] + tiny)

    dpo = ["--model_name_or_path", "sft/final_checkpoint", "--output_dir", "dpo", "--lion", "--async_grad"]
    s, lion = HfArgumentParser((dpo_llama2.ScriptArguments, dpo_llama2.LionArguments)).parse_args_into_dataclasses(args=dpo)
    assert s.lion and s.async_grad and s.model_name_or_path == "sft/final_checkpoint"
