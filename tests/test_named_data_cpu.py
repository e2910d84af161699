"""Named SFT / DPO / CLM datasets read like the reference:

* SFT: ``load_dataset(dataset_name, data_dir=subset, split=split,
  streaming=...)`` (/root/reference/sft_llama2.py:99-107) on a local copy of a
  stack-exchange-paired-layout repository (data/finetune parquet shards);
* DPO: question/response_j/response_k rows mapped to prompt/chosen/rejected
  (/root/reference/dpo_llama2.py:113-118) from data/rl, the evaluation set
  from data/evaluation (:164);
* a name that resolves to nothing is an error unless --synthetic_data.
"""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pd = pytest.importorskip("pandas")
datasets = pytest.importorskip("datasets")

from distributed_lion_pytorch_amd.utils import data as D  # noqa: E402


@pytest.fixture(autouse=True)
def _private_cache(tmp_path, monkeypatch):
    monkeypatch.setenv("HF_DATASETS_CACHE", str(tmp_path / "hf_datasets"))


def _se_rows(tag, n):
    return [{"qid": i, "question": f"{tag}{i:04d} " + "why " * 8, "date": "2023", "metadata": ["x"],
             "response_j": f"good-{tag}{i:04d} " + "yes " * 10, "response_k": f"bad-{tag}{i:04d} " + "no " * 10}
            for i in range(n)]


@pytest.fixture
def se_repo(tmp_path):
    """A tiny local mirror of the stack-exchange-paired layout: parquet shards in
    data/finetune and data/evaluation, json lines in data/rl."""
    root = tmp_path / "stack-exchange-paired"
    for sub in ("finetune", "rl", "evaluation"):
        (root / "data" / sub).mkdir(parents=True)
    ft = _se_rows("ft", 300)
    pd.DataFrame(ft[:150]).to_parquet(root / "data" / "finetune" / "train-00000-of-00002.parquet")
    pd.DataFrame(ft[150:]).to_parquet(root / "data" / "finetune" / "train-00001-of-00002.parquet")
    with open(root / "data" / "rl" / "train.jsonl", "w") as f:
        for r in _se_rows("rl", 80):
            f.write(json.dumps(r) + "\n")
    pd.DataFrame(_se_rows("ev", 12)).to_parquet(root / "data" / "evaluation" / "train-00000-of-00001.parquet")
    return str(root)


def test_load_named_rows_reads_a_local_repository(se_repo):
    rows = D.load_named_rows(se_repo, data_dir="data/finetune", split="train")
    assert len(rows) == 300 and rows[0]["question"].startswith("ft")
    stream = D.load_named_rows(se_repo, data_dir="data/rl", split="train", streaming=True)
    got = [r["question"][:6] for r in stream]
    assert got == [f"rl{i:04d}" for i in range(80)]
    assert [r["question"][:6] for r in stream][:3] == got[:3]  # re-iterable


def test_missing_names_raise(tmp_path, se_repo):
    with pytest.raises(D.DatasetUnavailable, match="synthetic_data"):
        D.load_named_rows(str(tmp_path / "no-such-dataset"))
    with pytest.raises(D.DatasetUnavailable):
        D.load_named_rows("lvwerra/stack-exchange-paired", data_dir="data/finetune")  # offline hub name
    with pytest.raises(D.DatasetUnavailable, match="no 'data/nope'"):
        D.load_named_rows(se_repo, data_dir="data/nope")


def test_sft_trains_on_the_named_rows(se_repo):
    """The packed SFT stream is made of the data/finetune rows, formatted like
    the reference (Question / Answer = response_j), not synthetic words."""
    import sft_llama2
    from transformers import HfArgumentParser

    tok = D.ByteTokenizer()
    for streaming in ("true", "false"):
        sa = HfArgumentParser(sft_llama2.ScriptArguments).parse_args_into_dataclasses(
            args=["--dataset_name", se_repo, "--seq_length", "64", "--size_valid_set", "10", "--shuffle_buffer",
                  "20", "--streaming", streaming])[0]
        train, valid = sft_llama2.create_datasets(tok, sa, seed=0)
        it = iter(train)
        text = "".join(tok.decode(next(it)["input_ids"].tolist()) for _ in range(40))
        qs = {t[:6] for t in text.split("Question: ")[1:] if len(t) >= 6}
        assert qs and all(q.startswith("ft") for q in qs), qs
        assert "Answer: good-ft" in text and "bad-ft" not in text
        vtext = "".join(tok.decode(valid[i]["input_ids"].tolist()) for i in range(len(valid)))
        assert "Question: ft" in vtext


def test_sft_entrypoint_on_a_repository_and_missing_name(se_repo, tmp_path):
    import sft_llama2

    common = ["--model_name", "llama-tiny", "--seq_length", "64", "--size_valid_set", "10", "--shuffle_buffer", "50",
              "--max_steps", "2", "--per_device_train_batch_size", "2", "--use_cpu", "--report_to", "none", "--lion",
              "--async_grad", "--save_strategy", "no", "--final_save", "false", "--torch_dtype", "float32"]
    tr = sft_llama2.main(common + ["--dataset_name", se_repo, "--output_dir", str(tmp_path / "a")])
    assert tr.state.global_step == 2
    with pytest.raises(D.DatasetUnavailable):
        sft_llama2.main(common + ["--dataset_name", str(tmp_path / "typo"), "--output_dir", str(tmp_path / "b")])
    with pytest.raises(D.DatasetUnavailable):  # the default hub name, offline, without --synthetic_data
        sft_llama2.main(common + ["--output_dir", str(tmp_path / "c")])


def test_dpo_maps_reference_rows_and_reads_the_evaluation_subset(se_repo, tmp_path):
    import dpo_llama2

    common = ["--model_name_or_path", "llama-tiny", "--max_length", "512", "--max_prompt_length", "256",
              "--max_steps", "1", "--per_device_train_batch_size", "2", "--gradient_accumulation_steps", "1",
              "--lion", "--async_grad", "--use_cpu", "--torch_dtype", "float32", "--eval_steps", "0",
              "--warmup_steps", "1", "--final_save", "false"]
    tr = dpo_llama2.main(common + ["--dataset_name", se_repo, "--output_dir", str(tmp_path / "a")])
    assert tr.state.global_step == 1
    train, ev = tr.train_dataset, tr.eval_dataset
    assert len(train) == 80 and len(ev) == 12
    assert all(r["prompt"].startswith("Question: rl") and r["prompt"].endswith("\n\nAnswer: ") for r in train)
    assert all(r["chosen"].startswith("good-rl") and r["rejected"].startswith("bad-rl") for r in train)
    assert all(r["prompt"].startswith("Question: ev") for r in ev)
    # a single file in the reference's row format (the r5 crash: KeyError 'prompt')
    f = tmp_path / "pairs.jsonl"
    f.write_text("".join(json.dumps(r) + "\n" for r in _se_rows("fl", 40)))
    tr = dpo_llama2.main(common + ["--dataset_name", str(f), "--output_dir", str(tmp_path / "b")])
    assert len(tr.train_dataset) + len(tr.eval_dataset) == 40
    assert tr.eval_dataset[0]["prompt"].startswith("Question: fl0000")
    with pytest.raises(D.DatasetUnavailable):
        dpo_llama2.main(common + ["--dataset_name", str(tmp_path / "typo"), "--output_dir", str(tmp_path / "c")])


def test_run_clm_missing_dataset_name_raises(tmp_path):
    import run_clm
    from transformers import HfArgumentParser

    parser = HfArgumentParser((run_clm.ModelArguments, run_clm.DataTrainingArguments,
                               run_clm.AsyncTrainingArguments))
    m, d, t = parser.parse_args_into_dataclasses(args=["--output_dir", str(tmp_path), "--use_cpu",
                                                       "--dataset_name", str(tmp_path / "typo")])
    with pytest.raises(FileNotFoundError, match="synthetic_data"):
        run_clm.build_datasets(d, t, D.ByteTokenizer(), 512, 32)
