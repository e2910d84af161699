"""run_clm.py data-pipeline fidelity to /root/reference/run_clm.py:
disjoint train/validation splits (``train[:p%]`` / ``train[p%:]``, or the
dataset's own validation split), ``max_train/eval_samples`` on real data,
``--streaming`` refused, embedding resize for a larger tokenizer, model card,
group_texts over 1000-text batches (no separator token),
``preprocessing_num_workers`` and ``overwrite_cache``."""
import os
import re
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import run_clm  # noqa: E402
from distributed_lion_pytorch_amd.utils import data as data_mod  # noqa: E402
from distributed_lion_pytorch_amd.utils.data import ByteTokenizer  # noqa: E402


@pytest.fixture(autouse=True)
def _private_cache(tmp_path, monkeypatch):
    monkeypatch.setenv("HF_DATASETS_CACHE", str(tmp_path / "hf_datasets"))

BASE = ["--report_to", "none", "--use_cpu", "--config_name", "gpt2-tiny", "--per_device_train_batch_size", "2",
        "--learning_rate", "1e-3", "--warmup_steps", "1", "--lion", "--async_grad"]


def _args(extra):
    from transformers import HfArgumentParser

    parser = HfArgumentParser((run_clm.ModelArguments, run_clm.DataTrainingArguments,
                               run_clm.AsyncTrainingArguments))
    return parser.parse_args_into_dataclasses(args=BASE + ["--output_dir", "/tmp/unused"] + extra)


def _texts(n):
    # one distinctive line per row: every block can be traced back to its line
    return [f"row {i:05d} " + "x" * 40 for i in range(n)]


def _rows_of(ds, tok):
    rows = set()
    for i in range(len(ds)):
        ids = ds[i]["input_ids"].tolist()
        txt = tok.decode(ids)
        rows |= {int(x) for x in re.findall(r"row (\d{5}) ", txt)}  # complete row headers only
    return rows


def test_split_is_disjoint_front_percent():
    tr, va = run_clm.split_train_validation(list(range(200)), 5)
    assert va == list(range(10)) and tr == list(range(10, 200))
    tr, va = run_clm.split_train_validation(list(range(30)), 5)  # 1.5 -> rounds to 2
    assert len(va) == 2 and not set(tr) & set(va)


def test_train_file_without_validation_uses_disjoint_split(tmp_path):
    f = tmp_path / "corpus.txt"
    f.write_text("\n".join(_texts(400)) + "\n")
    m, d, t = _args(["--train_file", str(f), "--block_size", "32", "--validation_split_percentage", "10"])
    tok = ByteTokenizer()
    train, val = run_clm.build_datasets(d, t, tok, 512, 32)
    rt, rv = _rows_of(train, tok), _rows_of(val, tok)
    assert rv and rt and not (rt & rv), "validation blocks must not contain training rows"
    assert max(rv) < 41 and min(rt) >= 39  # validation = the first 10 % (40 rows) of the file
    # max_train_samples / max_eval_samples cap real data too
    m, d, t = _args(["--train_file", str(f), "--block_size", "32", "--max_train_samples", "7",
                     "--max_eval_samples", "3"])
    train, val = run_clm.build_datasets(d, t, tok, 512, 32)
    assert len(train) == 7 and len(val) == 3


def test_dataset_own_validation_split_is_used(tmp_path):
    datasets = pytest.importorskip("datasets")
    dd = datasets.DatasetDict({"train": datasets.Dataset.from_dict({"text": _texts(300)}),
                               "validation": datasets.Dataset.from_dict({"text": [f"row {i:05d} " + "y" * 40
                                                                                   for i in range(900, 960)]})})
    path = str(tmp_path / "ds")
    dd.save_to_disk(path)
    m, d, t = _args(["--dataset_name", path, "--block_size", "32"])
    tok = ByteTokenizer()
    train, val = run_clm.build_datasets(d, t, tok, 512, 32)
    assert _rows_of(val, tok) <= set(range(900, 960)) and _rows_of(train, tok) <= set(range(300))
    assert min(_rows_of(train, tok)) == 0  # nothing was carved out of train


def test_streaming_is_refused(tmp_path):
    with pytest.raises(ValueError, match="streaming"):
        run_clm.main(BASE + ["--synthetic_data", "--streaming", "--output_dir", str(tmp_path), "--max_steps", "1"])


def test_embeddings_resized_for_larger_tokenizer(tmp_path):
    out = str(tmp_path / "resize")
    tr = run_clm.main(BASE + ["--synthetic_data", "--synthetic_samples", "16", "--block_size", "32",
                              "--config_overrides", "vocab_size=100", "--max_steps", "1", "--do_train",
                              "--output_dir", out])
    model = tr.model
    assert model.get_input_embeddings().weight.shape[0] == len(ByteTokenizer()) == 259
    assert model.config.vocab_size == 259
    assert model.get_output_embeddings().weight is model.get_input_embeddings().weight  # still tied
    assert os.path.isfile(os.path.join(out, "README.md"))  # model card


def _reference_group_texts(texts, tok, block_size):
    """/root/reference/run_clm.py:463-544 restated: tokenizer map then group_texts
    map, both batched (1000 texts), remainder of each batch dropped."""
    from itertools import chain

    out = []
    for i in range(0, len(texts), 1000):
        ids = tok(texts[i:i + 1000])["input_ids"]
        flat = list(chain(*ids))
        n = len(flat) // block_size * block_size
        out += [flat[j:j + block_size] for j in range(0, n, block_size)]
    return out


def test_group_texts_matches_reference_batches():
    tok = ByteTokenizer()
    texts = [f"line {i} " + "z" * (i % 37) for i in range(2500)]
    ds = data_mod.clm_blocks(texts, tok, 64)
    ref = _reference_group_texts(texts, tok, 64)
    assert len(ds) == len(ref) and all(ds[i]["input_ids"].tolist() == ref[i] for i in range(len(ref)))
    assert tok.eos_token_id not in ds.data  # no separator token between texts (reference parity)


def test_preprocessing_workers_match_serial():
    tok = ByteTokenizer()
    texts = [f"w {i} " + "q" * (i % 11) for i in range(2300)]
    a = data_mod.clm_blocks(texts, tok, 32)
    b = data_mod.clm_blocks(texts, tok, 32, num_workers=2)
    assert torch.equal(a.data, b.data)


class _CountingTok(ByteTokenizer):
    calls = 0

    def __call__(self, text, **kw):
        type(self).calls += 1
        return super().__call__(text, **kw)


def test_cache_hit_and_overwrite_cache(tmp_path):
    tok = _CountingTok()
    texts = [f"c {i} " + "y" * 20 for i in range(1500)]
    cache = str(tmp_path / "cache")
    first = data_mod.clm_blocks(texts, tok, 32, cache_dir=cache)
    n = _CountingTok.calls
    again = data_mod.clm_blocks(texts, tok, 32, cache_dir=cache)
    assert _CountingTok.calls == n and torch.equal(first.data, again.data)  # served from the cache
    data_mod.clm_blocks(texts, tok, 32, cache_dir=cache, overwrite_cache=True)
    assert _CountingTok.calls > n  # recomputed
    other = data_mod.clm_blocks(texts[:-1], tok, 32, cache_dir=cache)  # different texts: different key
    assert len(os.listdir(cache)) == 2 and len(other) <= len(first)
