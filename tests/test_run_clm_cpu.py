"""run_clm.py data-pipeline fidelity to /root/reference/run_clm.py:
disjoint train/validation splits (``train[:p%]`` / ``train[p%:]``, or the
dataset's own validation split), ``max_train/eval_samples`` on real data,
local files read by extension (csv / json / txt columns, not raw text),
``--streaming`` over a local file (lazy, bounded buffer, rank-sharded blocks),
embedding resize for a larger tokenizer, model card,
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


def test_streaming_needs_local_files_and_max_steps(tmp_path):
    with pytest.raises(ValueError, match="streaming"):
        run_clm.main(BASE + ["--synthetic_data", "--streaming", "--output_dir", str(tmp_path), "--max_steps", "1"])
    f = tmp_path / "c.txt"
    f.write_text("\n".join(_texts(50)) + "\n")
    with pytest.raises(ValueError, match="max_steps"):
        run_clm.main(BASE + ["--train_file", str(f), "--streaming", "--do_train", "--output_dir", str(tmp_path)])


def _all_text(ds, tok):
    return "".join(tok.decode(ds[i]["input_ids"].tolist()) for i in range(len(ds)))


def test_json_and_jsonl_train_files_read_the_text_column(tmp_path):
    """A .json / .jsonl train file is parsed: the blocks hold the "text"
    column's contents, never the JSON syntax (round 4 tokenized the raw file)."""
    import json

    rows = [{"id": i, "text": f"row {i:05d} " + "j" * 40} for i in range(300)]
    tok = ByteTokenizer()
    for name, body in (("c.jsonl", "\n".join(json.dumps(r) for r in rows) + "\n"), ("c.json", json.dumps(rows))):
        f = tmp_path / name
        f.write_text(body)
        m, d, t = _args(["--train_file", str(f), "--block_size", "32", "--validation_split_percentage", "10"])
        train, val = run_clm.build_datasets(d, t, tok, 512, 32)
        txt = _all_text(train, tok) + _all_text(val, tok)
        assert "row 00150 jjj" in txt and '"text"' not in txt and '"id"' not in txt and "{" not in txt
        assert min(_rows_of(train, tok)) >= 29 and max(_rows_of(val, tok)) < 31  # first 10 % = validation


def test_csv_train_file_reads_the_text_column_or_the_first(tmp_path):
    tok = ByteTokenizer()
    f = tmp_path / "c.csv"
    f.write_text("id,text\n" + "".join(f'{i},"row {i:05d} , {"c" * 40}"\n' for i in range(200)))
    m, d, t = _args(["--train_file", str(f), "--block_size", "32"])
    train, val = run_clm.build_datasets(d, t, tok, 512, 32)
    txt = _all_text(train, tok)
    assert "row 00100 , ccc" in txt and "id,text" not in txt and '"' not in txt
    # no "text" column: the first column is the text (reference run_clm.py:455-458)
    g = tmp_path / "d.csv"
    g.write_text("body,n\n" + "".join(f"row {i:05d} {'b' * 40},{i}\n" for i in range(200)))
    m, d, t = _args(["--train_file", str(g), "--block_size", "32"])
    train, _ = run_clm.build_datasets(d, t, tok, 512, 32)
    assert "row 00100 bbb" in _all_text(train, tok) and "body,n" not in _all_text(train, tok)


def test_txt_keeps_blank_lines_as_rows(tmp_path):
    """The text builder keeps empty lines as rows: with keep_linebreaks their
    "\n" is part of the token stream (round 4 dropped them)."""
    tok = ByteTokenizer()
    f = tmp_path / "c.txt"
    f.write_text("".join(f"row {i:05d}\n\n\n" for i in range(400)))
    m, d, t = _args(["--train_file", str(f), "--block_size", "16", "--validation_split_percentage", "1"])
    train, _ = run_clm.build_datasets(d, t, tok, 512, 16)
    assert "\n\n\nrow " in _all_text(train, tok)
    m, d, t = _args(["--train_file", str(f), "--block_size", "16", "--keep_linebreaks", "false"])
    train, _ = run_clm.build_datasets(d, t, tok, 512, 16)
    assert "\n" not in _all_text(train, tok) and "row 00200row 00201" in _all_text(train, tok)


def test_stream_equals_map_pipeline_and_is_bounded(tmp_path):
    """--streaming: the same blocks as the map-style pipeline (1000-text
    batches, remainders dropped), with at most one batch of texts held; a
    corpus of 5x the buffer streams through.  Ranks get disjoint blocks, the
    same count each."""
    datasets = pytest.importorskip("datasets")
    tok = ByteTokenizer()
    texts = [f"s {i:05d} " + "q" * (i % 53) for i in range(5000)]
    f = tmp_path / "big.txt"
    f.write_text("\n".join(texts) + "\n")
    rows = datasets.load_dataset("text", data_files={"train": str(f)}, streaming=True, keep_linebreaks=True)["train"]
    ref = data_mod.clm_blocks([t + "\n" for t in texts], tok, 64)
    st = data_mod.CLMStream(rows, "text", tok, 64, shard=False)
    got = [b["input_ids"] for b in st]
    assert len(got) == len(ref) and all(torch.equal(got[i], ref[i]["input_ids"]) for i in range(len(ref)))
    assert st.peak_buffer_rows == 1000 < len(texts)  # never more than one map batch held
    shards = []
    for rank in range(3):
        monkey = data_mod._dist_shard
        data_mod._dist_shard = lambda rank=rank: (rank, 3)
        try:
            shards.append([b["input_ids"] for b in data_mod.CLMStream(rows, "text", tok, 64, shard=True)])
        finally:
            data_mod._dist_shard = monkey
    n = len(ref) // 3
    assert [len(s) for s in shards] == [n, n, n]
    for rank in range(3):
        assert all(torch.equal(shards[rank][i], ref[3 * i + rank]["input_ids"]) for i in range(n))
    capped = list(data_mod.CLMStream(rows, "text", tok, 64, shard=False, max_blocks=7))
    assert len(capped) == 7


def test_run_clm_streaming_trains_on_a_local_file(tmp_path):
    f = tmp_path / "corpus.txt"
    f.write_text("\n".join(_texts(3000)) + "\n")
    out = str(tmp_path / "stream")
    tr = run_clm.main(BASE + ["--train_file", str(f), "--streaming", "--block_size", "32", "--max_steps", "3",
                              "--do_train", "--do_eval", "--max_eval_samples", "4", "--output_dir", out,
                              "--save_strategy", "no"])
    assert tr.state.global_step == 3
    assert isinstance(tr.train_dataset, data_mod.CLMStream) and tr.train_dataset.peak_buffer_rows <= 1000
    assert os.path.isfile(os.path.join(out, "eval_results.json"))


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
