"""SFT data semantics of the reference (sft_llama2.py:99-138) on local data:
seeded shuffle buffer, take/skip and random train/valid splits, an infinite
packed training stream read lazily (constant memory) and sharded per rank."""
import json

import pytest

from distributed_lion_pytorch_amd.utils import data as D


def test_shuffle_buffer_deterministic_per_seed_and_epoch():
    rows = list(range(200))
    a = list(D.ShuffledRows(rows, 16, seed=1))
    assert sorted(a) == rows and a != rows
    assert a == list(D.ShuffledRows(rows, 16, seed=1))
    assert a != list(D.ShuffledRows(rows, 16, seed=2))
    s = D.ShuffledRows(rows, 16, seed=1)
    s.set_epoch(1)
    assert list(s) != a and sorted(s) == rows


def test_random_split_disjoint_complete_seeded():
    rows = [{"i": i} for i in range(1000)]
    tr, va = D.random_split(rows, 0.005, seed=3)
    assert len(va) == 5 and len(tr) == 995
    ids_tr, ids_va = {r["i"] for r in tr}, {r["i"] for r in va}
    assert not ids_tr & ids_va and ids_tr | ids_va == set(range(1000))
    assert D.random_split(rows, 0.005, seed=3)[1] == va
    assert D.random_split(rows, 0.005, seed=4)[1] != va


def _corpus(tmp_path, n):
    path = tmp_path / "corpus.jsonl"
    with open(path, "w") as f:
        for i in range(n):
            f.write(json.dumps({"question": f"q{i:05d} " + "x" * 80, "response_j": "y" * 100}) + "\n")
    return str(path)


class _Counting:
    def __init__(self, rows):
        self.rows, self.pulled = rows, 0

    def __iter__(self):
        for r in self.rows:
            self.pulled += 1
            yield r


def test_packed_stream_is_lazy_and_bounded(tmp_path):
    """A corpus ~100x the packing buffer: producing a few sequences reads only
    a buffer's worth of rows, and the buffer never exceeds its bound."""
    tok = D.ByteTokenizer()
    rows = _Counting(D.Rows(_corpus(tmp_path, 5000)))  # ~1 MB of text
    ds = D.PackedStream(tok, rows, seq_length=64, infinite=True, chars_per_token=1.0, num_of_sequences=16, shard=False)
    it = iter(ds)
    seqs = [next(it) for _ in range(10)]
    assert all(s["input_ids"].shape == (64,) for s in seqs)
    assert ds.peak_buffer_chars <= ds.max_buffer_size + 300  # one row past the bound at most
    assert rows.pulled < 20  # ~1024 characters of ~200-character rows, not the whole file


def test_packed_stream_infinite_restarts_and_finite_stops(tmp_path):
    tok = D.ByteTokenizer()
    rows = D.Rows(_corpus(tmp_path, 20))  # ~4k characters
    fin = list(D.PackedStream(tok, rows, seq_length=64, infinite=False, chars_per_token=1.0, num_of_sequences=8,
                              shard=False))
    assert 0 < len(fin) < 100
    inf = iter(D.PackedStream(tok, rows, seq_length=64, infinite=True, chars_per_token=1.0, num_of_sequences=8,
                              shard=False))
    assert len([next(inf) for _ in range(3 * len(fin))]) == 3 * len(fin)


def test_packed_stream_shards_rows_per_rank(tmp_path, monkeypatch):
    tok = D.ByteTokenizer()
    rows = D.Rows(_corpus(tmp_path, 400))

    def questions(rank):
        monkeypatch.setattr(D, "_dist_shard", lambda: (rank, 2))
        ds = D.PackedStream(tok, rows, seq_length=64, infinite=False, chars_per_token=1.0, num_of_sequences=8)
        text = "".join(tok.decode(s["input_ids"].tolist()) for s in ds)
        return {t[:6] for t in text.split("Question: ")[1:] if t[:1] == "q" and len(t) >= 6}

    q0, q1 = questions(0), questions(1)
    assert q0 and q1 and not q0 & q1
    assert all(int(q[1:]) % 2 == 0 for q in q0) and all(int(q[1:]) % 2 == 1 for q in q1)


def test_sft_entrypoint_streams_a_local_jsonl(tmp_path):
    import os

    import sft_llama2

    path = _corpus(tmp_path, 300)
    out = str(tmp_path / "sft")
    sft_llama2.main(["--model_name", "llama-tiny", "--dataset_name", path, "--seq_length", "64", "--size_valid_set",
                     "10", "--shuffle_buffer", "50", "--output_dir", out, "--max_steps", "3",
                     "--per_device_train_batch_size", "2", "--use_cpu", "--report_to", "none", "--lion",
                     "--async_grad", "--logging_steps", "1", "--save_strategy", "no"])
    assert os.path.isfile(os.path.join(out, "final_checkpoint", "adapter_model.safetensors"))
