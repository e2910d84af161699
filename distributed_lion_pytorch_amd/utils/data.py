"""Offline data plumbing: a byte-level tokenizer, synthetic corpora in the shapes
the reference's entrypoints consume, CLM block grouping and SFT packing.

There is no network in this environment (no hub tokenizers or datasets), so:
* :class:`ByteTokenizer` is a dependency-free HF-style tokenizer (UTF-8 bytes +
  BOS/EOS/PAD) used when no local tokenizer directory is given;
* ``synthetic_*`` build deterministic datasets of the reference's shapes:
  CLM token blocks (run_clm.py:509-544 group_texts; ``clm_blocks`` groups real
  text the same way), stack-exchange-like
  "Question/Answer" SFT text (sft_llama2.py:93-96) and prompt/chosen/rejected
  DPO triples (dpo_llama2.py:84-125).
"""
from __future__ import annotations

import json
import os
import random
from typing import Dict, Iterable, List, Optional, Sequence

import torch
from torch.utils.data import Dataset

_WORDS = ("the of and to in is for on that with as by at from this be are it an or was which can not "
          "model data train gpu memory kernel vote sign update rank worker gradient optimizer lion bit "
          "python code error function value loop array tensor device stream layer batch token").split()


class ByteTokenizer:
    """UTF-8 byte tokenizer with HF-tokenizer-compatible call/pad/save API."""

    vocab_size = 259
    bos_token_id, eos_token_id, pad_token_id = 256, 257, 258
    bos_token, eos_token, pad_token = "<s>", "</s>", "<pad>"
    padding_side = "right"
    model_max_length = 1 << 30
    name_or_path = "byte-tokenizer"

    def __len__(self) -> int:
        return self.vocab_size

    def encode(self, text: str, add_special_tokens: bool = False) -> List[int]:
        ids = list(text.encode("utf-8"))
        return [self.bos_token_id] + ids if add_special_tokens else ids

    def decode(self, ids: Sequence[int], skip_special_tokens: bool = True) -> str:
        b = bytes(i for i in ids if i < 256)
        return b.decode("utf-8", errors="replace")

    def __call__(self, text, truncation: bool = False, max_length: Optional[int] = None,
                 add_special_tokens: bool = False, padding=False, return_tensors=None, **_) -> Dict:
        single = isinstance(text, str)
        texts = [text] if single else list(text)
        ids = [self.encode(t, add_special_tokens) for t in texts]
        if truncation and max_length:
            ids = [x[:max_length] for x in ids]
        if padding:
            width = max_length if padding == "max_length" and max_length else max(len(x) for x in ids)
            ids = [x + [self.pad_token_id] * (width - len(x)) for x in ids]
        mask = [[0 if t == self.pad_token_id else 1 for t in x] for x in ids]
        out = {"input_ids": ids[0] if single else ids, "attention_mask": mask[0] if single else mask}
        if return_tensors == "pt":
            out = {k: torch.tensor(v) for k, v in out.items()}
        return out

    def save_pretrained(self, out_dir: str) -> None:
        os.makedirs(out_dir, exist_ok=True)
        with open(os.path.join(out_dir, "byte_tokenizer.json"), "w") as f:
            json.dump({"type": "ByteTokenizer", "vocab_size": self.vocab_size}, f)


def load_tokenizer(name_or_path: Optional[str]):
    """Local HF tokenizer directory if it exists, else the byte tokenizer."""
    if name_or_path and os.path.isdir(name_or_path):
        try:
            from transformers import AutoTokenizer

            return AutoTokenizer.from_pretrained(name_or_path)
        except Exception:
            pass
    return ByteTokenizer()


# ---------------------------------------------------------------- CLM data
class SyntheticCLMDataset(Dataset):
    """Deterministic random token blocks: {'input_ids', 'labels'} of length block_size."""

    def __init__(self, n: int, block_size: int, vocab_size: int, seed: int = 0):
        self.n, self.block, self.vocab, self.seed = n, block_size, vocab_size, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        ids = torch.randint(0, self.vocab, (self.block,), generator=g)
        return {"input_ids": ids, "labels": ids.clone()}


# The reference's CLM preprocessing (run_clm.py:463-544): ``datasets.map`` of
# the tokenizer, then of group_texts, both ``batched=True`` -- i.e. per batch
# of 1000 texts the token lists are concatenated (no separator token) and cut
# into block_size chunks, the remainder of EACH batch dropped -- with
# ``num_proc=preprocessing_num_workers`` and ``load_from_cache_file=not
# overwrite_cache``.  Same stream here, without the hub datasets machinery:
# batches tokenized in a spawn-started worker pool (no fork of a process that
# may hold a GPU context) and the resulting blocks cached as one .npy keyed by
# the texts, the tokenizer and block_size.
MAP_BATCH = 1000


class TokenBlocks(Dataset):
    """[n, block_size] token blocks as {'input_ids', 'labels'} rows."""

    def __init__(self, blocks: torch.Tensor):
        self.data = blocks

    def __len__(self):
        return self.data.shape[0]

    def __getitem__(self, i):
        ids = self.data[i].long()
        return {"input_ids": ids, "labels": ids.clone()}


def _group_batch(token_lists: Sequence[Sequence[int]], block_size: int) -> List[List[int]]:
    flat: List[int] = []
    for ids in token_lists:
        flat.extend(ids)
    n = len(flat) // block_size
    return [flat[i * block_size:(i + 1) * block_size] for i in range(n)]


_POOL_TOKENIZER = None


def _pool_init(tokenizer):
    global _POOL_TOKENIZER
    _POOL_TOKENIZER = tokenizer


def _pool_batch(args):
    texts, block_size = args
    return _group_batch(_POOL_TOKENIZER(list(texts))["input_ids"], block_size)


def _blocks_cache_key(texts: Sequence[str], tokenizer, block_size: int) -> str:
    import hashlib

    h = hashlib.sha256()
    ident = (type(tokenizer).__name__, str(getattr(tokenizer, "name_or_path", "")), len(tokenizer), block_size, MAP_BATCH)
    h.update(repr(ident).encode())
    for t in texts:
        h.update(t.encode("utf-8", "surrogatepass"))
        h.update(b"\x00")
    return h.hexdigest()[:24]


def default_cache_dir() -> str:
    base = os.environ.get("HF_DATASETS_CACHE") or os.path.join(
        os.environ.get("HF_HOME", os.path.join(os.path.expanduser("~"), ".cache", "huggingface")), "datasets")
    return os.path.join(base, "dlion_clm")


def clm_blocks(texts: Sequence[str], tokenizer, block_size: int, num_workers: Optional[int] = None,
               cache_dir: Optional[str] = None, overwrite_cache: bool = False) -> TokenBlocks:
    """Tokenize + group ``texts`` exactly as the reference's two batched maps do
    (see above).  ``num_workers`` > 1 tokenizes batches in parallel processes;
    ``cache_dir`` (None: no cache) holds the blocks for reuse unless
    ``overwrite_cache``."""
    import numpy as np

    texts = list(texts)
    path = None
    if cache_dir is not None:
        path = os.path.join(cache_dir, f"clm-{_blocks_cache_key(texts, tokenizer, block_size)}.npy")
        if not overwrite_cache and os.path.isfile(path):
            return TokenBlocks(torch.from_numpy(np.load(path)))
    batches = [texts[i:i + MAP_BATCH] for i in range(0, len(texts), MAP_BATCH)]
    if num_workers is not None and num_workers > 1 and len(batches) > 1:
        import multiprocessing as mp

        with mp.get_context("spawn").Pool(min(num_workers, len(batches)), initializer=_pool_init,
                                          initargs=(tokenizer,)) as pool:
            grouped = pool.map(_pool_batch, [(b, block_size) for b in batches])
    else:
        grouped = [_group_batch(tokenizer(b)["input_ids"], block_size) for b in batches]
    rows = [r for g in grouped for r in g]
    dtype = np.int32 if len(tokenizer) < 2 ** 31 else np.int64
    arr = np.asarray(rows, dtype=dtype).reshape(len(rows), block_size)
    if path is not None:
        os.makedirs(cache_dir, exist_ok=True)
        tmp = f"{path}.{os.getpid()}.tmp.npy"
        np.save(tmp, arr)
        os.replace(tmp, path)  # atomic: ranks that read concurrently see a whole file or none
    return TokenBlocks(torch.from_numpy(arr))


# ------------------------------------------------- run_clm local files
# The reference loads --train_file / --validation_file by extension through
# ``datasets.load_dataset(extension, data_files=...)`` ("txt" -> the "text"
# builder with ``keep_linebreaks``; csv; json) and, without a validation file,
# carves ``train[:p%]`` / ``train[p%:]`` out of the train file
# (/root/reference/run_clm.py:343-381).  The text column is "text" if present,
# else the first column (:455-458).  Same here, offline: ``datasets`` reads
# local files without the hub; without ``datasets`` a small reader of the same
# three formats stands in (blank lines stay rows, as in the text builder).
def file_builder(path: str) -> str:
    """The ``datasets`` builder name for a data file (reference: its extension,
    ``txt`` -> ``text``; ``jsonl`` is read by the json builder too)."""
    ext = path.rsplit(".", 1)[-1].lower()
    return {"txt": "text", "jsonl": "json"}.get(ext, ext)


def text_column(columns: Sequence[str]) -> str:
    cols = list(columns)
    if not cols:
        raise ValueError("the data file has no columns")
    return "text" if "text" in cols else cols[0]


def _fallback_rows(builder: str, path: str, keep_linebreaks: bool) -> List[Dict]:
    """The three builders' row semantics without ``datasets``."""
    import csv

    if builder == "text":
        with open(path, encoding="utf-8") as f:
            return [{"text": ln if keep_linebreaks else ln.rstrip("\n")} for ln in f]
    if builder == "json":
        with open(path, encoding="utf-8") as f:
            head = f.read(1)
            while head and head.isspace():
                head = f.read(1)
            f.seek(0)
            if head == "[":
                return list(json.load(f))
            return [json.loads(ln) for ln in f if ln.strip()]
    if builder == "csv":
        with open(path, encoding="utf-8", newline="") as f:
            return list(csv.DictReader(f))
    raise ValueError(f"unsupported data file type {builder!r} (csv, json, jsonl, txt)")


def _percent_split(n: int, pct: float):
    """HF percent slicing boundary (``train[:p%]``: rounded to the closest row)."""
    return int(round(n * pct / 100.0))


def load_local_splits(train_file: Optional[str], validation_file: Optional[str], keep_linebreaks: bool = True,
                      validation_split_percentage: float = 5, streaming: bool = False,
                      cache_dir: Optional[str] = None):
    """(train_rows, validation_rows, text_column) for run_clm's local files.

    Without streaming the rows are ``datasets`` Datasets (or lists of dicts);
    with streaming they are lazy re-iterable row sources (``datasets``
    IterableDataset ``take`` / ``skip``): nothing of the corpus is held in
    memory.  The validation rows without a validation file are the first
    ``validation_split_percentage`` percent of the train file, exactly the
    reference's ``train[:p%]`` / ``train[p%:]`` (a streaming run counts the
    rows in one lazy pass to place that boundary)."""
    src = train_file if train_file is not None else validation_file
    if src is None:
        raise ValueError("no data file given")
    builder = file_builder(src)
    kw = {"keep_linebreaks": keep_linebreaks} if builder == "text" else {}
    files = {}
    if train_file is not None:
        files["train"] = train_file
    if validation_file is not None:
        files["validation"] = validation_file
    try:
        import datasets
    except ImportError:  # pragma: no cover - datasets is installed in this image
        datasets = None
    if datasets is None:
        raw = {k: _fallback_rows(builder, v, keep_linebreaks) for k, v in files.items()}
        tr, va = raw.get("train"), raw.get("validation")
        if va is None and tr is not None:
            n_val = _percent_split(len(tr), validation_split_percentage)
            tr, va = tr[n_val:], tr[:n_val]
        cols = list((tr or va)[0].keys()) if (tr or va) else ["text"]
        return tr, va, text_column(cols)
    if streaming:
        raw = datasets.load_dataset(builder, data_files=files, streaming=True, **kw)
        tr, va = raw.get("train"), raw.get("validation")
        if va is None and tr is not None:
            n_val = _percent_split(sum(1 for _ in tr), validation_split_percentage)
            tr, va = tr.skip(n_val), tr.take(n_val)
        probe = tr if tr is not None else va
        cols = probe.column_names
        if cols is None:  # features resolved from the first row
            first = next(iter(probe), None)
            cols = list(first.keys()) if first is not None else ["text"]
        return tr, va, text_column(cols)
    raw = datasets.load_dataset(builder, data_files=files, cache_dir=cache_dir, **kw)
    tr, va = raw.get("train"), raw.get("validation")
    if va is None and tr is not None:
        p = validation_split_percentage
        va = datasets.load_dataset(builder, data_files=files, split=f"train[:{p}%]", cache_dir=cache_dir, **kw)
        tr = datasets.load_dataset(builder, data_files=files, split=f"train[{p}%:]", cache_dir=cache_dir, **kw)
    return tr, va, text_column((tr if tr is not None else va).column_names)


# ------------------------------------------------- named SFT / DPO datasets
# The reference reads ``load_dataset(dataset_name, data_dir=subset,
# split=split, streaming=..., num_proc=...)`` (sft_llama2.py:99-107,
# dpo_llama2.py:102-107).  Offline the name is a local file or a local copy of
# the dataset repository (e.g. a mirror of lvwerra/stack-exchange-paired with
# its data/finetune, data/rl, data/evaluation parquet shards); a hub name is
# tried too (it resolves when the dataset sits in the HF cache).  Anything
# else is an error: training on the synthetic corpus must be asked for
# (``--synthetic_data``), never a silent fallback.
class DatasetUnavailable(FileNotFoundError):
    pass


def load_named_rows(name: str, data_dir: Optional[str] = None, split: str = "train", streaming: bool = False,
                    num_workers: Optional[int] = None, cache_dir: Optional[str] = None):
    """Re-iterable dict rows of ``name``:

    * a json-lines / json file: read lazily by :class:`Rows` (``data_dir``
      does not apply to a single file);
    * another data file (parquet, csv, txt): ``datasets`` by extension;
    * a directory saved by ``Dataset.save_to_disk``: ``load_from_disk`` (its
      ``split`` when it is a DatasetDict);
    * any other directory, or a hub name: ``datasets.load_dataset(name,
      data_dir=data_dir, split=split, streaming=streaming)`` with
      ``num_proc=num_workers`` when not streaming, like the reference.

    Raises :class:`DatasetUnavailable` when none of these resolves."""
    if not name:
        raise DatasetUnavailable("no dataset name given")
    if os.path.isfile(name):
        builder = file_builder(name)
        if builder == "json":
            return Rows(name)
        import datasets

        kw = {"keep_linebreaks": True} if builder == "text" else {}
        return datasets.load_dataset(builder, data_files={"train": name}, split="train", streaming=streaming,
                                     cache_dir=cache_dir, **kw)
    try:
        import datasets
    except ImportError as e:  # pragma: no cover - datasets is installed in this image
        raise DatasetUnavailable(f"dataset {name!r} needs the `datasets` package ({e})") from e
    if os.path.isdir(name):
        if os.path.isfile(os.path.join(name, "dataset_dict.json")) or \
                os.path.isfile(os.path.join(name, "state.json")):
            ds = datasets.load_from_disk(name)
            if isinstance(ds, datasets.DatasetDict):
                ds = ds[split]
            return ds.to_iterable_dataset() if streaming else ds
        if data_dir and not os.path.isdir(os.path.join(name, data_dir)):
            raise DatasetUnavailable(f"dataset directory {name!r} has no {data_dir!r} subdirectory")
    try:
        return datasets.load_dataset(name, data_dir=data_dir, split=split, streaming=streaming,
                                     num_proc=None if streaming else num_workers, cache_dir=cache_dir)
    except Exception as e:  # offline hub name, empty directory, unknown split
        raise DatasetUnavailable(
            f"dataset {name!r} (data_dir={data_dir!r}, split={split!r}) could not be loaded: "
            f"{type(e).__name__}: {e}. Point --dataset_name at a local file or dataset directory, "
            "or pass --synthetic_data to train on the synthetic corpus") from e


def _pair_length_ok(r, max_length: int) -> bool:
    return (len(r["prompt"]) + len(r["chosen"]) <= max_length
            and len(r["prompt"]) + len(r["rejected"]) <= max_length)


def stack_exchange_pairs_dataset(ds, max_length: int, num_proc: Optional[int] = None):
    """:func:`stack_exchange_pairs` + the reference's length filter for a
    ``datasets.Dataset``, as its batched ``map`` / ``filter`` (dpo_llama2.py:
    120-125, :158-161): the rows stay in Arrow (memory-mapped) instead of a
    Python list -- the stack-exchange-paired rl split has millions of rows."""
    cols = list(ds.column_names)
    if {"prompt", "chosen", "rejected"} <= set(cols):
        out = ds.select_columns(["prompt", "chosen", "rejected"])
    elif {"question", "response_j", "response_k"} <= set(cols):
        def to_pairs(b):
            return {"prompt": ["Question: " + q + "\n\nAnswer: " for q in b["question"]],
                    "chosen": b["response_j"], "rejected": b["response_k"]}

        out = ds.map(to_pairs, batched=True, num_proc=num_proc, remove_columns=cols)
    else:
        raise KeyError("a DPO row needs prompt/chosen/rejected or question/response_j/response_k, "
                       f"got columns {sorted(cols)}")
    return out.filter(lambda r: _pair_length_ok(r, max_length), num_proc=num_proc)


def stack_exchange_pairs(rows):
    """DPO rows in trl's prompt / chosen / rejected form.  Rows of the
    stack-exchange-paired layout are mapped like the reference
    (dpo_llama2.py:113-118): prompt = "Question: " + question + "\\n\\nAnswer: ",
    chosen = response_j, rejected = response_k; rows that already carry
    prompt / chosen / rejected pass through."""
    out = []
    for r in rows:
        if "prompt" in r and "chosen" in r and "rejected" in r:
            out.append({"prompt": r["prompt"], "chosen": r["chosen"], "rejected": r["rejected"]})
        elif "question" in r and "response_j" in r and "response_k" in r:
            out.append({"prompt": "Question: " + r["question"] + "\n\nAnswer: ",
                        "chosen": r["response_j"], "rejected": r["response_k"]})
        else:
            raise KeyError("a DPO row needs prompt/chosen/rejected or question/response_j/response_k, "
                           f"got columns {sorted(r)}")
    return out


def column_texts(rows, col: str) -> List[str]:
    """A column of a Dataset / list of row dicts as a list of strings."""
    if rows is None:
        return []
    if hasattr(rows, "column_names") and not isinstance(rows, list):
        return list(rows[col])
    return [r[col] for r in rows]


class CLMStream(torch.utils.data.IterableDataset):
    """run_clm's ``--streaming`` pipeline on a lazy row source: the
    reference's two batched maps (tokenize, then group_texts over 1000-text
    batches with each batch's remainder dropped, run_clm.py:463-544) applied
    one batch at a time, so at most ``map_batch`` texts and their tokens are
    held (``peak_buffer_rows`` / ``peak_buffer_tokens`` record it) -- a corpus
    larger than memory streams through.

    With ``shard`` (training) every rank runs the same deterministic block
    stream and keeps blocks ``i % W == rank`` from each complete group of W,
    so all ranks yield the same number of blocks (equal step counts, no rank
    ends its epoch early) without rank 0 reading and broadcasting every batch
    (``rank_sharded``: the trainer hands it to a plain DataLoader).
    ``max_blocks`` caps the global block count (``max_train_samples``)."""

    rank_sharded = True

    def __init__(self, rows, column: str, tokenizer, block_size: int, shard: bool = True,
                 max_blocks: Optional[int] = None, map_batch: int = MAP_BATCH):
        self.rows, self.col, self.tok, self.block = rows, column, tokenizer, int(block_size)
        self.shard, self.max_blocks, self.map_batch = shard, max_blocks, int(map_batch)
        self.rank_sharded = bool(shard)
        self.peak_buffer_rows = 0
        self.peak_buffer_tokens = 0

    def _batches(self):
        buf: List[str] = []
        for row in self.rows:
            buf.append(row[self.col])
            if len(buf) == self.map_batch:
                yield buf
                buf = []
        if buf:
            yield buf

    def blocks(self):
        """The global (unsharded) block stream."""
        n = 0
        for texts in self._batches():
            self.peak_buffer_rows = max(self.peak_buffer_rows, len(texts))
            ids = self.tok(texts)["input_ids"]
            self.peak_buffer_tokens = max(self.peak_buffer_tokens, sum(len(x) for x in ids))
            for blk in _group_batch(ids, self.block):
                if self.max_blocks is not None and n >= self.max_blocks:
                    return
                n += 1
                yield blk

    def __iter__(self):
        rank, world = _dist_shard() if self.shard else (0, 1)
        group: List[List[int]] = []
        for blk in self.blocks():
            group.append(blk)
            if len(group) < world:
                continue
            x = torch.tensor(group[rank], dtype=torch.long)
            group = []
            yield {"input_ids": x, "labels": x.clone()}


# ---------------------------------------------------------------- SFT data
def _sentence(rng: random.Random, n: int) -> str:
    return " ".join(rng.choice(_WORDS) for _ in range(n))


def synthetic_qa(n: int, seed: int = 0) -> List[Dict[str, str]]:
    rng = random.Random(seed)
    return [{"question": _sentence(rng, rng.randint(8, 40)) + "?",
             "response_j": _sentence(rng, rng.randint(20, 120)) + ".",
             "response_k": _sentence(rng, rng.randint(20, 120)) + "."} for _ in range(n)]


def prepare_sample_text(example: Dict[str, str]) -> str:
    """Prompt format of the reference SFT script (sft_llama2.py:93-96)."""
    return f"Question: {example['question']}\n\nAnswer: {example['response_j']}"


class ConstantLengthDataset(Dataset):
    """Packed fixed-length training chunks (trl ConstantLengthDataset semantics,
    sft_llama2.py:122-129): samples are formatted, tokenized (with the
    tokenizer's special tokens, trl's default), joined with EOS
    and cut into ``seq_length`` blocks.  Map-style (pre-packed once), so every
    rank reads its own shard instead of rank 0 broadcasting each batch."""

    def __init__(self, tokenizer, dataset: Sequence[Dict], formatting_func=prepare_sample_text,
                 seq_length: int = 1024, eos_token_id: Optional[int] = None):
        eos = tokenizer.eos_token_id if eos_token_id is None else eos_token_id
        toks: List[int] = []
        for ex in dataset:
            toks.extend(tokenizer(formatting_func(ex), add_special_tokens=True)["input_ids"])
            toks.append(eos)
        n = max(1, len(toks) // seq_length)
        if len(toks) < seq_length:
            toks = (toks * (seq_length // max(1, len(toks)) + 1))
        self.data = torch.tensor(toks[: n * seq_length], dtype=torch.long).view(n, seq_length)

    def __len__(self):
        return self.data.shape[0]

    def __getitem__(self, i):
        return {"input_ids": self.data[i], "labels": self.data[i].clone()}


def chars_token_ratio(dataset: Iterable[Dict], tokenizer, formatting_func=prepare_sample_text,
                      nb_examples: int = 400) -> float:
    """Average characters per token over the first ``nb_examples`` rows
    (sft_llama2.py:62-75); reads only those rows of a stream."""
    import itertools

    chars = toks = 0
    for ex in itertools.islice(iter(dataset), nb_examples):
        text = formatting_func(ex)
        chars += len(text)
        toks += len(tokenizer(text)["input_ids"])
    return chars / max(1, toks)


# ------------------------------------------------------- streaming SFT data
# The reference streams its SFT corpus from the hub (sft_llama2.py:99-138):
# ``take(size_valid_set)`` is the validation set, ``skip(size_valid_set)``
# shuffled through a ``shuffle_buffer``-row buffer is the training set, and
# trl's ConstantLengthDataset packs it with ``infinite=True`` from a character
# buffer sized seq_length * chars_per_token * num_of_sequences.  Offline the
# rows come from a local json-lines file read lazily (constant memory -- a
# corpus larger than host RAM streams), each rank keeps its own 1/W of the
# rows (no rank-0 read + broadcast per batch), and the shuffle is seeded by the
# training seed (the reference's seed=None is not reproducible).
class Rows:
    """Re-iterable row source: a list, or a json-lines / json file read lazily
    (a ``.json`` array is loaded whole -- it cannot be streamed)."""

    def __init__(self, source):
        self.source = source

    def __iter__(self):
        if isinstance(self.source, str):
            if not self.source.endswith(".jsonl"):
                with open(self.source) as f:
                    yield from json.load(f)
                return
            with open(self.source) as f:
                for line in f:
                    if line.strip():
                        yield json.loads(line)
        else:
            yield from self.source


class RowSlice:
    """``datasets`` take / skip on a re-iterable: rows [start, stop)."""

    def __init__(self, rows, start: int = 0, stop: Optional[int] = None):
        self.rows, self.start, self.stop = rows, start, stop

    def __iter__(self):
        import itertools

        return itertools.islice(iter(self.rows), self.start, self.stop)


class ShuffledRows:
    """Buffer shuffle (``IterableDataset.shuffle(buffer_size, seed)``): a
    ``buffer_size``-row reservoir, each row emitted from a random slot.  Pass
    ``epoch`` k reshuffles with seed + k (``set_epoch``)."""

    def __init__(self, rows, buffer_size: int, seed: int = 0):
        self.rows, self.buffer_size, self.seed, self.epoch = rows, max(1, int(buffer_size)), int(seed), 0

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def __iter__(self):
        rng = random.Random(self.seed * 1_000_003 + self.epoch)
        buf: List = []
        for row in self.rows:
            if len(buf) < self.buffer_size:
                buf.append(row)
                continue
            i = rng.randrange(self.buffer_size)
            buf[i], row = row, buf[i]
            yield row
        rng.shuffle(buf)
        yield from buf


def random_split(rows: Sequence, test_size: float, seed: int = 0):
    """``Dataset.train_test_split(test_size)`` (sft_llama2.py:114): a seeded
    random permutation, the first ceil(test_size * n) rows for validation."""
    import math

    rows = list(rows)
    order = list(range(len(rows)))
    random.Random(seed).shuffle(order)
    n_test = max(1, math.ceil(test_size * len(rows))) if rows else 0
    return [rows[i] for i in order[n_test:]], [rows[i] for i in order[:n_test]]


def _dist_shard():
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


class PackedStream(torch.utils.data.IterableDataset):
    """trl ``ConstantLengthDataset(infinite=...)`` semantics on a row stream:
    rows are formatted into a character buffer of seq_length *
    chars_per_token * num_of_sequences, tokenized, joined with EOS and cut
    into ``seq_length`` chunks (a partial tail chunk is dropped); with
    ``infinite`` the rows restart (next shuffle epoch) when exhausted.  Each
    rank reads every row but keeps rows i % W == rank (``shard``), so ranks
    train on disjoint data with no broadcast.  ``peak_buffer_chars`` records
    the largest character buffer held (memory is bounded by it, not by the
    corpus).  Samples are tokenized with the tokenizer's default special
    tokens (trl's ``add_special_tokens=True``: a BOS per sample for Llama),
    then joined with EOS.  An infinite stream whose rank shard holds no rows
    (fewer rows than ranks) raises instead of ending: that rank would stop
    training while the others block in the vote collectives."""

    rank_sharded = True

    def __init__(self, tokenizer, rows, formatting_func=prepare_sample_text, seq_length: int = 1024,
                 infinite: bool = False, chars_per_token: float = 3.6, num_of_sequences: int = 1024,
                 eos_token_id: Optional[int] = None, shard: bool = True):
        self.tok, self.rows, self.fmt = tokenizer, rows, formatting_func
        self.seq_length, self.infinite = seq_length, infinite
        self.max_buffer_size = int(seq_length * chars_per_token * num_of_sequences)
        self.eos = tokenizer.eos_token_id if eos_token_id is None else eos_token_id
        self.shard = shard
        self.peak_buffer_chars = 0

    def _rows(self, epoch: int, rank: int, world: int):
        if hasattr(self.rows, "set_epoch"):
            self.rows.set_epoch(epoch)
        for i, row in enumerate(self.rows):
            if i % world == rank:
                yield row

    def __iter__(self):
        rank, world = _dist_shard() if self.shard else (0, 1)
        epoch, seen = 0, 0  # rows taken in the current epoch
        it = self._rows(epoch, rank, world)
        more = True
        while more:
            buf: List[str] = []
            n = 0
            while n < self.max_buffer_size:
                try:
                    text = self.fmt(next(it))
                    seen += 1
                except StopIteration:
                    if self.infinite and seen == 0:
                        raise ValueError(f"rank {rank} of {world}: no rows in this rank's shard of the "
                                         "training stream (fewer rows than ranks); an infinite stream "
                                         "cannot end on one rank only") from None
                    if not self.infinite:
                        more = False
                        break
                    epoch, seen = epoch + 1, 0
                    it = self._rows(epoch, rank, world)
                    continue
                buf.append(text)
                n += len(text)
            self.peak_buffer_chars = max(self.peak_buffer_chars, n)
            if not buf:
                break
            ids: List[int] = []
            for t in self.tok(buf, add_special_tokens=True)["input_ids"]:
                ids.extend(t)
                ids.append(self.eos)
            for i in range(0, len(ids) - self.seq_length + 1, self.seq_length):
                x = torch.tensor(ids[i:i + self.seq_length], dtype=torch.long)
                yield {"input_ids": x, "labels": x.clone()}


# ---------------------------------------------------------------- DPO data
def synthetic_paired(n: int, seed: int = 0, target_chars: Optional[int] = None) -> List[Dict[str, str]]:
    """prompt / chosen / rejected triples in the reference's format (dpo_llama2.py:84-125).
    ``target_chars``: every prompt + response is padded with words to just
    under that many characters (throughput runs at the full ``max_length``;
    the default rows are a few hundred characters)."""
    out = []
    rng = random.Random(seed + 1)
    for ex in synthetic_qa(n, seed):
        row = {"prompt": "Question: " + ex["question"] + "\n\nAnswer: ",
               "chosen": ex["response_j"], "rejected": ex["response_k"]}
        if target_chars:
            # prompt ~ 40 % of the budget, each response the rest
            row["prompt"] = _fill(rng, row["prompt"], int(0.4 * target_chars))
            for k in ("chosen", "rejected"):
                row[k] = _fill(rng, row[k], target_chars - len(row["prompt"]))
        out.append(row)
    return out


def _fill(rng: random.Random, text: str, n: int) -> str:
    """``text`` extended with random words to at most ``n`` characters (at least n - 12)."""
    while len(text) < n - 12:
        text += " " + rng.choice(_WORDS)
    return text[:n]
