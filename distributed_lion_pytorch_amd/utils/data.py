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
    sft_llama2.py:122-129): samples are formatted, tokenized, joined with EOS
    and cut into ``seq_length`` blocks.  Map-style (pre-packed once), so every
    rank reads its own shard instead of rank 0 broadcasting each batch."""

    def __init__(self, tokenizer, dataset: Sequence[Dict], formatting_func=prepare_sample_text,
                 seq_length: int = 1024, eos_token_id: Optional[int] = None):
        eos = tokenizer.eos_token_id if eos_token_id is None else eos_token_id
        toks: List[int] = []
        for ex in dataset:
            toks.extend(tokenizer(formatting_func(ex), add_special_tokens=False)["input_ids"])
            toks.append(eos)
        n = max(1, len(toks) // seq_length)
        if len(toks) < seq_length:
            toks = (toks * (seq_length // max(1, len(toks)) + 1))
        self.data = torch.tensor(toks[: n * seq_length], dtype=torch.long).view(n, seq_length)

    def __len__(self):
        return self.data.shape[0]

    def __getitem__(self, i):
        return {"input_ids": self.data[i], "labels": self.data[i].clone()}


def chars_token_ratio(dataset: Sequence[Dict], tokenizer, formatting_func=prepare_sample_text,
                      nb_examples: int = 400) -> float:
    """Average characters per token (sft_llama2.py:62-75)."""
    chars = toks = 0
    for ex in list(dataset)[:nb_examples]:
        text = formatting_func(ex)
        chars += len(text)
        toks += len(tokenizer(text)["input_ids"])
    return chars / max(1, toks)


# ---------------------------------------------------------------- DPO data
def synthetic_paired(n: int, seed: int = 0) -> List[Dict[str, str]]:
    """prompt / chosen / rejected triples in the reference's format (dpo_llama2.py:84-125)."""
    out = []
    for ex in synthetic_qa(n, seed):
        out.append({"prompt": "Question: " + ex["question"] + "\n\nAnswer: ",
                    "chosen": ex["response_j"], "rejected": ex["response_k"]})
    return out
