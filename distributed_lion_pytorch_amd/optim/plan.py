"""Flat multi-tensor plan: where every parameter's sign bits live on the wire.

The reference issues one ``all_gather`` per parameter tensor (148 for GPT-2,
291 for Llama-2-7B).  Here all parameters that share a param
group and dtype are laid out in one flat *bit space*, cut into a few large
buckets, and each bucket is encoded by one kernel launch and exchanged by one
collective.  Parameter storage is never re-pointed (HF ``save_pretrained`` and
tied weights keep working, SURVEY §7.4 risk 3): kernels reach the tensors
through a pointer table (``seg`` rows) instead.

Layout rules (shared with csrc/lion_kernels.hip):
  * a tensor of ``n`` elements owns ``ceil(n / 2048) * 2048`` bits; its bits
    start at bucket-relative element ``bit_off`` (a multiple of 2048);
  * a bucket's byte size is padded to a multiple of ``256 * world`` so the
    all-to-all shards are 256-byte aligned and 4-byte divisible;
  * kernels run over fixed 8192-element chunks (one 256-thread block each).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import torch

ALIGN_ELEMS = 2048
CHUNK_ELEMS = 8192
SEG_COLS = 8


def _ceil(a: int, b: int) -> int:
    return (a + b - 1) // b * b


@dataclass
class Segment:
    param: torch.Tensor
    numel: int
    bit_off: int  # bucket-relative, in elements (== bits)
    index: int  # row in the seg table


@dataclass
class Bucket:
    index: int
    group: int  # param-group index (hyper-parameters are uniform in a bucket)
    dtype: torch.dtype
    segments: List[Segment]
    byte_off: int  # offset of this bucket in the flat send buffer
    nbytes: int  # padded byte size of this bucket's bit plane
    chunk_off: int = 0  # first row of this bucket in the chunk table
    n_chunks: int = 0
    chunks: List[tuple] = field(default_factory=list)

    @property
    def numel(self) -> int:
        return sum(s.numel for s in self.segments)


class FlatPlan:
    """Bucketed bit-space layout for a fixed list of parameters.

    ``entries`` is a list of ``(param, group_index)`` in optimizer order; all
    ranks build the identical plan because they iterate the same param groups.
    """

    def __init__(self, entries: Sequence[tuple], world: int, bucket_bytes: int = 32 << 20,
                 device: Optional[torch.device] = None):
        self.world = max(1, int(world))
        self.bucket_bytes = max(ALIGN_ELEMS // 8, int(bucket_bytes))
        self.device = device if device is not None else (entries[0][0].device if entries else torch.device("cpu"))
        self.params = [p for p, _ in entries]
        self.key = self.make_key(entries)
        pad_unit = 256 * self.world

        # group by (param group, dtype) preserving order; identical on every rank
        order: dict = {}
        for p, gi in entries:
            order.setdefault((gi, p.dtype), []).append(p)

        self.buckets: List[Bucket] = []
        self.segments: List[Segment] = []
        byte_off = 0
        for (gi, dtype), plist in order.items():
            cur: List[torch.Tensor] = []
            cur_bits = 0
            for p in plist:
                region = _ceil(p.numel(), ALIGN_ELEMS)
                if cur and (cur_bits + region) // 8 > self.bucket_bytes:
                    byte_off = self._close(gi, dtype, cur, byte_off, pad_unit)
                    cur, cur_bits = [], 0
                cur.append(p)
                cur_bits += region
            if cur:
                byte_off = self._close(gi, dtype, cur, byte_off, pad_unit)
        self.total_bytes = byte_off

        # chunk table
        chunk_rows = []
        for b in self.buckets:
            b.chunk_off = len(chunk_rows)
            for s in b.segments:
                for start in range(0, _ceil(s.numel, ALIGN_ELEMS), CHUNK_ELEMS):
                    chunk_rows.append((s.index, start))
            b.n_chunks = len(chunk_rows) - b.chunk_off
        self.n_seg = len(self.segments)
        self.seg_off = 0
        self.chunk_off = SEG_COLS * self.n_seg
        self._chunk_rows = chunk_rows
        self.total_chunks = len(chunk_rows)
        self.meta_numel = self.chunk_off + 2 * len(chunk_rows)
        self._meta_dev: Optional[torch.Tensor] = None
        self._ptr_key = None

    @staticmethod
    def make_key(entries) -> tuple:
        return tuple((id(p), gi, p.dtype, p.numel()) for p, gi in entries)

    def _close(self, gi, dtype, plist, byte_off, pad_unit) -> int:
        segs = []
        bit = 0
        for p in plist:
            s = Segment(param=p, numel=p.numel(), bit_off=bit, index=len(self.segments))
            self.segments.append(s)
            segs.append(s)
            bit += _ceil(p.numel(), ALIGN_ELEMS)
        nbytes = _ceil(bit // 8, pad_unit)
        self.buckets.append(Bucket(index=len(self.buckets), group=gi, dtype=dtype, segments=segs,
                                   byte_off=byte_off, nbytes=nbytes))
        return byte_off + nbytes

    # ------------------------------------------------------------ device meta
    def meta(self, grads: Sequence[torch.Tensor], moms: Sequence[torch.Tensor]) -> torch.Tensor:
        """Device int64 table [seg rows | chunk rows].  The chunk rows depend
        only on the layout and are uploaded once; the seg rows (pointers) are
        re-uploaded when any pointer changed (grads are re-allocated when
        zero_grad sets None) -- 8 int64 per tensor from a persistent pinned
        buffer, asynchronously (the host side costs ~0.1 ms per step)."""
        ptr_key = tuple(g.data_ptr() for g in grads) + tuple(m.data_ptr() for m in moms) + tuple(
            p.data_ptr() for p in self.params)
        if self._meta_dev is not None and ptr_key == self._ptr_key:
            return self._meta_dev
        rows = []
        for s, g, m in zip(self.segments, grads, moms):
            p = s.param
            for t in (g, m):
                if t.dtype != p.dtype or t.numel() != p.numel() or not t.is_contiguous():
                    raise ValueError("dlion: grad/momentum must be contiguous and match the parameter dtype/numel")
            if not p.is_contiguous():
                raise ValueError("dlion: parameters must be contiguous")
            vec = p.data_ptr() % 16 == 0 and g.data_ptr() % 16 == 0 and m.data_ptr() % 16 == 0 and p.numel() % 8 == 0
            rows.append((p.data_ptr(), g.data_ptr(), m.data_ptr(), p.numel(), s.bit_off, int(vec), 0, 0))
        seg = torch.tensor(rows, dtype=torch.int64).reshape(-1) if rows else torch.empty(0, dtype=torch.int64)
        n = SEG_COLS * self.n_seg
        if self.device.type != "cuda":
            if self._meta_dev is None:
                self._meta_dev = torch.empty(self.meta_numel, dtype=torch.int64)
                if self._chunk_rows:
                    self._meta_dev[self.chunk_off:] = torch.tensor(self._chunk_rows, dtype=torch.int64).reshape(-1)
            self._meta_dev[:n] = seg
        else:
            if self._meta_dev is None:
                host = torch.empty(self.meta_numel, dtype=torch.int64)
                if self._chunk_rows:
                    host[self.chunk_off:] = torch.tensor(self._chunk_rows, dtype=torch.int64).reshape(-1)
                self._meta_dev = torch.empty(self.meta_numel, dtype=torch.int64, device=self.device)
                self._meta_dev.copy_(host.pin_memory(), non_blocking=True)
                self._seg_host = torch.empty(max(1, n), dtype=torch.int64).pin_memory()
                self._seg_event = torch.cuda.Event()
            else:
                self._seg_event.synchronize()  # the previous upload from the pinned buffer is done
            self._seg_host[:n] = seg
            self._meta_dev[:n].copy_(self._seg_host[:n], non_blocking=True)
            self._seg_event.record()
        self._ptr_key = ptr_key
        return self._meta_dev

    def bucket_grads(self, b: Bucket, grads_by_seg):
        return [grads_by_seg[s.index] for s in b.segments]

    def describe(self) -> dict:
        return {
            "n_tensors": self.n_seg,
            "n_buckets": len(self.buckets),
            "total_bytes": self.total_bytes,
            "numel": sum(s.numel for s in self.segments),
            "bucket_bytes": [b.nbytes for b in self.buckets],
        }
