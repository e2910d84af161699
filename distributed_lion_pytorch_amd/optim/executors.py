"""Backends that execute the plan's per-bucket work.

``HipExecutor`` drives the gfx950 kernels (one launch per bucket and phase);
``TorchExecutor`` runs the PyTorch oracle segment by segment -- it is the CPU
path (gloo tests) and the numerics reference for the kernels.  Both write the
same bit layout, so the exchange layer is backend-agnostic.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch

from ..ops import hip
from ..ops import reference as ref
from .plan import ALIGN_ELEMS, Bucket, FlatPlan


@dataclass
class HParams:
    lr: float
    wd: float
    beta1: float
    beta2: float

    @property
    def decay(self) -> float:
        return 1.0 - self.lr * self.wd


def _region_bytes(numel: int) -> int:
    return (numel + ALIGN_ELEMS - 1) // ALIGN_ELEMS * ALIGN_ELEMS // 8


class HipExecutor:
    name = "hip"

    def __init__(self, plan: FlatPlan):
        self.plan = plan
        self.ops = hip.ops()

    def _chunk_off(self, b: Bucket) -> int:
        return self.plan.chunk_off + 2 * b.chunk_off

    def local(self, meta, b: Bucket, hp: HParams, grads=None, moms=None, gscale=None) -> None:
        self.ops.lion_local(meta, self.plan.seg_off, self._chunk_off(b), b.n_chunks, hip.DTYPE_CODE[b.dtype],
                            hp.decay, -hp.lr, hp.beta1, 1.0 - hp.beta1, hp.beta2, 1.0 - hp.beta2, gscale)

    def encode(self, meta, b: Bucket, bits: torch.Tensor, hp: HParams, update_m: bool = True,
               stochastic: bool = False, rr: float = 0.0, seed: int = 0, step: int = 0,
               grads=None, moms=None, gscale=None) -> None:
        self.ops.lion_encode(meta, self.plan.seg_off, self._chunk_off(b), b.n_chunks, hip.DTYPE_CODE[b.dtype], bits,
                             hp.beta1, 1.0 - hp.beta1, hp.beta2, 1.0 - hp.beta2, update_m, stochastic, rr,
                             seed & 0x7FFFFFFFFFFFFFFF, step & 0xFFFFFFFF, gscale)

    def grad_sumsq(self, meta, b: Bucket, partial: torch.Tensor) -> None:
        """partial[b.chunk_off + i] = sum of g^2 over chunk i of bucket b."""
        self.ops.grad_sumsq(meta, self.plan.seg_off, self._chunk_off(b), b.n_chunks, hip.DTYPE_CODE[b.dtype],
                            partial, b.chunk_off)

    def clip_coef(self, partial: torch.Tensor, n: int, max_norm: float, out: torch.Tensor) -> None:
        self.ops.clip_coef(partial, n, max_norm, out)

    def apply(self, meta, b: Bucket, planes: torch.Tensor, stride: int, alive: torch.Tensor, mode: int, tie: int,
              neg: Optional[torch.Tensor], hp: HParams, own: Optional[torch.Tensor] = None,
              agree: Optional[torch.Tensor] = None) -> None:
        self.ops.lion_vote_apply(meta, self.plan.seg_off, self._chunk_off(b), b.n_chunks, hip.DTYPE_CODE[b.dtype],
                                 planes, stride, alive, mode, tie, neg, hp.decay, -hp.lr, own, agree)

    def vote_reduce(self, recv: torch.Tensor, nbytes: int, alive: torch.Tensor, tie: int, out: torch.Tensor,
                    neg_out: Optional[torch.Tensor], ties: Optional[torch.Tensor] = None) -> None:
        self.ops.vote_reduce(recv, nbytes, alive, tie, out, neg_out, ties)


class TorchExecutor:
    name = "torch"

    def __init__(self, plan: FlatPlan):
        self.plan = plan

    def local(self, meta, b: Bucket, hp: HParams, grads=None, moms=None, gscale=None) -> None:
        assert gscale is None, "the torch executor clips gradients in place (Lion.clip_grad_norm_)"
        for s in b.segments:
            ref.update_fn(s.param, grads[s.index], moms[s.index], hp.lr, hp.wd, hp.beta1, hp.beta2)

    def encode(self, meta, b: Bucket, bits: torch.Tensor, hp: HParams, update_m: bool = True,
               stochastic: bool = False, rr: float = 0.0, seed: int = 0, step: int = 0,
               grads=None, moms=None, gscale=None) -> None:
        assert gscale is None, "the torch executor clips gradients in place (Lion.clip_grad_norm_)"
        gen = None
        if stochastic:
            gen = torch.Generator(device=bits.device)
            gen.manual_seed((seed * 1_000_003 + step) & 0x7FFFFFFFFFFFFFFF)
        for s in b.segments:
            g, m = grads[s.index], moms[s.index]
            if stochastic:
                # rr = (1 + 1/b1) * max_grad_norm  ->  recover max_grad_norm for the oracle
                mgn = rr / (1 + 1 / hp.beta1)
                vb = ref.stochastic_bits(g, m, hp.beta1, mgn, gen)
            else:
                vb = ref.sign_bits(g, m, hp.beta1)
            nb = _region_bytes(s.numel)
            o = s.bit_off // 8
            bits[o:o + nb] = ref.pack_bits(vb, nb * 8)
            if update_m:
                ref.momentum_update_(g, m, hp.beta2)

    def apply(self, meta, b: Bucket, planes: torch.Tensor, stride: int, alive: torch.Tensor, mode: int, tie: int,
              neg: Optional[torch.Tensor], hp: HParams, own: Optional[torch.Tensor] = None,
              agree: Optional[torch.Tensor] = None) -> None:
        w = planes.numel() // stride if mode != ref.VOTE_PREVOTED else 1
        pl = planes.reshape(w, stride)
        for s in b.segments:
            o, nb = s.bit_off // 8, _region_bytes(s.numel)
            if mode == ref.VOTE_PREVOTED:
                pos = ref.unpack_bits(pl[0, o:o + nb], s.numel)
                ngb = None if neg is None else ref.unpack_bits(neg[o:o + nb], s.numel)
                delta = ref.prevoted_delta(pos, ngb)
            else:
                bits = ref.unpack_bits(pl[:, o:o + nb], s.numel)
                delta = ref.vote_delta(bits, alive, mode, tie)
            if agree is not None and own is not None:
                mine = ref.unpack_bits(own[o:o + nb], s.numel)
                agree[0] += ((mine.float() * 2 - 1) * delta > 0).sum().to(agree.dtype)
                if mode != ref.VOTE_PREVOTED:  # pre-voted planes: K4 counted the ties
                    live = alive.to(torch.bool)
                    twice = 2 * bits[live].to(torch.int64).sum(0)
                    agree[1] += ((twice == int(live.sum())) & (int(live.sum()) > 0)).sum().to(agree.dtype)
            ref.apply_delta_(s.param, delta.to(s.param.device), hp.lr, hp.wd)

    def vote_reduce(self, recv: torch.Tensor, nbytes: int, alive: torch.Tensor, tie: int, out: torch.Tensor,
                    neg_out: Optional[torch.Tensor], ties: Optional[torch.Tensor] = None) -> None:
        w = alive.numel()
        bits = ref.unpack_bits(recv[: w * nbytes].view(w, nbytes))
        pos, ngb = ref.vote_reduce_bits(bits, alive, tie)
        if ties is not None:
            live = alive.to(torch.bool)
            n_live = int(live.sum())
            twice = 2 * bits[live].to(torch.int64).sum(0)
            ties += ((twice == n_live) & (n_live > 0)).sum().to(ties.dtype)
        out[:nbytes] = ref.pack_bits(pos)
        if neg_out is not None:
            neg_out[:nbytes] = ref.pack_bits(ngb)


def make_executor(plan: FlatPlan, backend: str = "auto"):
    """backend: 'hip' | 'torch' | 'auto' (HIP on a GPU, loudly required)."""
    if backend == "torch":
        return TorchExecutor(plan)
    if backend == "hip":
        return HipExecutor(plan)
    if plan.device.type == "cuda":
        if hip.available() or not hip.fallback_allowed():
            return HipExecutor(plan)  # raises with a clear message if the .so is missing
        return TorchExecutor(plan)
    return TorchExecutor(plan)
