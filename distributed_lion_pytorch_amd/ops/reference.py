"""Pure-PyTorch oracle of the Distributed Lion semantics.

This module restates the behavioural contract of the reference optimizer
(``/root/reference/distributed_lion.py``) with plain ATen ops
so that it can serve three purposes:

1. the numerics oracle that the gfx950 kernels are tested against (bf16
   results are bit-identical because both round after every ATen-visible op);
2. the CPU execution path (gloo multi-process tests, no GPU);
3. the reference-compatible *functional* API (``update_fn``,
   ``update_fn_distributed``, ``update_fn_distributed_stoc``, ``majority_vote``,
   ``flatten_and_pad``, ``restore_flattened_tensor``), including an optional
   ``wire_dtype=torch.int64`` that reproduces the reference's 1 byte/param
   payload for A/B benchmarking.

Known reference defects are fixed here, explicitly: the stochastic path stores
and uses ``max_grad_norm`` (D2), does a real update at W == 1 (D3) and clamps
the Bernoulli probability (D4).
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch
import torch.distributed as dist

# tie rules for an even split of votes
TIE_NEGATIVE = 0  # reference parity: torch.mode over {False, True} ties -> False -> delta = -1
TIE_ZERO = 1
TIE_POSITIVE = 2
TIE_CODES = {"negative": TIE_NEGATIVE, "ref_negative": TIE_NEGATIVE, "zero": TIE_ZERO, "positive": TIE_POSITIVE}

VOTE_MAJORITY = 0
VOTE_AVERAGE = 1
VOTE_PREVOTED = 2
VOTE_CODES = {"majority": VOTE_MAJORITY, "average": VOTE_AVERAGE}


def exists(val) -> bool:
    return val is not None


# ------------------------------------------------------------------ codec
def flatten_and_pad(tensor: torch.Tensor, multiple: int = 8):
    """Flatten and zero-pad to a multiple of ``multiple`` (ref :14-24)."""
    flat = tensor.reshape(-1)
    pad = (-flat.numel()) % multiple
    if pad:
        flat = torch.cat([flat, flat.new_zeros(pad)])
    return flat, tensor.shape


def restore_flattened_tensor(padded: torch.Tensor, original_shape) -> torch.Tensor:
    """Drop padding and reshape (ref :27-31)."""
    n = 1
    for s in original_shape:
        n *= int(s)
    return padded[:n].reshape(original_shape)


_SHIFTS = {}


def _shifts(device) -> torch.Tensor:
    key = str(device)
    if key not in _SHIFTS:
        _SHIFTS[key] = torch.arange(8, dtype=torch.uint8, device=device)
    return _SHIFTS[key]


def pack_bits(bits: torch.Tensor, nbits: Optional[int] = None) -> torch.Tensor:
    """bool[n] -> uint8[ceil(nbits/8)], little-endian inside each byte.

    Element ``e`` lands in byte ``e // 8``, bit ``e % 8`` -- the reference's
    layout (ref :75-77) at 1 bit per element.
    """
    flat = bits.reshape(-1).to(torch.uint8)
    nbits = flat.numel() if nbits is None else nbits
    pad = nbits - flat.numel()
    if pad < 0:
        raise ValueError("nbits smaller than the bit count")
    pad += (-nbits) % 8
    if pad:
        flat = torch.cat([flat, flat.new_zeros(pad)])
    return (flat.view(-1, 8) << _shifts(flat.device)).sum(dim=1, dtype=torch.uint8)


def unpack_bits(packed: torch.Tensor, n: Optional[int] = None) -> torch.Tensor:
    """uint8[..., nb] -> bool[..., nb*8] (or the first ``n`` bits)."""
    out = ((packed.unsqueeze(-1) >> _shifts(packed.device)) & 1).bool()
    out = out.reshape(*packed.shape[:-1], packed.shape[-1] * 8)
    return out if n is None else out[..., :n]


def majority_vote(boolean_tensors: Sequence[torch.Tensor], tie: int = TIE_NEGATIVE) -> torch.Tensor:
    """Element-wise majority of W boolean tensors (ref :33-43).

    With the default tie rule an even split returns False, like ``torch.mode``
    in the reference.  Implemented with a popcount instead of ``stack + mode``.
    """
    count = torch.zeros(boolean_tensors[0].shape, dtype=torch.int32, device=boolean_tensors[0].device)
    for b in boolean_tensors:
        count += b.to(torch.int32)
    w = len(boolean_tensors)
    if tie == TIE_POSITIVE:
        return 2 * count >= w
    return 2 * count > w


# ------------------------------------------------------------ elementwise
def interp(grad: torch.Tensor, exp_avg: torch.Tensor, beta1: float) -> torch.Tensor:
    """beta1*m + (1-beta1)*g, rounded in the parameter dtype like the reference."""
    return exp_avg.clone().mul_(beta1).add_(grad, alpha=1 - beta1)


def sign_bits(grad: torch.Tensor, exp_avg: torch.Tensor, beta1: float) -> torch.Tensor:
    """Vote bit = sign(interp) > 0; zero and NaN vote negative (ref :68-71)."""
    return interp(grad, exp_avg, beta1) > 0


def stochastic_bits(grad, exp_avg, beta1: float, max_grad_norm: float, generator=None) -> torch.Tensor:
    """Stochastic binarization (ref :106-108), probability clamped to [0, 1] (D4)."""
    r = (1 + 1 / beta1) * max_grad_norm
    raw = interp(grad, exp_avg, beta1).float()
    prob = ((raw + r) / (2 * r)).clamp_(0.0, 1.0)
    return torch.bernoulli(prob, generator=generator) > 0


def momentum_update_(grad, exp_avg, beta2: float) -> None:
    exp_avg.mul_(beta2).add_(grad, alpha=1 - beta2)


def vote_delta(planes_bits: torch.Tensor, alive: torch.Tensor, mode: int = VOTE_MAJORITY,
               tie: int = TIE_NEGATIVE) -> torch.Tensor:
    """planes_bits: bool[W, n]; alive: bool/uint8[W]  ->  float32 delta[n].

    Matches lion_vote_apply_kernel: majority -> {+1, -1, tie}, average ->
    (2c - n_live) * (1/n_live), no voters -> 0.
    """
    alive_b = alive.to(torch.bool)
    n_live = int(alive_b.sum())
    if n_live == 0:
        return torch.zeros(planes_bits.shape[1], dtype=torch.float32, device=planes_bits.device)
    cnt = planes_bits[alive_b].to(torch.int32).sum(0)
    twice = 2 * cnt
    if mode == VOTE_AVERAGE:
        inv = torch.tensor(1.0 / n_live, dtype=torch.float32).item()
        return (twice - n_live).to(torch.float32) * inv
    tie_val = {TIE_NEGATIVE: -1.0, TIE_ZERO: 0.0, TIE_POSITIVE: 1.0}[tie]
    d = torch.full(cnt.shape, tie_val, dtype=torch.float32, device=cnt.device)
    d[twice > n_live] = 1.0
    d[twice < n_live] = -1.0
    return d


def prevoted_delta(pos_bits: torch.Tensor, neg_bits: Optional[torch.Tensor]) -> torch.Tensor:
    neg = ~pos_bits if neg_bits is None else neg_bits
    d = torch.zeros(pos_bits.shape, dtype=torch.float32, device=pos_bits.device)
    d[neg] = -1.0
    d[pos_bits] = 1.0
    return d


def vote_reduce_bits(planes_bits: torch.Tensor, alive: torch.Tensor, tie: int):
    """bool[W, n] -> (pos bool[n], neg bool[n]) -- the K4 oracle."""
    alive_b = alive.to(torch.bool)
    n_live = int(alive_b.sum())
    if n_live == 0:
        z = torch.zeros(planes_bits.shape[1], dtype=torch.bool, device=planes_bits.device)
        return z, z.clone()
    twice = 2 * planes_bits[alive_b].to(torch.int32).sum(0)
    pos = (twice > n_live) | ((twice == n_live) & (tie == TIE_POSITIVE))
    neg = (twice < n_live) | ((twice == n_live) & (tie == TIE_NEGATIVE))
    return pos, neg


def apply_delta_(p: torch.Tensor, delta: torch.Tensor, lr: float, wd: float) -> None:
    """p <- round(round(p*(1-lr*wd)) - lr*delta)  (ref :64 then :92)."""
    p.mul_(1 - lr * wd)
    p.add_(delta.view(p.shape), alpha=-lr)


# ------------------------------------------- reference-compatible functions
def update_fn(p, grad, exp_avg, lr, wd, beta1, beta2) -> None:
    """Single-node Lion step (ref :47-59); sign(0) leaves the coordinate."""
    p.mul_(1 - lr * wd)
    p.add_(interp(grad, exp_avg, beta1).sign_(), alpha=-lr)
    momentum_update_(grad, exp_avg, beta2)


def _gather_vote(bits: torch.Tensor, shape, group, wire_dtype, tie: int) -> torch.Tensor:
    packed = pack_bits(bits)
    if wire_dtype != torch.uint8:
        packed = packed.to(wire_dtype)  # int64 reproduces the reference payload (1 B/param)
    world = dist.get_world_size(group)
    bufs = [torch.empty_like(packed) for _ in range(world)]
    dist.all_gather(bufs, packed, group=group)
    n = bits.numel()
    planes = [unpack_bits(b.to(torch.uint8), n) for b in bufs]
    return majority_vote(planes, tie=tie).view(shape)


def update_fn_distributed(p, grad, exp_avg, lr, wd, beta1, beta2, group=None, wire_dtype=torch.uint8,
                          tie: int = TIE_NEGATIVE) -> None:
    """Per-tensor distributed majority-vote step (ref :61-96 semantics)."""
    p.mul_(1 - lr * wd)
    vote = _gather_vote(sign_bits(grad, exp_avg, beta1), p.shape, group, wire_dtype, tie)
    p.add_(vote.to(torch.int8) * 2 - 1, alpha=-lr)
    momentum_update_(grad, exp_avg, beta2)


def update_fn_distributed_stoc(p, grad, exp_avg, lr, wd, beta1, beta2, max_grad_norm, group=None,
                               wire_dtype=torch.uint8, generator=None, tie: int = TIE_NEGATIVE) -> None:
    """Stochastic-binarization variant (ref :98-136 semantics, D2-D4 fixed)."""
    p.mul_(1 - lr * wd)
    bits = stochastic_bits(grad, exp_avg, beta1, max_grad_norm, generator)
    vote = _gather_vote(bits, p.shape, group, wire_dtype, tie)
    p.add_(vote.to(torch.int8) * 2 - 1, alpha=-lr)
    momentum_update_(grad, exp_avg, beta2)
