"""4-bit blockwise quantization of frozen weights (NF4 / FP4), the engine's
replacement for the bitsandbytes 4-bit base models of the reference
(/root/reference/sft_llama2.py:141-149 ``BitsAndBytesConfig(load_in_4bit=True,
bnb_4bit_quant_type="nf4", bnb_4bit_compute_dtype=torch.bfloat16)``;
dpo_llama2.py:133-152 ``load_in_4bit=True`` policy and reference models).

Format (csrc/quant.hip): the weight flattened row-major in 64-element blocks;
per block an fp32 ``absmax`` and 64 4-bit indices into a 16-entry codebook,
two per byte, first element in the high nibble.  ``w ~= code[idx] * absmax``.

On the GPU both directions are gfx950 kernels (``dlion::quant4`` /
``dlion::dequant4_``); off the GPU the same math runs in PyTorch
(:func:`quantize_4bit_ref` / :func:`dequantize_4bit_ref` are also the oracle
of the GPU tests: identical indices and bit-identical dequantized values).
"""
from __future__ import annotations

import torch

from . import hip

BLOCK = 64

# NormalFloat4: quantiles of N(0, 1) normalised to [-1, 1] with an exact zero
# (QLoRA, Dettmers et al. 2023) -- the table bitsandbytes ships.
NF4_CODE = (
    -1.0, -0.6961928009986877, -0.5250730514526367, -0.39491748809814453,
    -0.28444138169288635, -0.18477343022823334, -0.09105003625154495, 0.0,
    0.07958029955625534, 0.16093020141124725, 0.24611230194568634, 0.33791524171829224,
    0.44070982933044434, 0.5626170039176941, 0.7229568362236023, 1.0,
)
# FP4 (e2m1, sign-magnitude index order), normalised to max 1 -- bitsandbytes' fp4 table.
FP4_CODE = (
    0.0, 0.0052083333, 0.6666666667, 1.0, 0.3333333333, 0.5, 0.1666666667, 0.25,
    -0.0, -0.0052083333, -0.6666666667, -1.0, -0.3333333333, -0.5, -0.1666666667, -0.25,
)
CODES = {"nf4": NF4_CODE, "fp4": FP4_CODE}


def code_tensor(quant_type: str, device=None) -> torch.Tensor:
    if quant_type not in CODES:
        raise ValueError(f"unknown 4-bit quant_type {quant_type!r}; known: {sorted(CODES)}")
    return torch.tensor(CODES[quant_type], dtype=torch.float32, device=device)


def quantize_4bit_ref(w: torch.Tensor, code: torch.Tensor):
    """PyTorch oracle: (q uint8 [n/2], absmax fp32 [n/64])."""
    blocks = w.detach().reshape(-1, BLOCK).float()
    absmax = blocks.abs().amax(dim=1)
    safe = torch.where(absmax > 0, absmax, torch.ones_like(absmax))
    x = torch.where(absmax[:, None] > 0, blocks / safe[:, None], torch.zeros_like(blocks))
    idx = (x.unsqueeze(-1) - code.to(x.device)).abs().argmin(dim=-1).to(torch.uint8)  # first minimum on ties
    idx = idx.reshape(-1, 2)
    q = (idx[:, 0] << 4) | idx[:, 1]
    return q.contiguous(), absmax.contiguous()


def dequantize_4bit_ref(q: torch.Tensor, absmax: torch.Tensor, code: torch.Tensor, dtype=torch.bfloat16):
    """PyTorch oracle: flat [n] tensor of ``dtype``."""
    hi = (q >> 4).long()
    lo = (q & 15).long()
    idx = torch.stack([hi, lo], dim=1).reshape(-1, BLOCK)
    vals = code.to(q.device)[idx] * absmax[:, None]
    return vals.reshape(-1).to(dtype)


def _check_shape(n: int) -> None:
    if n % BLOCK:
        raise ValueError(f"4-bit quantization needs numel % {BLOCK} == 0, got {n}")


def quantize_4bit(w: torch.Tensor, code: torch.Tensor):
    """(q, absmax) of ``w`` (flattened row-major); HIP kernel on the GPU."""
    _check_shape(w.numel())
    if w.is_cuda:
        return hip.ops().quant4(w.detach().contiguous(), code.to(w.device))
    return quantize_4bit_ref(w, code)


def dequantize_4bit(q: torch.Tensor, absmax: torch.Tensor, code: torch.Tensor, shape, dtype=torch.bfloat16,
                    out: torch.Tensor | None = None) -> torch.Tensor:
    """The compute-dtype weight of ``shape``; written into ``out`` (a
    contiguous tensor, e.g. a row block of a concatenated weight) if given."""
    n = 2 * q.numel()
    if out is not None and not out.is_contiguous():
        raise ValueError("dequantize_4bit: out must be contiguous (it is written linearly)")
    if q.is_cuda:
        if out is None:
            out = torch.empty(shape, dtype=dtype, device=q.device)
        hip.ops().dequant4_(q, absmax, code, out)
        return out
    w = dequantize_4bit_ref(q, absmax, code, dtype if out is None else out.dtype).view(shape)
    if out is not None:
        assert out.numel() == n
        out.copy_(w)
        return out
    return w
