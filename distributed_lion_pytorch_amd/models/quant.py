"""4-bit frozen base layers: the engine's ``load_in_4bit`` (bitsandbytes'
``Linear4bit`` as used by the reference's SFT / DPO scripts,
/root/reference/sft_llama2.py:141-154, dpo_llama2.py:133-152).

:class:`Linear4bit` keeps a frozen ``nn.Linear`` weight as 4-bit codebook
indices + per-64-block fp32 absmax (ops/quant.py, csrc/quant.hip) and expands
it to the compute dtype only around its GEMMs (forward, and the input-gradient
GEMM of backward), so a replica holds ~0.56 B/param of base weights instead of
2.  Projections sharing an input (Llama q/k/v, gate/up) are expanded into one
concatenated buffer and run as ONE GEMM each way (:func:`linear4bit_multi`),
the same fusion the bf16 path uses (ops/linear.py ``linear_multi_nk``).  LoRA
adapters wrap these layers unchanged (models/lora.py) -- QLoRA.

:func:`quantize_model` replaces every ``nn.Linear`` except the skipped ones
(``lm_head`` by default, as bitsandbytes / transformers do) in place.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Iterable, Optional, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.linear import _adjacent_views, autocast_inputs, gemm_fwd
from ..ops.quant import BLOCK, code_tensor, dequantize_4bit, quantize_4bit


@dataclass
class QuantConfig:
    """Subset of transformers' ``BitsAndBytesConfig`` the reference uses."""

    load_in_4bit: bool = True
    bnb_4bit_quant_type: str = "nf4"
    bnb_4bit_compute_dtype: Optional[torch.dtype] = None
    bnb_4bit_use_double_quant: bool = False
    llm_int8_skip_modules: Sequence[str] = ("lm_head",)

    def __post_init__(self):
        if self.bnb_4bit_use_double_quant:
            raise NotImplementedError("double quantization of the absmax table is not implemented "
                                      "(the reference does not use it); absmax stays fp32 (0.0625 B/param)")
        if isinstance(self.bnb_4bit_compute_dtype, str):
            self.bnb_4bit_compute_dtype = getattr(torch, self.bnb_4bit_compute_dtype)


BitsAndBytesConfig = QuantConfig  # reference-facing name


class Linear4bit(nn.Module):
    """Frozen y = x W^T (+ b) with W stored 4-bit (``qweight``, ``absmax``,
    ``quant_map`` buffers; HF-style state_dict round trip)."""

    def __init__(self, in_features: int, out_features: int, bias: bool = False, quant_type: str = "nf4",
                 compute_dtype: Optional[torch.dtype] = torch.bfloat16, device=None):
        super().__init__()
        n = in_features * out_features
        if n % BLOCK:
            raise ValueError(f"Linear4bit needs in*out % {BLOCK} == 0, got {in_features}x{out_features}")
        self.in_features = in_features
        self.out_features = out_features
        self.quant_type = quant_type
        self.compute_dtype = compute_dtype or torch.bfloat16
        self.register_buffer("qweight", torch.zeros(n // 2, dtype=torch.uint8, device=device))
        self.register_buffer("absmax", torch.zeros(n // BLOCK, dtype=torch.float32, device=device))
        self.register_buffer("quant_map", code_tensor(quant_type, device))
        self.bias = nn.Parameter(torch.zeros(out_features, dtype=self.compute_dtype, device=device),
                                 requires_grad=False) if bias else None

    @classmethod
    @torch.no_grad()
    def from_linear(cls, lin: nn.Linear, quant_type: str = "nf4", compute_dtype=None) -> "Linear4bit":
        w = lin.weight
        cd = compute_dtype or w.dtype
        m = cls(lin.in_features, lin.out_features, lin.bias is not None, quant_type, cd, device="meta")
        m.quant_map = code_tensor(quant_type, w.device)
        q, absmax = quantize_4bit(w, m.quant_map)
        m.qweight, m.absmax = q, absmax
        if lin.bias is not None:
            m.bias = nn.Parameter(lin.bias.detach().to(cd), requires_grad=False)
        return m

    def _apply(self, fn, recurse=True):
        # model.to(dtype) / .half() must move the fp32 absmax / codebook, never round them
        keep = {k: self._buffers[k] for k in ("absmax", "quant_map")}
        super()._apply(fn, recurse)
        for k, t in keep.items():
            moved = fn(t)
            self._buffers[k] = moved if moved.dtype == torch.float32 else t.to(moved.device)
        return self

    @torch.no_grad()
    def requantize_(self, w: torch.Tensor) -> None:
        """Store ``w`` [out, in] (e.g. after a LoRA merge)."""
        q, absmax = quantize_4bit(w.to(self.qweight.device), self.quant_map)
        self.qweight.copy_(q)
        self.absmax.copy_(absmax)

    def dequantize(self, dtype=None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        return dequantize_4bit(self.qweight, self.absmax, self.quant_map, (self.out_features, self.in_features),
                               dtype or self.compute_dtype, out=out)

    @property
    def weight(self) -> torch.Tensor:
        """The compute-dtype weight (materialised on each access)."""
        return self.dequantize()

    def forward(self, x):
        return linear4bit_multi(x, (self,), self.bias)[0]

    def extra_repr(self) -> str:
        return (f"in_features={self.in_features}, out_features={self.out_features}, bias={self.bias is not None}, "
                f"quant_type={self.quant_type}, compute_dtype={self.compute_dtype}")


def _dequant_cat(layers, dtype, device) -> torch.Tensor:
    K = layers[0].in_features
    W = torch.empty(sum(l.out_features for l in layers), K, dtype=dtype, device=device)
    off = 0
    for l in layers:
        l.dequantize(dtype, out=W[off:off + l.out_features])
        off += l.out_features
    return W


def _transposed_ok(layers, dy) -> bool:
    return (dy.is_cuda and dy.dtype in (torch.bfloat16, torch.float16)
            and all(l.in_features % 128 == 0 and l.out_features % 64 == 0 for l in layers))


def _dequant_cat_t(layers, dtype, device) -> torch.Tensor:
    """[W1; W2; ...]^T = [W1^T | W2^T | ...] ([K, sum N]) expanded from 4 bits."""
    from ..ops import hip

    K = layers[0].in_features
    Wt = torch.empty(K, sum(l.out_features for l in layers), dtype=dtype, device=device)
    off = 0
    for l in layers:
        hip.ops().dequant4_t_(l.qweight, l.absmax, l.quant_map, Wt[:, off:off + l.out_features])
        off += l.out_features
    return Wt


class _Linear4bitMulti(torch.autograd.Function):
    """[y1 | y2 | ...] = x @ [W1; W2; ...]^T (+ b for one layer) with the 4-bit
    weights expanded into one transient buffer; backward re-expands it for
    dx = dy @ W (the frozen weights get no gradient; nothing but the layer
    handles is saved, so activation checkpointing recomputes nothing extra)."""

    @staticmethod
    def forward(ctx, x2d, bias, *layers):
        W = _dequant_cat(layers, x2d.dtype, x2d.device)
        y = F.linear(x2d, W, bias) if bias is not None or not x2d.is_cuda else gemm_fwd(x2d, W)
        del W
        ctx.layers = layers
        ctx.sizes = [l.out_features for l in layers]
        ctx.has_bias = bias is not None
        return tuple(y.split(ctx.sizes, dim=-1))

    @staticmethod
    def backward(ctx, *grads):
        dt = next(g for g in grads if g is not None)
        grads = [torch.zeros(dt.shape[0], n, dtype=dt.dtype, device=dt.device) if g is None else g
                 for g, n in zip(grads, ctx.sizes)]
        dy = _adjacent_views(grads) if len(grads) > 1 else grads[0]
        if dy is None:
            dy = torch.cat(grads, -1)
        dy = dy.reshape(-1, dy.shape[-1])
        dx = None
        if ctx.needs_input_grad[0]:
            if _transposed_ok(ctx.layers, dy):
                # dX = dY . W as the NT product against W^T, expanded straight into the transposed
                # layout (csrc/quant.hip dequant4_t): no NN GEMM, no transpose pass
                dx = gemm_fwd(dy, _dequant_cat_t(ctx.layers, dy.dtype, dy.device))
            else:
                dx = dy @ _dequant_cat(ctx.layers, dy.dtype, dy.device)
        db = dy.sum(0) if ctx.has_bias and ctx.needs_input_grad[1] else None
        return (dx, db) + (None,) * len(ctx.layers)


def linear4bit_multi(x: torch.Tensor, layers: Sequence[Linear4bit], bias: Optional[torch.Tensor] = None) -> tuple:
    """(x @ W1^T, x @ W2^T, ...) for 4-bit layers sharing the input x, as one
    GEMM on the concatenated expanded weights; ``bias`` only with one layer."""
    assert bias is None or len(layers) == 1
    lead = x.shape[:-1]
    x2d = x.reshape(-1, x.shape[-1])
    if x2d.dtype not in (torch.bfloat16, torch.float16, torch.float32):
        x2d = x2d.to(layers[0].compute_dtype)
    if x.is_cuda:
        x2d, bias = autocast_inputs(x2d, bias)
        with torch.autocast("cuda", enabled=False):
            outs = _Linear4bitMulti.apply(x2d, bias if bias is None else bias.to(x2d.dtype), *layers)
    else:
        outs = _Linear4bitMulti.apply(x2d, bias if bias is None else bias.to(x2d.dtype), *layers)
    return tuple(o.view(lead + (o.shape[-1],)) for o in outs)


def _skipped(name: str, skip: Iterable[str]) -> bool:
    leaf = name.split(".")[-1]
    return any(leaf == s or name == s or name.endswith("." + s) for s in skip)


@torch.no_grad()
def quantize_model(model: nn.Module, config: Optional[QuantConfig] = None, **kw) -> nn.Module:
    """Replace every nn.Linear (except ``llm_int8_skip_modules``) by a frozen
    :class:`Linear4bit`, layer by layer (peak extra memory: one weight)."""
    config = config or QuantConfig(**kw)
    if not config.load_in_4bit:
        return model
    n = 0
    for name, module in list(model.named_modules()):
        for child_name, child in list(module.named_children()):
            full = f"{name}.{child_name}" if name else child_name
            # LoRA adapters stay trainable (quantizing an injected model keeps them as they are)
            if (type(child) is nn.Linear and not _skipped(full, config.llm_int8_skip_modules)
                    and child_name not in ("lora_A", "lora_B")):
                setattr(module, child_name, Linear4bit.from_linear(child, config.bnb_4bit_quant_type,
                                                                   config.bnb_4bit_compute_dtype))
                n += 1
    if n == 0:
        raise ValueError("quantize_model: no nn.Linear to quantize")
    # (not HF's quantization_config / is_loaded_in_4bit: transformers would route those to bitsandbytes)
    model.dlion_quant_config = config
    return model


@torch.no_grad()
def dequantize_model(model: nn.Module) -> nn.Module:
    """Replace every :class:`Linear4bit` by an ``nn.Linear`` of its compute
    dtype (frozen, like the 4-bit layer was); no-op for unquantized models."""
    for name, module in list(model.named_modules()):
        for child_name, child in list(module.named_children()):
            if isinstance(child, Linear4bit):
                lin = nn.Linear(child.in_features, child.out_features, bias=child.bias is not None,
                                device=child.qweight.device, dtype=child.compute_dtype)
                lin.weight.copy_(child.dequantize())
                if child.bias is not None:
                    lin.bias.copy_(child.bias)
                lin.requires_grad_(False)
                setattr(module, child_name, lin)
    if "dlion_quant_config" in model.__dict__:
        del model.dlion_quant_config
    return model


def quantized_bytes(model: nn.Module) -> int:
    """Resident bytes of the 4-bit layers (qweight + absmax + map)."""
    return sum(m.qweight.numel() + m.absmax.numel() * 4 + 64 for m in model.modules() if isinstance(m, Linear4bit))
