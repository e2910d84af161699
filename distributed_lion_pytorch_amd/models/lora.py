"""Native LoRA adapters (peft is not available in this environment).

Covers what the reference uses from peft (/root/reference/sft_llama2.py:44-51,
188-199; dpo_llama2.py:192-207): ``LoraConfig(r, lora_alpha, lora_dropout,
target_modules, bias="none", task_type="CAUSAL_LM")``, wrapping the base model
(base weights frozen, adapters trainable), ``print_trainable_parameters``,
adapter save/load in peft's file layout (``adapter_config.json`` +
``adapter_model.safetensors`` with ``base_model.model.<path>.lora_A.weight``
keys) and ``merge_and_unload``.

Fixes reference defect D12: the optimizer must be built over the trainable
(adapter) parameters *after* injection -- :func:`trainable_parameters`.
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import asdict, dataclass, field
from typing import List, Optional

import torch
import torch.nn as nn

from ..ops import fused
from ..ops.linear import linear_nk
from .quant import Linear4bit


@dataclass
class LoraConfig:
    r: int = 8
    lora_alpha: int = 16
    lora_dropout: float = 0.05
    target_modules: List[str] = field(default_factory=lambda: ["q_proj", "v_proj"])
    bias: str = "none"
    task_type: str = "CAUSAL_LM"
    modules_to_save: Optional[List[str]] = None

    def to_dict(self) -> dict:
        d = asdict(self)
        d["peft_type"] = "LORA"
        return d


class LoraLinear(nn.Module):
    """y = x W^T (+b) + dropout(x) A^T B^T * (alpha / r); W frozen, B zero-init."""

    def __init__(self, base: nn.Module, r: int, alpha: int, dropout: float):
        super().__init__()
        self.base_layer = base
        self.r = r
        self.scaling = alpha / r
        if isinstance(base, Linear4bit):  # QLoRA: adapters in the compute dtype
            dev, dt = base.qweight.device, base.compute_dtype
        else:
            dev, dt = base.weight.device, base.weight.dtype
        self.lora_A = nn.Linear(base.in_features, r, bias=False, device=dev, dtype=dt)
        self.lora_B = nn.Linear(r, base.out_features, bias=False, device=dev, dtype=dt)
        self.dropout = nn.Dropout(dropout) if dropout > 0 else nn.Identity()
        nn.init.kaiming_uniform_(self.lora_A.weight, a=math.sqrt(5))
        nn.init.zeros_(self.lora_B.weight)
        self.merged = False

    @property
    def weight(self):
        return self.base_layer.weight

    def lora_delta(self, x):
        """The adapter path alone: dropout(x) A^T B^T * (alpha / r)."""
        return self.lora_B(self.lora_A(self.dropout(x))) * self.scaling

    def add_adapter(self, x, y):
        """y + lora_delta(x); on the GPU the fused csrc/lora.hip kernels
        (ops/fused.lora_add), with the dropout mask drawn in-kernel."""
        if self.merged:
            return y
        p = self.dropout.p if isinstance(self.dropout, nn.Dropout) and self.dropout.training else 0.0
        return fused.lora_add(y, x, self.lora_A.weight, self.lora_B.weight, self.scaling, p)

    def forward(self, x):
        if isinstance(self.base_layer, Linear4bit):
            return self.add_adapter(x, self.base_layer(x))
        return self.add_adapter(x, linear_nk(x, self.base_layer.weight, self.base_layer.bias))

    @torch.no_grad()
    def merge(self):
        if not self.merged:
            delta = (self.lora_B.weight.float() @ self.lora_A.weight.float()) * self.scaling
            if isinstance(self.base_layer, Linear4bit):  # peft: dequantize, add, requantize
                self.base_layer.requantize_(self.base_layer.dequantize(torch.float32) + delta)
            else:
                self.base_layer.weight.add_(delta.to(self.base_layer.weight.dtype))
            self.merged = True


def _match(name: str, targets) -> bool:
    leaf = name.split(".")[-1]
    return any(leaf == t or name.endswith("." + t) for t in targets)


def inject_lora(model: nn.Module, config: LoraConfig) -> nn.Module:
    """Replace target nn.Linear modules with LoraLinear, freeze everything else."""
    for p in model.parameters():
        p.requires_grad_(False)
    replaced = 0
    for name, module in list(model.named_modules()):
        for child_name, child in list(module.named_children()):
            full = f"{name}.{child_name}" if name else child_name
            if isinstance(child, (nn.Linear, Linear4bit)) and _match(full, config.target_modules):
                setattr(module, child_name, LoraLinear(child, config.r, config.lora_alpha, config.lora_dropout))
                replaced += 1
    if replaced == 0:
        raise ValueError(f"LoRA: no module matches target_modules={config.target_modules}")
    if config.bias in ("all", "lora_only"):
        for n, p in model.named_parameters():
            if n.endswith(".bias"):
                p.requires_grad_(True)
    for n, p in model.named_parameters():
        if "lora_A" in n or "lora_B" in n:
            p.requires_grad_(True)
        if config.modules_to_save and any(m in n for m in config.modules_to_save):
            p.requires_grad_(True)
    model.lora_config = config
    return model


def trainable_parameters(model: nn.Module):
    return [p for p in model.parameters() if p.requires_grad]


def print_trainable_parameters(model: nn.Module) -> str:
    """Same report as the reference's helper (sft_llama2.py:78-90)."""
    trainable = sum(p.numel() for p in model.parameters() if p.requires_grad)
    total = sum({p.data_ptr(): p.numel() for p in model.parameters()}.values())
    msg = f"trainable params: {trainable} || all params: {total} || trainable%: {100 * trainable / max(total, 1):.4f}"
    print(msg)
    return msg


def lora_state_dict(model: nn.Module) -> dict:
    out = {}
    for n, p in model.named_parameters():
        if "lora_A" in n or "lora_B" in n:
            out["base_model.model." + n] = p.detach().cpu().contiguous()
    return out


def save_adapter(model: nn.Module, out_dir: str) -> None:
    from safetensors.torch import save_file

    os.makedirs(out_dir, exist_ok=True)
    save_file(lora_state_dict(model), os.path.join(out_dir, "adapter_model.safetensors"))
    cfg = getattr(model, "lora_config", LoraConfig()).to_dict()
    with open(os.path.join(out_dir, "adapter_config.json"), "w") as f:
        json.dump(cfg, f, indent=2)


def load_adapter(model: nn.Module, adapter_dir: str) -> nn.Module:
    from safetensors.torch import load_file

    with open(os.path.join(adapter_dir, "adapter_config.json")) as f:
        cfg = json.load(f)
    cfg = LoraConfig(**{k: v for k, v in cfg.items() if k in LoraConfig.__dataclass_fields__})
    if not any(isinstance(m, LoraLinear) for m in model.modules()):
        inject_lora(model, cfg)
    sd = load_file(os.path.join(adapter_dir, "adapter_model.safetensors"))
    own = dict(model.named_parameters())
    with torch.no_grad():
        for k, v in sd.items():
            n = k[len("base_model.model."):] if k.startswith("base_model.model.") else k
            own[n].copy_(v.to(own[n].dtype))
    return model


def merge_and_unload(model: nn.Module) -> nn.Module:
    """Fold adapters into the base weights and restore plain nn.Linear modules
    (reference: AutoPeftModelForCausalLM(...).merge_and_unload(), sft_llama2.py:195-199)."""
    for name, module in list(model.named_modules()):
        for child_name, child in list(module.named_children()):
            if isinstance(child, LoraLinear):
                child.merge()
                setattr(module, child_name, child.base_layer)
    for p in model.parameters():
        p.requires_grad_(True)
    if hasattr(model, "lora_config"):
        del model.lora_config
    return model
