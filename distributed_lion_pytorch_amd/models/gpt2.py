"""GPT-2 (causal LM) with HF-compatible parameter names and checkpoint format.

The reference trains ``transformers.GPT2LMHeadModel`` built from the ``gpt2``
config (/root/reference/run_clm.py:397-442; README.md:20-37).  This module is
a native re-implementation of the same architecture -- identical parameter
names/shapes (``transformer.h.{i}.attn.c_attn.weight`` stored [in, out] like
HF ``Conv1D``), identical init, tied ``lm_head`` -- so ``state_dict()`` loads
into HF's class and vice versa, while the compute path is ours:

* projections are single hipBLASLt GEMMs on the [in, out] weights (``addmm``);
* attention, bias+GELU, residual+LayerNorm and the LM-head cross-entropy go
  through :mod:`distributed_lion_pytorch_amd.ops.fused`, which dispatches to
  hand-written gfx950 kernels when the extension is present.
"""
from __future__ import annotations

import math
from dataclasses import asdict, dataclass, field
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import fused
from ..ops.linear import linear_kn


@dataclass
class GPT2Config:
    vocab_size: int = 50257
    n_positions: int = 1024
    n_embd: int = 768
    n_layer: int = 12
    n_head: int = 12
    n_inner: Optional[int] = None
    activation_function: str = "gelu_new"
    resid_pdrop: float = 0.1
    embd_pdrop: float = 0.1
    attn_pdrop: float = 0.1
    layer_norm_epsilon: float = 1e-5
    initializer_range: float = 0.02
    tie_word_embeddings: bool = True
    bos_token_id: int = 50256
    eos_token_id: int = 50256
    extra: dict = field(default_factory=dict)

    model_type = "gpt2"

    @classmethod
    def from_name(cls, name: str) -> "GPT2Config":
        sizes = {
            "gpt2": dict(n_embd=768, n_layer=12, n_head=12),
            "gpt2-medium": dict(n_embd=1024, n_layer=24, n_head=16),
            "gpt2-large": dict(n_embd=1280, n_layer=36, n_head=20),
            "gpt2-xl": dict(n_embd=1600, n_layer=48, n_head=25),
            "gpt2-tiny": dict(n_embd=64, n_layer=2, n_head=4, vocab_size=512, n_positions=128),
        }
        key = name.split("/")[-1]
        if key not in sizes:
            raise KeyError(f"unknown GPT-2 size {name!r}")
        return cls(**sizes[key])

    @classmethod
    def from_dict(cls, d: dict) -> "GPT2Config":
        known = {k: d[k] for k in cls.__dataclass_fields__ if k in d and k != "extra"}
        extra = {k: v for k, v in d.items() if k not in cls.__dataclass_fields__}
        return cls(**known, extra=extra)

    def to_hf_dict(self) -> dict:
        d = asdict(self)
        extra = d.pop("extra")
        d.update(extra)
        d["model_type"] = "gpt2"
        d["architectures"] = ["GPT2LMHeadModel"]
        d["n_ctx"] = self.n_positions
        return d

    @property
    def inner(self) -> int:
        return self.n_inner if self.n_inner is not None else 4 * self.n_embd


class Conv1D(nn.Module):
    """Affine map with HF's [in, out] weight layout: y = x @ W + b (one GEMM)."""

    def __init__(self, nx: int, nf: int):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(nx, nf))
        self.bias = nn.Parameter(torch.zeros(nf))

    def forward(self, x):
        return linear_kn(x, self.weight, self.bias)


class Attention(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.n_head = cfg.n_head
        self.head_dim = cfg.n_embd // cfg.n_head
        self.c_attn = Conv1D(cfg.n_embd, 3 * cfg.n_embd)
        self.c_proj = Conv1D(cfg.n_embd, cfg.n_embd)
        self.attn_pdrop = cfg.attn_pdrop
        self.resid_pdrop = cfg.resid_pdrop

    def forward(self, x):
        B, T, C = x.shape
        qkv = self.c_attn(x).view(B, T, 3, self.n_head, self.head_dim)
        y = fused.causal_attention(qkv, self.attn_pdrop if self.training else 0.0)  # [B, T, C]
        return self.c_proj(y)


class MLP(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.c_fc = Conv1D(cfg.n_embd, cfg.inner)
        self.c_proj = Conv1D(cfg.inner, cfg.n_embd)
        if cfg.activation_function not in ("gelu_new", "gelu_pytorch_tanh", "gelu"):
            raise ValueError(f"unsupported activation {cfg.activation_function}")
        self.exact_gelu = cfg.activation_function == "gelu"

    def forward(self, x):
        shp = x.shape[:-1]
        h = fused.linear_gelu(x.reshape(-1, x.shape[-1]), self.c_fc.weight, self.c_fc.bias, exact=self.exact_gelu)
        return self.c_proj(h.view(*shp, -1))


class Block(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.ln_1 = nn.LayerNorm(cfg.n_embd, eps=cfg.layer_norm_epsilon)
        self.attn = Attention(cfg)
        self.ln_2 = nn.LayerNorm(cfg.n_embd, eps=cfg.layer_norm_epsilon)
        self.mlp = MLP(cfg)
        self.resid_pdrop = cfg.resid_pdrop

    def forward(self, x):
        p = self.resid_pdrop if self.training else 0.0
        x = fused.dropout_add(self.attn(fused.layer_norm(x, self.ln_1)), x, p)
        x = fused.dropout_add(self.mlp(fused.layer_norm(x, self.ln_2)), x, p)
        return x


class GPT2Model(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.wte = nn.Embedding(cfg.vocab_size, cfg.n_embd)
        self.wpe = nn.Embedding(cfg.n_positions, cfg.n_embd)
        self.h = nn.ModuleList([Block(cfg) for _ in range(cfg.n_layer)])
        self.ln_f = nn.LayerNorm(cfg.n_embd, eps=cfg.layer_norm_epsilon)
        self.embd_pdrop = cfg.embd_pdrop
        self.gradient_checkpointing = False

    def forward(self, input_ids):
        B, T = input_ids.shape
        pos = torch.arange(T, device=input_ids.device)
        x = self.wte(input_ids) + self.wpe(pos)[None]
        if self.training and self.embd_pdrop > 0:
            x = F.dropout(x, self.embd_pdrop, True)
        for blk in self.h:
            if self.gradient_checkpointing and self.training:
                x = torch.utils.checkpoint.checkpoint(blk, x, use_reentrant=False)
            else:
                x = blk(x)
        return fused.layer_norm(x, self.ln_f)


class CausalLMOutput(dict):
    """Minimal ModelOutput look-alike (attribute + key access, tuple index 0 = loss or logits)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __getitem__(self, k):
        if isinstance(k, int):
            vals = [v for v in self.values() if v is not None]
            return vals[k]
        return super().__getitem__(k)

    def to_tuple(self):
        return tuple(v for v in self.values() if v is not None)


class GPT2LMHeadModel(nn.Module):
    config_class = GPT2Config
    base_model_prefix = "transformer"
    _tied_weights_keys = ["lm_head.weight"]

    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.config = cfg
        self.transformer = GPT2Model(cfg)
        self.lm_head = nn.Linear(cfg.n_embd, cfg.vocab_size, bias=False)
        if cfg.tie_word_embeddings:
            self.lm_head.weight = self.transformer.wte.weight
        self.apply(self._init_weights)
        # GPT-2 "special scaled init" of the residual projections (as HF)
        for name, p in self.named_parameters():
            if name.endswith("c_proj.weight"):
                nn.init.normal_(p, mean=0.0, std=cfg.initializer_range / math.sqrt(2 * cfg.n_layer))

    def _init_weights(self, m):
        std = self.config.initializer_range
        if isinstance(m, (nn.Linear, Conv1D)):
            nn.init.normal_(m.weight, mean=0.0, std=std)
            if getattr(m, "bias", None) is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, mean=0.0, std=std)
        elif isinstance(m, nn.LayerNorm):
            nn.init.ones_(m.weight)
            nn.init.zeros_(m.bias)

    # HF-ish conveniences used by trainers / entrypoints
    def get_input_embeddings(self):
        return self.transformer.wte

    def gradient_checkpointing_enable(self, **_):
        self.transformer.gradient_checkpointing = True

    def num_parameters(self) -> int:
        return sum({p.data_ptr(): p.numel() for p in self.parameters()}.values())

    def forward(self, input_ids, labels=None, attention_mask=None, return_logits: bool = True, **_):
        h = self.transformer(input_ids)
        loss = None
        logits = None
        if labels is not None:
            # shift inside the fused LM-head + cross-entropy (HF semantics:
            # position t predicts label t+1, ignore_index -100)
            loss = fused.lm_head_cross_entropy(h[:, :-1], self.lm_head.weight, labels[:, 1:])
            if return_logits and not self.training:
                logits = F.linear(h, self.lm_head.weight)
        else:
            logits = F.linear(h, self.lm_head.weight)
        return CausalLMOutput(loss=loss, logits=logits)

    def flops_per_token(self, seq_len: int) -> float:
        """Training FLOPs per token (6N + attention), for MFU reporting."""
        c = self.config
        n = self.num_parameters() - c.n_positions * c.n_embd
        attn = 12 * c.n_layer * c.n_embd * seq_len  # 6 * 2 * L * T * d (QK^T and PV, fwd+bwd)
        return 6 * n + attn
