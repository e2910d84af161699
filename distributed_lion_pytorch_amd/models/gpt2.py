"""GPT-2 (causal LM): HF-format checkpoints, MI355X-native compute path.

The reference trains ``transformers.GPT2LMHeadModel`` built from the ``gpt2``
config (/root/reference/run_clm.py:397-442; README.md:20-37).  This module
re-implements the architecture as a ``transformers.PreTrainedModel`` over the
stock ``GPT2Config`` -- identical parameter names/shapes
(``transformer.h.{i}.attn.c_attn.weight`` stored [in, out] like HF
``Conv1D``), identical init and tied ``lm_head`` -- so ``save_pretrained`` /
``from_pretrained`` / HF ``Trainer`` checkpoints interoperate with HF's own
class, while every hot op runs through our kernels:

* projections: hipBLASLt GEMMs on the [in, out] weights with split-K weight
  gradients (ops/linear.py);
* attention: gfx950 flash attention on the packed qkv, in-kernel dropout
  (ops/fused.causal_attention -> csrc/attention.hip);
* LM head + loss: fused softmax-cross-entropy kernel, no fp32 logits
  (ops/fused.lm_head_cross_entropy -> csrc/xent_kernels.hip).
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F
from transformers import GPT2Config, PreTrainedModel
from transformers.modeling_outputs import CausalLMOutputWithCrossAttentions

from ..ops import fused
from ..ops.linear import linear_kn, no_wgrad_deferral_this_window

GPT2_SIZES = {
    "gpt2": dict(n_embd=768, n_layer=12, n_head=12),
    "gpt2-medium": dict(n_embd=1024, n_layer=24, n_head=16),
    "gpt2-large": dict(n_embd=1280, n_layer=36, n_head=20),
    "gpt2-xl": dict(n_embd=1600, n_layer=48, n_head=25),
    "gpt2-tiny": dict(n_embd=64, n_layer=2, n_head=4, vocab_size=512, n_positions=256, bos_token_id=511,
                      eos_token_id=511),
}


def gpt2_config(name: str = "gpt2", **overrides) -> GPT2Config:
    """HF GPT2Config for a named size (no hub access needed)."""
    key = name.rstrip("/").split("/")[-1]
    if key not in GPT2_SIZES:
        raise KeyError(f"unknown GPT-2 size {name!r}; known: {sorted(GPT2_SIZES)}")
    kw = dict(GPT2_SIZES[key])
    kw.update(overrides)
    return GPT2Config(**kw)


class Conv1D(nn.Module):
    """Affine map with HF's [in, out] weight layout: y = x @ W + b."""

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

    def forward(self, x, proj_bias: bool = True):
        """proj_bias=False leaves c_proj's bias to the caller's fused
        residual+dropout+LayerNorm kernel (its gradient comes out of it too)."""
        y = fused.qkv_attention(x, self.c_attn.weight, self.c_attn.bias, self.n_head,
                                self.attn_pdrop if self.training else 0.0)  # [B, T, C]
        return self.c_proj(y) if proj_bias else linear_kn(y, self.c_proj.weight, None)


class MLP(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        inner = cfg.n_inner if cfg.n_inner is not None else 4 * cfg.n_embd
        self.c_fc = Conv1D(cfg.n_embd, inner)
        self.c_proj = Conv1D(inner, cfg.n_embd)
        if cfg.activation_function not in ("gelu_new", "gelu_pytorch_tanh", "gelu", "gelu_fast"):
            raise ValueError(f"unsupported activation {cfg.activation_function}")
        self.exact_gelu = cfg.activation_function == "gelu"

    def forward(self, x, proj_bias: bool = True):
        shp = x.shape[:-1]
        x2 = x.reshape(-1, x.shape[-1])
        if torch.is_grad_enabled() and x2.is_cuda:
            # training: the whole MLP is one autograd op with the bias+GELU
            # forward and backward fused into GEMM epilogues (ops/fused._MLP)
            y = fused.mlp_gelu(x2, self.c_fc.weight, self.c_fc.bias, self.c_proj.weight,
                               exact=self.exact_gelu).view(*shp, -1)
            return y + self.c_proj.bias if proj_bias else y
        h = fused.linear_gelu(x2, self.c_fc.weight, self.c_fc.bias, exact=self.exact_gelu)
        h = h.view(*shp, -1)
        return self.c_proj(h) if proj_bias else linear_kn(h, self.c_proj.weight, None)


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
        p = self.embd_pdrop if self.training else 0.0
        x = fused.embed(input_ids, self.wte.weight, self.wpe.weight, p)  # gather + add + dropout, one kernel
        if self.gradient_checkpointing and self.training:
            no_wgrad_deferral_this_window()  # keep checkpointing's memory saving (ops/linear.py)
            for blk in self.h:
                x = torch.utils.checkpoint.checkpoint(blk, x, use_reentrant=False)
            return fused.layer_norm(x, self.ln_f)
        # fused path: every "dropout(branch) + residual add + next LayerNorm"
        # boundary is one kernel (ops/fused.dropout_add_norm -> norm_kernels.hip)
        first = self.h[0].ln_1
        h = fused.norm(x, first.weight, first.bias, first.eps)
        for i, blk in enumerate(self.h):
            p = blk.resid_pdrop if self.training else 0.0
            x, h = fused.dropout_add_norm(blk.attn(h, proj_bias=False), x, blk.ln_2.weight, blk.ln_2.bias,
                                          blk.ln_2.eps, p, bias=blk.attn.c_proj.bias)
            nxt = self.h[i + 1].ln_1 if i + 1 < len(self.h) else self.ln_f
            x, h = fused.dropout_add_norm(blk.mlp(h, proj_bias=False), x, nxt.weight, nxt.bias, nxt.eps, p,
                                          bias=blk.mlp.c_proj.bias)
        return h


class GPT2LMHeadModel(PreTrainedModel):
    config_class = GPT2Config
    base_model_prefix = "transformer"
    _tied_weights_keys = {"lm_head.weight": "transformer.wte.weight"}
    supports_gradient_checkpointing = True
    _no_split_modules = ["Block"]

    def __init__(self, config: GPT2Config):
        super().__init__(config)
        self.transformer = GPT2Model(config)
        self.lm_head = nn.Linear(config.n_embd, config.vocab_size, bias=False)
        self.post_init()
        self.reset_parameters()

    # -- init identical to HF GPT2PreTrainedModel._init_weights + scaled c_proj
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

    @torch.no_grad()
    def reset_parameters(self):
        self.apply(self._init_weights)
        for name, p in self.named_parameters():
            if name.endswith("c_proj.weight"):
                nn.init.normal_(p, mean=0.0, std=self.config.initializer_range / math.sqrt(2 * self.config.n_layer))
        self.tie_weights()

    def tie_weights(self, *args, **kwargs):
        if getattr(self.config, "tie_word_embeddings", True):
            self.lm_head.weight = self.transformer.wte.weight

    def get_input_embeddings(self):
        return self.transformer.wte

    def set_input_embeddings(self, emb):
        self.transformer.wte = emb

    def get_output_embeddings(self):
        return self.lm_head

    def _set_gradient_checkpointing(self, enable: bool = True, gradient_checkpointing_func=None):
        self.transformer.gradient_checkpointing = enable

    def gradient_checkpointing_enable(self, gradient_checkpointing_kwargs=None):
        self.transformer.gradient_checkpointing = True

    def gradient_checkpointing_disable(self):
        self.transformer.gradient_checkpointing = False

    def forward(self, input_ids=None, labels=None, attention_mask=None, num_items_in_batch=None,
                return_dict: Optional[bool] = None, **kwargs):
        h = self.transformer(input_ids)
        loss = None
        logits = None
        if labels is not None:
            # shift inside the fused LM-head + cross-entropy (HF semantics:
            # position t predicts label t+1, ignore_index -100).  With
            # num_items_in_batch the sum is normalised by it (HF GA-aware loss).
            loss = fused.causal_lm_loss(h, self.lm_head.weight, labels, normalizer=num_items_in_batch)
            if not self.training:
                logits = F.linear(h, self.lm_head.weight)
        else:
            logits = F.linear(h, self.lm_head.weight)
        return CausalLMOutputWithCrossAttentions(loss=loss, logits=logits)

    def sequence_logps(self, input_ids: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        """Sum of log p(label_t | <t) per sequence (DPO); labels -100 ignored."""
        h = self.transformer(input_ids)
        return fused.token_logps(h, self.lm_head.weight, fused.shift_labels(labels)).sum(-1)

    def flops_per_token(self, seq_len: int) -> float:
        """Training FLOPs per token (6N + attention), for MFU reporting."""
        c = self.config
        n = self.num_parameters() - c.n_positions * c.n_embd
        return 6 * n + 12 * c.n_layer * c.n_embd * seq_len
