"""Llama (Llama-2 / Llama-3 family): HF-format checkpoints, native compute path.

The reference fine-tunes ``meta-llama/Llama-2-7b-hf`` (SFT, /root/reference/
sft_llama2.py:22,141-154; DPO, dpo_llama2.py:133-152) through HF/peft/trl.
This is a ``transformers.PreTrainedModel`` over the stock ``LlamaConfig``
with HF parameter names (``model.layers.{i}.self_attn.q_proj.weight`` ...),
so HF Llama checkpoints load and our checkpoints load into HF, but the
compute path is ours: RMSNorm, rotary embeddings (rotate-half convention),
grouped-query causal attention on the gfx950 flash kernel, SwiGLU MLP, split-K
weight gradients, fused LM-head cross-entropy.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F
from transformers import LlamaConfig, MistralConfig, PreTrainedModel, Qwen2Config
from transformers.modeling_outputs import CausalLMOutputWithPast

from ..ops import fused
from ..ops.linear import linear_multi_nk, linear_nk, no_wgrad_deferral_this_window

LLAMA_SIZES = {
    "llama-2-7b": dict(hidden_size=4096, intermediate_size=11008, num_hidden_layers=32, num_attention_heads=32,
                       num_key_value_heads=32, vocab_size=32000, rope_theta=10000.0, max_position_embeddings=4096,
                       rms_norm_eps=1e-5),
    "llama-2-13b": dict(hidden_size=5120, intermediate_size=13824, num_hidden_layers=40, num_attention_heads=40,
                        num_key_value_heads=40, vocab_size=32000, rope_theta=10000.0, max_position_embeddings=4096,
                        rms_norm_eps=1e-5),
    "llama-3-8b": dict(hidden_size=4096, intermediate_size=14336, num_hidden_layers=32, num_attention_heads=32,
                       num_key_value_heads=8, vocab_size=128256, rope_theta=500000.0, max_position_embeddings=8192,
                       rms_norm_eps=1e-5),
    "llama-tiny": dict(hidden_size=128, intermediate_size=352, num_hidden_layers=2, num_attention_heads=2,
                       num_key_value_heads=1, vocab_size=512, rope_theta=10000.0, max_position_embeddings=512,
                       rms_norm_eps=1e-5),
    # Llama-architecture families (models below): Mistral-7B v0.1 and Qwen2 sizes
    "mistral-7b": dict(model_type="mistral", hidden_size=4096, intermediate_size=14336, num_hidden_layers=32,
                       num_attention_heads=32, num_key_value_heads=8, vocab_size=32000, rope_theta=10000.0,
                       max_position_embeddings=32768, sliding_window=4096, rms_norm_eps=1e-5),
    "qwen2-0.5b": dict(model_type="qwen2", hidden_size=896, intermediate_size=4864, num_hidden_layers=24,
                       num_attention_heads=14, num_key_value_heads=2, vocab_size=151936, rope_theta=1000000.0,
                       max_position_embeddings=32768, rms_norm_eps=1e-6, tie_word_embeddings=True),
    "qwen2-7b": dict(model_type="qwen2", hidden_size=3584, intermediate_size=18944, num_hidden_layers=28,
                     num_attention_heads=28, num_key_value_heads=4, vocab_size=152064, rope_theta=1000000.0,
                     max_position_embeddings=32768, rms_norm_eps=1e-6),
}
_ALIASES = {"Llama-2-7b-hf": "llama-2-7b", "Llama-2-7b": "llama-2-7b", "Meta-Llama-3-8B": "llama-3-8b",
            "Llama-3-8B": "llama-3-8b", "Llama-2-13b-hf": "llama-2-13b", "Mistral-7B-v0.1": "mistral-7b",
            "Qwen2-0.5B": "qwen2-0.5b", "Qwen2-7B": "qwen2-7b"}


def llama_config(name: str = "llama-2-7b", **overrides) -> LlamaConfig:
    key = name.rstrip("/").split("/")[-1]
    key = _ALIASES.get(key, key).lower()
    if key not in LLAMA_SIZES:
        raise KeyError(f"unknown Llama size {name!r}; known: {sorted(LLAMA_SIZES)}")
    kw = dict(LLAMA_SIZES[key])
    kw.update(overrides)
    kw.setdefault("tie_word_embeddings", False)
    cls = {"mistral": MistralConfig, "qwen2": Qwen2Config}.get(kw.pop("model_type", "llama"), LlamaConfig)
    return cls(**kw)


class RMSNorm(nn.Module):
    def __init__(self, dim: int, eps: float):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(dim))
        self.eps = eps

    def forward(self, x):
        return fused.rms_norm(x, self.weight, self.eps)


def _rope_theta(cfg) -> float:
    rp = getattr(cfg, "rope_parameters", None)
    if isinstance(rp, dict) and "rope_theta" in rp:
        return float(rp["rope_theta"])
    return float(getattr(cfg, "rope_theta", 10000.0) or 10000.0)


class Rotary(nn.Module):
    """cos/sin tables computed once per (T, device, dtype) -- no per-step trig.

    The inverse frequencies are NOT a module buffer: ``model.to(bfloat16)``
    would round them to bf16 (0.4 % relative), and at position ~1000 that is
    an angle error of several radians -- the bf16 training path had
    effectively scrambled positions for the high-frequency pairs (caught by
    tests/test_parity_full_gpu.py against HF fp32).  They are computed in fp32
    exactly as HF's LlamaRotaryEmbedding does, at table-build time."""

    def __init__(self, head_dim: int, theta: float):
        super().__init__()
        self.head_dim, self.theta = int(head_dim), float(theta)
        self._cache = {}

    @property
    def inv_freq(self) -> torch.Tensor:
        return 1.0 / (self.theta ** (torch.arange(0, self.head_dim, 2, dtype=torch.int64).float() / self.head_dim))

    def tables(self, T: int, device, dtype):
        key = (T, device, dtype)
        if key not in self._cache:
            t = torch.arange(T, device=device, dtype=torch.float32)
            f = torch.outer(t, self.inv_freq.to(device))
            emb = torch.cat([f, f], dim=-1)
            self._cache = {key: (emb.cos().to(dtype), emb.sin().to(dtype))}
        return self._cache[key]


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """x [B, T, H, D]; HF rotate-half convention."""
    return fused.rope(x, cos, sin)


def _attention_biases(cfg) -> tuple:
    """(q/k/v bias, o bias): Llama's ``attention_bias`` covers all four
    projections; Qwen2 always has q/k/v biases and none on o_proj."""
    if getattr(cfg, "model_type", "") == "qwen2":
        return True, False
    b = bool(getattr(cfg, "attention_bias", False))
    return b, b


def _layer_window(cfg, i: int) -> int:
    """Layer i's sliding attention window (0: full causal), as HF builds the
    masks: Mistral applies ``sliding_window`` (4096 in v0.1) to every layer;
    configs with ``layer_types`` (Qwen2 with ``use_sliding_window``: the layers
    from ``max_window_layers`` on) only to the "sliding_attention" ones."""
    w = getattr(cfg, "sliding_window", None)
    if not w:
        return 0
    types = getattr(cfg, "layer_types", None)
    if types is not None:
        return int(w) if types[i] == "sliding_attention" else 0
    if getattr(cfg, "model_type", "") == "qwen2" and not getattr(cfg, "use_sliding_window", False):
        return 0
    return int(w)


class LlamaAttention(nn.Module):
    def __init__(self, cfg: LlamaConfig, layer_idx: int = 0):
        super().__init__()
        self.window = _layer_window(cfg, layer_idx)  # 0: full causal
        self.n_head = cfg.num_attention_heads
        self.n_kv = cfg.num_key_value_heads
        self.head_dim = getattr(cfg, "head_dim", None) or cfg.hidden_size // cfg.num_attention_heads
        qkv_bias, o_bias = _attention_biases(cfg)
        self.q_proj = nn.Linear(cfg.hidden_size, self.n_head * self.head_dim, bias=qkv_bias)
        self.k_proj = nn.Linear(cfg.hidden_size, self.n_kv * self.head_dim, bias=qkv_bias)
        self.v_proj = nn.Linear(cfg.hidden_size, self.n_kv * self.head_dim, bias=qkv_bias)
        self.o_proj = nn.Linear(self.n_head * self.head_dim, cfg.hidden_size, bias=o_bias)
        self.attn_dropout = float(getattr(cfg, "attention_dropout", 0.0) or 0.0)

    def forward(self, x, cos, sin):
        B, T, _ = x.shape
        q, k, v = _proj(x, (self.q_proj, self.k_proj, self.v_proj))
        q = q.view(B, T, self.n_head, self.head_dim)
        k = k.view(B, T, self.n_kv, self.head_dim)
        v = v.view(B, T, self.n_kv, self.head_dim)
        y = fused.rope_attention(q, k, v, cos, sin, self.attn_dropout if self.training else 0.0, self.window)
        return _lin(self.o_proj, y)


def _lin(layer: nn.Module, x):
    """nn.Linear (possibly LoRA-wrapped) through the split-K wgrad path."""
    if type(layer) is nn.Linear:
        return linear_nk(x, layer.weight, layer.bias)
    return layer(x)


def _proj(x, layers):
    """Projections sharing the input x (q/k/v, gate/up) as ONE GEMM on the
    concatenated weights (ops/linear.py linear_multi_nk); LoRA-wrapped layers
    contribute their frozen base weight to the fused GEMM and add their
    adapter path to their own output.  Falls back to one GEMM per layer off the
    GPU or for unknown wrappers; biases (Qwen2 q/k/v) are added to the fused
    GEMM's outputs."""
    from .lora import LoraLinear
    from .quant import Linear4bit, linear4bit_multi

    bases, q4, biases = [], [], []
    for layer in layers:
        base = layer.base_layer if isinstance(layer, LoraLinear) else layer
        biases.append(getattr(base, "bias", None))
        if type(base) is nn.Linear:
            bases.append(base.weight)
        elif isinstance(base, Linear4bit):  # QLoRA base: one expansion + one GEMM (models/quant.py)
            q4.append(base)
        else:
            return tuple(_lin(layer, x) for layer in layers)
    if q4:
        if bases or any(b is not None for b in biases):
            return tuple(_lin(layer, x) for layer in layers)
        outs = linear4bit_multi(x, q4)
    elif not x.is_cuda or len({w.dtype for w in bases}) != 1:
        return tuple(_lin(layer, x) for layer in layers)
    else:
        outs = linear_multi_nk(x, bases)
        # Qwen2's q/k/v biases: one small add per output keeps the single fused GEMM
        # (its gradient passes the output gradient through unchanged)
        outs = tuple(o if b is None else o + b.to(o.dtype) for o, b in zip(outs, biases))
    return tuple(layer.add_adapter(x, o) if isinstance(layer, LoraLinear) else o for layer, o in zip(layers, outs))


class LlamaMLP(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.gate_proj = nn.Linear(cfg.hidden_size, cfg.intermediate_size, bias=False)
        self.up_proj = nn.Linear(cfg.hidden_size, cfg.intermediate_size, bias=False)
        self.down_proj = nn.Linear(cfg.intermediate_size, cfg.hidden_size, bias=False)

    def forward(self, x):
        g, u = _proj(x, (self.gate_proj, self.up_proj))
        return _lin(self.down_proj, fused.swiglu(g, u))


class LlamaDecoderLayer(nn.Module):
    def __init__(self, cfg: LlamaConfig, layer_idx: int = 0):
        super().__init__()
        self.self_attn = LlamaAttention(cfg, layer_idx)
        self.mlp = LlamaMLP(cfg)
        self.input_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.post_attention_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)

    def forward(self, x, cos, sin):
        x = x + self.self_attn(self.input_layernorm(x), cos, sin)
        return x + self.mlp(self.post_attention_layernorm(x))


class LlamaModel(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.embed_tokens = nn.Embedding(cfg.vocab_size, cfg.hidden_size)
        self.layers = nn.ModuleList([LlamaDecoderLayer(cfg, i) for i in range(cfg.num_hidden_layers)])
        self.norm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        head_dim = getattr(cfg, "head_dim", None) or cfg.hidden_size // cfg.num_attention_heads
        self.rotary = Rotary(head_dim, _rope_theta(cfg))
        self.gradient_checkpointing = False

    def forward(self, input_ids):
        T = input_ids.shape[1]
        x = self.embed_tokens(input_ids)
        cos, sin = self.rotary.tables(T, x.device, x.dtype)
        if self.gradient_checkpointing and self.training:
            no_wgrad_deferral_this_window()  # keep checkpointing's memory saving (ops/linear.py)
            for layer in self.layers:
                x = torch.utils.checkpoint.checkpoint(layer, x, cos, sin, use_reentrant=False)
            return self.norm(x)
        # fused path: each "residual add + next RMSNorm" is one kernel
        first = self.layers[0].input_layernorm
        h = fused.norm(x, first.weight, None, first.eps, rms=True)
        for i, layer in enumerate(self.layers):
            pn = layer.post_attention_layernorm
            x, h = fused.dropout_add_norm(layer.self_attn(h, cos, sin), x, pn.weight, None, pn.eps, 0.0, rms=True)
            nxt = self.layers[i + 1].input_layernorm if i + 1 < len(self.layers) else self.norm
            x, h = fused.dropout_add_norm(layer.mlp(h), x, nxt.weight, None, nxt.eps, 0.0, rms=True)
        return h


class LlamaForCausalLM(PreTrainedModel):
    config_class = LlamaConfig
    base_model_prefix = "model"
    _tied_weights_keys = {"lm_head.weight": "model.embed_tokens.weight"}
    supports_gradient_checkpointing = True
    _no_split_modules = ["LlamaDecoderLayer"]

    def __init__(self, config: LlamaConfig):
        super().__init__(config)
        self.model = LlamaModel(config)
        self.lm_head = nn.Linear(config.hidden_size, config.vocab_size, bias=False)
        self.post_init()
        self.reset_parameters()

    def _init_weights(self, m):
        std = self.config.initializer_range
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, mean=0.0, std=std)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, mean=0.0, std=std)
        elif isinstance(m, RMSNorm):
            nn.init.ones_(m.weight)

    @torch.no_grad()
    def reset_parameters(self):
        self.apply(self._init_weights)
        self.tie_weights()

    def tie_weights(self, *args, **kwargs):
        if getattr(self.config, "tie_word_embeddings", False):
            self.lm_head.weight = self.model.embed_tokens.weight

    def get_input_embeddings(self):
        return self.model.embed_tokens

    def set_input_embeddings(self, emb):
        self.model.embed_tokens = emb

    def get_output_embeddings(self):
        return self.lm_head

    def gradient_checkpointing_enable(self, gradient_checkpointing_kwargs=None):
        self.model.gradient_checkpointing = True

    def gradient_checkpointing_disable(self):
        self.model.gradient_checkpointing = False

    def forward(self, input_ids=None, labels=None, attention_mask=None, num_items_in_batch=None,
                return_dict: Optional[bool] = None, **kwargs):
        h = self.model(input_ids)
        loss = logits = None
        if labels is not None:
            loss = fused.causal_lm_loss(h, self.lm_head.weight, labels, normalizer=num_items_in_batch)
            if not self.training:
                logits = F.linear(h, self.lm_head.weight)
        else:
            logits = F.linear(h, self.lm_head.weight)
        return CausalLMOutputWithPast(loss=loss, logits=logits)

    def sequence_logps(self, input_ids: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        """Sum of log p(label_t | <t) per sequence (DPO); labels -100 ignored."""
        return sequence_logps(self, input_ids, labels)

    def flops_per_token(self, seq_len: int) -> float:
        c = self.config
        n = self.num_parameters() - (0 if c.tie_word_embeddings else 0)
        return 6 * n + 12 * c.num_hidden_layers * c.hidden_size * seq_len


class MistralForCausalLM(LlamaForCausalLM):
    """Mistral: the Llama architecture (GQA, RoPE, SwiGLU, RMSNorm) with HF's
    Mistral parameter names (identical to Llama's) and sliding-window
    attention (4096 in v0.1): the flash kernels skip the key tiles outside each
    query tile's window and mask the boundary ones (csrc/attention.hip)."""

    config_class = MistralConfig


class Qwen2ForCausalLM(LlamaForCausalLM):
    """Qwen2: the Llama architecture with q/k/v projection biases (added to the
    fused q/k/v GEMM's outputs), tied input / output embeddings for the small
    sizes, and (``use_sliding_window``) sliding-window layers from
    ``max_window_layers`` on; HF's Qwen2 parameter names."""

    config_class = Qwen2Config


def sequence_logps(model, input_ids: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """Per-sequence summed token log-probabilities under ``model`` (any of our
    causal LMs): used by the DPO loss (policy and frozen reference)."""
    base = model.model if hasattr(model, "model") and isinstance(model.model, LlamaModel) else model.transformer
    h = base(input_ids)
    # fused LM head + log-softmax gather (no fp32 [B, T, V] logits), labels shifted in place of h
    return fused.token_logps(h, model.lm_head.weight, fused.shift_labels(labels)).sum(-1)
