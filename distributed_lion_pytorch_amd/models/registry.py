"""Model/config registry: named sizes without the hub, local HF dirs, native vs HF class."""
from __future__ import annotations

import os
from typing import Optional

import torch
from transformers import AutoConfig, PretrainedConfig

from .gpt2 import GPT2_SIZES, GPT2LMHeadModel, gpt2_config
from .llama import (LLAMA_SIZES, LlamaForCausalLM, MistralForCausalLM, Qwen2ForCausalLM, llama_config,
                    _ALIASES as _LLAMA_ALIASES)

NATIVE = {"gpt2": GPT2LMHeadModel, "llama": LlamaForCausalLM, "mistral": MistralForCausalLM,
          "qwen2": Qwen2ForCausalLM}


def load_config(name_or_path: str, overrides: Optional[str] = None) -> PretrainedConfig:
    if os.path.isdir(name_or_path):
        cfg = AutoConfig.from_pretrained(name_or_path)
    else:
        key = name_or_path.rstrip("/").split("/")[-1]
        if key in GPT2_SIZES or key == "gpt2":
            cfg = gpt2_config(key)
        elif key.lower() in LLAMA_SIZES or key in _LLAMA_ALIASES or key == "llama":  # incl. Mistral / Qwen2
            cfg = llama_config("llama-2-7b" if key == "llama" else key)
        else:
            raise KeyError(f"unknown model {name_or_path!r} (no hub access): use a local directory or one of "
                           f"{sorted(GPT2_SIZES) + sorted(LLAMA_SIZES)}")
    if overrides:
        cfg.update_from_string(overrides)
        types = getattr(cfg, "layer_types", None)
        if types is not None and len(types) != cfg.num_hidden_layers:
            # per-layer attention types (Qwen2) are derived at construction: rebuild them for the
            # overridden depth instead of saving a config HF's validator rejects
            d = cfg.to_dict()
            d.pop("layer_types")
            cfg = type(cfg)(**d)
    return cfg


def _dtype(name):
    if name in (None, "auto"):
        return None
    return getattr(torch, name) if isinstance(name, str) else name


def build_model(config: PretrainedConfig, model_name_or_path: Optional[str] = None, native: bool = True,
                torch_dtype=None):
    dtype = _dtype(torch_dtype)
    if native and config.model_type in NATIVE:
        cls = NATIVE[config.model_type]
        if model_name_or_path and os.path.isdir(model_name_or_path):
            model = cls.from_pretrained(model_name_or_path, config=config)
        else:
            model = cls(config)
    else:
        from transformers import AutoModelForCausalLM

        if model_name_or_path and os.path.isdir(model_name_or_path):
            model = AutoModelForCausalLM.from_pretrained(model_name_or_path, config=config)
        else:
            model = AutoModelForCausalLM.from_config(config)
    if dtype is not None:
        model = model.to(dtype)
    return model
