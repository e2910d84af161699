"""Loader for the in-tree gfx950 extension (``_dlion_C.so``).

The extension registers the ``torch.ops.dlion`` namespace (csrc/bindings.cpp).
On a GPU box the HIP path is mandatory: :func:`require` raises if the shared
object is missing or fails to load, instead of silently degrading to the
PyTorch oracle.  Setting ``DLION_ALLOW_TORCH_FALLBACK=1`` opts into the slow
oracle explicitly (used only for debugging).
"""
from __future__ import annotations

import os
import threading
from pathlib import Path

import torch

# DLION_LIB points at an alternative build of the same extension (kernel A/B runs)
LIB_PATH = Path(os.environ.get("DLION_LIB") or Path(__file__).resolve().parent.parent / "_dlion_C.so")

DTYPE_CODE = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}

_lock = threading.Lock()
_state = {"loaded": False, "error": None}


def load() -> bool:
    """Load the extension once; returns True on success."""
    with _lock:
        if _state["loaded"]:
            return True
        if _state["error"] is not None:
            return False
        if not LIB_PATH.exists():
            _state["error"] = f"{LIB_PATH} not built (run: python -m distributed_lion_pytorch_amd._build)"
            return False
        try:
            torch.ops.load_library(str(LIB_PATH))
            _state["loaded"] = True
        except Exception as exc:  # pragma: no cover - depends on the box
            _state["error"] = f"failed to load {LIB_PATH}: {exc}"
        return _state["loaded"]


def load_error() -> str | None:
    return _state["error"]


def gpu_present() -> bool:
    return torch.cuda.is_available()


def available() -> bool:
    """True when the HIP kernels can run (library loaded and a GPU is present)."""
    return gpu_present() and load()


def fallback_allowed() -> bool:
    return os.environ.get("DLION_ALLOW_TORCH_FALLBACK", "0") == "1"


def require() -> None:
    if not gpu_present():
        raise RuntimeError("dlion HIP kernels need a GPU")
    if not load():
        raise RuntimeError(
            "dlion: the gfx950 extension is required on a GPU box but could not be loaded: "
            f"{load_error()}. Set DLION_ALLOW_TORCH_FALLBACK=1 to run the (slow) PyTorch oracle instead."
        )


def ops():
    require()
    return torch.ops.dlion
