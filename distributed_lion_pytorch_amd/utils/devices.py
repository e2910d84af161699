"""Counting GPUs without creating a HIP context.

A launcher parent (``bench.py --gpus N``, ``launch.py``) must never initialise
the GPU before it starts the rank processes: on this pool replacing or forking
a process that holds a HIP context takes the machine down, and a context in
the parent also pins memory on device 0.  ``torch.cuda.device_count()`` is
context-free only while amdsmi works -- when amdsmi fails it silently falls
back to ``hipGetDeviceCount`` (``torch/cuda/__init__.py`` ``device_count``).
:func:`visible_gpu_count` never takes that fallback: amdsmi first, then the
KFD topology in sysfs, and ``None`` when neither answers (the caller then
refuses loudly instead of guessing).
"""
from __future__ import annotations

import glob
import os
from typing import List, Optional


def _visible_filter() -> Optional[List[str]]:
    """Entries of the first set visibility variable (HIP's order of precedence),
    or None when none is set."""
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return [x.strip() for x in v.split(",") if x.strip() != ""]
    return None


def _amdsmi_count() -> Optional[int]:
    try:
        import torch

        if not getattr(torch.version, "hip", None):
            return None
        from torch.cuda import _device_count_amdsmi  # applies the *_VISIBLE_DEVICES filters itself

        n = _device_count_amdsmi()
        return n if n >= 0 else None
    except Exception:  # noqa: BLE001 - no amdsmi: try sysfs
        return None


def _kfd_count(root: str = "/sys/class/kfd/kfd/topology/nodes") -> Optional[int]:
    nodes = sorted(glob.glob(os.path.join(root, "*", "properties")))
    if not nodes:
        return None
    gpus = 0
    for path in nodes:
        try:
            with open(path) as f:
                props = dict(line.split(None, 1) for line in f if len(line.split(None, 1)) == 2)
        except OSError:
            continue
        if int(props.get("simd_count", "0").strip() or 0) > 0:  # CPU nodes have no SIMDs
            gpus += 1
    vis = _visible_filter()
    if vis is not None:
        gpus = min(gpus, len(vis))
    return gpus


def visible_gpu_count() -> Optional[int]:
    """GPUs this process may use, counted without a HIP call; None if unknown."""
    n = _amdsmi_count()
    if n is not None:
        return n
    return _kfd_count()
