"""Drop-in module name of the reference optimizer (``from distributed_lion import Lion``).

Re-exports the MI355X-native implementation; see
distributed_lion_pytorch_amd/optim/lion.py (reference: /root/reference/distributed_lion.py).
"""
from distributed_lion_pytorch_amd.optim.lion import (  # noqa: F401
    Lion,
    exists,
    flatten_and_pad,
    majority_vote,
    restore_flattened_tensor,
    update_fn,
    update_fn_distributed,
    update_fn_distributed_stoc,
)

__all__ = ["Lion", "exists", "flatten_and_pad", "majority_vote", "restore_flattened_tensor", "update_fn",
           "update_fn_distributed", "update_fn_distributed_stoc"]
