"""Linear layers whose weight gradient is a split-K GEMM.

The training GEMMs of a transformer layer have two easy shapes (forward and
input-gradient: M = tokens, large) and one hard shape: the weight gradient
dW = X^T dY reduces over all M = B*T tokens (20480 in the GPT-2 bench) into a
small [K, N] output -- 9-36 256x256 output tiles for GPT-2 -- so a plain GEMM
fills 9-36 of the 256 CUs.  Measured on MI355X (tools/bench_gemm.py):
182-490 TF/s for hipBLASLt's own choice vs 540-840 TF/s when the token axis
is split S ways into a batched GEMM with fp32 output (``bmm(out_dtype=f32)``),
summed in fp32 and rounded once.  S is picked so that S x tiles ~ 160.

Gradient-accumulation fusion (``grad_accumulation_fusion``): with gradient
accumulation every micro-batch's weight gradient would otherwise be written
to a fresh tensor and then added into ``param.grad`` by autograd's
AccumulateGrad (one extra read-read-write pass over every weight per
micro-batch).  With fusion on, the backward deposits the weight gradient
straight into ``param.grad``: the split-K reduction adds the running gradient
in the same pass (``sum_partials_acc_``), the unsplit GEMM accumulates with
beta = 1 (``addmm_``).  The backward then returns no gradient for the weight,
so this bypasses AccumulateGrad and its hooks -- enable it only in loops
that own the gradients (the native TrainStep does; DDP gradient hooks would
not see these weights).

Split-K accumulators across micro-batches: inside one fusion window (the
micro-batches of one optimizer step) a split-K weight gradient is not reduced
per micro-batch.  Its fp32 partials live in a persistent [S, K, N] buffer; the
first micro-batch writes it (``bmm``), later ones accumulate in the GEMM
epilogue (``baddbmm``, beta = 1), and the window's exit reduces every buffer
into ``param.grad`` once.  Measured at the GPT-2 shapes with GA = 8
(tools/bench_wgrad_acc.py): 3-8 us less per weight gradient per micro-batch,
and the micro-batch sum is fp32 instead of a bf16 running gradient.  Buffers
are capped by ``_ACC_BUDGET`` bytes (large models have S = 1 and never use it).

Memory cost: the buffers hold S x (weight numel) fp32 per split-K weight (about
2 GB at GPT-2-124M) and stay allocated between steps so that the next window
reuses them.  They are only used when the window is known to span more than
one micro-batch (``grad_accumulation_fusion(micro_batches=n)`` with n > 1, or
n unknown); ``release_split_k_accumulators()`` frees them.  A change of split factor inside a window
(micro-batches with different token counts) first flushes the running
partials into ``param.grad``, then starts a fresh buffer.

Deferred weight gradients (own TN kernel, csrc/gemm_tn.hip): inside a
multi-micro-batch window the weight gradient is not computed per micro-batch
at all.  Its two token-major operands (the layer input and the output
gradient) are kept, and the window's exit runs ONE GEMM per weight whose
reduction axis is the concatenation of all micro-batches (the kernel takes up
to 16 operand segments): the fp32 split-K partials are written once per step
instead of read-modified-written every micro-batch, and each split runs a
long K.  Measured at the GPT-2 bench shapes (tools/bench_wgrad.py --window 8):
c_fc / mlp c_proj 103 -> 80 us, c_attn 86 -> 62 us, attn c_proj 43 -> 29 us
per micro-batch.  The kept operands cost memory (~500 MB per GPT-2 layer per
micro-batch at 20480 tokens), capped by ``DLION_WGRAD_DEFER_GB`` (default:
a quarter of the device memory); past the cap, or at 16 segments, a weight's
segments are reduced early into its accumulator.
"""
from __future__ import annotations

import contextlib
import math
import os
import weakref

import torch

_ACC_BUDGET = 8 << 30  # bytes of fp32 accumulators
_WDEFER_ON = True  # window-level deferred weight gradients (tests compare the per-micro-batch form)
_WDEFER_MAX_SEG = 16  # csrc/gemm_tn.hip kMaxSeg


class _FusionState:
    """The fusion window's state -- process-wide on purpose: PyTorch runs the
    CUDA backward on its own per-device autograd thread, so a window opened by
    the training loop's thread must be visible there (a thread-local copy
    deposited every micro-batch immediately).  Entries are keyed by parameter,
    so several models trained in one window (e.g. a policy and a trainable
    second model) keep separate accumulators; one training loop per process
    owns the window.  Device memory held here is bounded by ``_ACC_BUDGET`` +
    ``_wdefer_budget()``, which trainer/memory.py counts."""

    def __init__(self):
        self.fuse = {"on": False, "multi": True, "nodefer": False, "n_mb": 8}  # n_mb: micro-batches per window (8 if unknown)
        self.acc: dict = {}  # key -> [weakrefs of params, fp32 buffer [S, ...], [(param ref, col0, ncols)]]
        self.pending: list = []  # keys written in the current window, in order
        self.wdefer: dict = {}  # key -> [params, cols, [a segments], [b segments], [versions]]
        self.wdefer_bytes = [0]


_ST = _FusionState()


@contextlib.contextmanager
def grad_accumulation_fusion(enabled: bool = True, micro_batches: int | None = None):
    """Fusion window = the micro-batches of one optimizer step.  ``micro_batches``
    (if known) gates the split-K accumulators: with one micro-batch they save
    nothing, so the weight gradient is reduced straight into ``param.grad``."""
    prev = (_ST.fuse["on"], _ST.fuse["multi"])
    outer = bool(enabled) and not prev[0]
    _ST.fuse["on"] = bool(enabled)
    if outer:
        _ST.fuse["multi"] = micro_batches is None or int(micro_batches) > 1
        _ST.fuse["n_mb"] = int(micro_batches) if micro_batches else 8
    ok = False
    try:
        yield
        ok = True
    finally:
        _ST.fuse["on"], _ST.fuse["multi"] = prev
        if outer:
            if ok:
                flush_split_k_accumulators()
                flush_deferred_partials()
            _ST.pending.clear()
            _clear_deferred()
            _drop_deferred()
            _TCOPY.clear()
            _ST.fuse["nodefer"] = False


def begin_fusion_window(micro_batches: int | None = None) -> bool:
    """Non-context form of :func:`grad_accumulation_fusion` for loops that do
    not own the micro-batch iteration (the HF Trainer's ``training_step`` runs
    once per micro-batch).  Returns False if a window is already open."""
    if _ST.fuse["on"]:
        return False
    _ST.fuse["on"] = True
    _ST.fuse["multi"] = micro_batches is None or int(micro_batches) > 1
    _ST.fuse["n_mb"] = int(micro_batches) if micro_batches else 8
    return True


def end_fusion_window(flush: bool = True) -> None:
    """Close the window opened by :func:`begin_fusion_window`: every weight
    gradient of the window is in ``param.grad`` afterwards."""
    if not _ST.fuse["on"]:
        return
    _ST.fuse["on"], _ST.fuse["multi"] = False, True
    if flush:
        flush_split_k_accumulators()
        flush_deferred_partials()
    _ST.pending.clear()
    _clear_deferred()
    _drop_deferred()
    _TCOPY.clear()
    _ST.fuse["nodefer"] = False


def fusion_window_open() -> bool:
    return bool(_ST.fuse["on"])


def no_wgrad_deferral_this_window() -> None:
    """Called by activation-checkpointed forwards: keeping every micro-batch's
    layer inputs alive until the window's exit would undo the checkpointing's
    memory saving, so this window computes its weight gradients per
    micro-batch (into the fp32 accumulators) instead."""
    if _ST.fuse["on"]:
        _ST.fuse["nodefer"] = True


def _flush_entry(ent) -> None:
    flat = ent[1].view(ent[1].shape[0], -1)
    for ref, c0, n in ent[2]:
        p = ref()
        if p is not None:
            deposit_grad(p, flat[:, c0:c0 + n])


def _wdefer_budget() -> int:
    gb = os.environ.get("DLION_WGRAD_DEFER_GB")
    if gb is not None:
        return int(float(gb) * (1 << 30))
    try:
        return torch.cuda.get_device_properties(torch.cuda.current_device()).total_memory // 4
    except Exception:
        return 0


def _run_deferred(key) -> None:
    """One TN GEMM over every kept segment of `key` into its accumulator."""
    from . import hip

    params, cols, segs_a, segs_b, vers = _ST.wdefer.pop(key)
    _ST.wdefer_bytes[0] -= sum(t.numel() * t.element_size() for t in segs_a + segs_b)
    for i, (t, v) in enumerate(zip((x for pair in zip(segs_a, segs_b) for x in pair), vers)):
        if t._version != v:
            shapes = [tuple(r().shape) if r() is not None else None for r in params]
            raise RuntimeError(f"dlion: an operand kept for a deferred weight gradient was modified in place "
                               f"(weights {shapes}, micro-batch {i // 2}, operand {'ab'[i % 2]} {tuple(t.shape)}, "
                               f"version {v} -> {t._version})")
    ent = _ST.acc[key]
    accumulate = key in _ST.pending
    hip.ops().gemm_tn_(segs_a, segs_b, ent[1], accumulate)
    if not accumulate:
        _ST.pending.append(key)


def _run_all_deferred() -> None:
    for key in list(_ST.wdefer):
        _run_deferred(key)


def _drop_deferred() -> None:
    _ST.wdefer.clear()
    _ST.wdefer_bytes[0] = 0


def _defer_wgrad(params, cols, a, b, s) -> bool:
    """Keep a^T b's operands for one window-level GEMM (see the module notes).
    False if not applicable (fallback: _acc_gemm now)."""
    if not (_WDEFER_ON and _ST.fuse["multi"]) or _ST.fuse["nodefer"]:
        return False
    key = tuple(id(p) for p in params)
    nb = a.numel() * a.element_size() + b.numel() * b.element_size()
    ent = _ST.wdefer.get(key)
    if ent is not None:
        a0, b0 = ent[2][0], ent[3][0]
        if (a.shape != a0.shape or b.shape != b0.shape or a.stride() != a0.stride() or b.stride() != b0.stride()
                or any(r() is not p for r, p in zip(ent[0], params))):
            _run_deferred(key)
            ent = None
    if _ST.wdefer_bytes[0] + nb > _wdefer_budget():
        if ent is not None:
            _run_deferred(key)
        return False
    if ent is None:
        # the accumulator [s, R, C] the window's exit reduces into param.grad
        if not _ensure_acc(params, cols, (s, a.shape[1], b.shape[1]), a.device):
            return False
        ent = _ST.wdefer[key] = [[weakref.ref(p) for p in params], cols, [], [], []]
    ent[2].append(a)
    ent[3].append(b)
    ent[4].extend([a._version, b._version])
    _ST.wdefer_bytes[0] += nb
    if len(ent[2]) == _WDEFER_MAX_SEG:
        _run_deferred(key)
    return True


def flush_split_k_accumulators() -> None:
    """Reduce every split-K accumulator written in this window into its
    parameters' ``.grad`` (one fused sum + deposit per weight)."""
    _run_all_deferred()
    for key in _ST.pending:
        ent = _ST.acc.get(key)
        if ent is not None:
            _flush_entry(ent)
    _ST.pending.clear()


def release_split_k_accumulators() -> None:
    """Free every split-K accumulator (flushing the open window's partials
    into ``param.grad`` first).  Call after training to return the memory."""
    flush_split_k_accumulators()
    flush_deferred_partials()
    _drop_deferred()
    _ST.acc.clear()


def _ensure_acc(params, cols, shape, device) -> bool:
    """Make sure the window accumulator of `params` has `shape` (flushing a
    differently shaped one that already holds this window's partials)."""
    key = tuple(id(p) for p in params)
    ent = _ST.acc.get(key)
    if ent is not None and all(r() is p for r, p in zip(ent[0], params)) and tuple(ent[1].shape) == tuple(shape):
        return True
    if ent is not None:
        if key in _ST.pending:
            # split factor / token count changed inside the window: the
            # partials so far go into param.grad before the buffer is replaced
            _flush_entry(ent)
            _ST.pending.remove(key)
        _ST.acc.pop(key)
    used = sum(e[1].numel() * 4 for e in _ST.acc.values() if all(r() is not None for r in e[0]))
    for k in [k for k, e in _ST.acc.items() if any(r() is None for r in e[0])]:
        _ST.acc.pop(k)  # parameters gone: drop their buffers
        if k in _ST.pending:
            _ST.pending.remove(k)
    if used + math.prod(shape) * 4 > _ACC_BUDGET:
        return False
    buf = torch.empty(shape, device=device, dtype=torch.float32)
    _ST.acc[key] = [[weakref.ref(p) for p in params], buf, [(weakref.ref(p), c0, n) for p, (c0, n) in zip(params, cols)]]
    return True


def _acc_gemm(params, cols, a, b, s) -> bool:
    """Accumulate the s split-K partials of a^T b (fp32, [s, R, C]; a [T, R],
    b [T, C] token-major) into the window's buffer for `params` (column blocks
    `cols` of the flattened R*C).  False if the buffer cannot be used (over
    budget, single-micro-batch window): the caller then deposits into
    ``param.grad`` directly, on top of any flushed partials."""
    if not _ST.fuse["multi"]:
        return False
    key = tuple(id(p) for p in params)
    if key in _ST.wdefer:
        _run_deferred(key)  # keep the micro-batch order of the accumulation simple
    if not _ensure_acc(params, cols, (s, a.shape[1], b.shape[1]), a.device):
        return False
    ent = _ST.acc[key]
    accumulate = key in _ST.pending
    wgrad_partials(a, b, s, out=ent[1], accumulate=accumulate)
    if not accumulate:
        _ST.pending.append(key)
    return True


# ------------------------------------------------------- weight-gradient GEMMs
# dW = a^T b over the tokens: both operands token-major.  The own TN kernel
# (csrc/gemm_tn.hip) writes / accumulates fp32 split-K partials; measured at
# the GPT-2 shapes against torch.bmm / baddbmm (hipBLASLt) with each side's
# best split (tools/bench_wgrad.py, 20480 tokens): c_attn 69 vs 94 us, c_fc
# 86 vs 110, mlp c_proj 86 vs 107, attn c_proj 40 vs 38.
def _tn_eligible(a: torch.Tensor, b: torch.Tensor) -> bool:
    return (a.is_cuda and a.dtype == b.dtype == torch.bfloat16 and a.dim() == b.dim() == 2
            and a.shape[0] == b.shape[0] and a.shape[0] % 128 == 0 and a.shape[1] % 8 == 0 and b.shape[1] % 8 == 0
            and a.stride(1) == 1 and b.stride(1) == 1 and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0
            and a.stride(0) >= a.shape[1] and b.stride(0) >= b.shape[1]
            and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0
            and a.shape[0] * max(a.stride(0), b.stride(0)) < 2 ** 31)


_TN_WAVE = 256  # grid-size target of tn_split_factor: one block per CU
_TN_MIN_TILES = 16  # below: hipBLASLt (attn c_proj 768x768, 9 tiles: 43 us vs 55 us in the step)


_TN_CU_RATE = 4.9e12  # FLOP/s of one CU in the TN kernel (1.25 PF/s over 256 CUs)
_TN_BW = 5.0e12  # B/s for the fp32 partials (written once, read once by the reduction)


def tn_split_factor(M: int, R: int, C: int, max_split: int = 16, direct: bool = False) -> int:
    """Splits of the token axis for the own TN kernel: minimises waves of
    (256x256 tiles x splits) blocks x per-block time + the fp32 partial
    traffic (splits x R x C x 8 bytes).  GPT-2 c_fc: 7 (252 blocks, one wave),
    c_attn: 9; the LM head's 591 tiles: 3 (7 waves instead of 3 long ones).
    direct: the unsplit launch writes the bf16 gradient itself (no fp32
    partials, no reduction pass), and a last wave that holds only part of
    the CUs runs ~0.7 x a full wave's time (the blocks get the chip's HBM and
    power to themselves): Llama-3-8B down_proj (896 tiles) 810 us unsplit vs
    814 + 108 us at s = 2 (tools/r5/bench_tn_llama.py, profiles/r5/)."""
    tiles = math.ceil(R / 256) * math.ceil(C / 256)
    best, best_cost = 1, None
    t_full = (2.0 * 65536 * M) / _TN_CU_RATE
    for s in range(1, max(1, min(max_split, M // 128)) + 1):
        if direct and s == 1:
            full_waves, rem = divmod(tiles, _TN_WAVE)
            cost = (full_waves + (0.7 if rem else 0.0)) * t_full
        else:
            waves = math.ceil(tiles * s / _TN_WAVE)
            cost = waves * (2.0 * 65536 * M / s) / _TN_CU_RATE + 8.0 * s * R * C / _TN_BW
        if best_cost is None or cost < best_cost:
            best, best_cost = s, cost
    return best


def wgrad_splits(a: torch.Tensor, b: torch.Tensor) -> tuple:
    """(split count, own TN kernel?) for a^T b."""
    from . import hip

    M, R, C = a.shape[0], a.shape[1], b.shape[1]
    # small outputs: hipBLASLt per micro-batch, but the own kernel when the
    # window defers the GEMM (attn c_proj over 8 micro-batches: 29 vs 43 us/mb)
    deferred = _WDEFER_ON and _ST.fuse["on"] and _ST.fuse["multi"] and not _ST.fuse["nodefer"]
    if ((deferred or math.ceil(R / 256) * math.ceil(C / 256) >= _TN_MIN_TILES) and _tn_eligible(a, b)
            and hip.available()):
        if deferred:
            # the window's GEMM reduces over every micro-batch's tokens: size the
            # split for that K (GPT-2 attn c_proj, 9 tiles: 28 splits = 252 blocks
            # instead of the per-micro-batch choice of 16 = 144 blocks, 0.77 PF/s)
            # (capped by one micro-batch's rows: a window flushed early -- budget, 16
            # segments -- may run with a single segment)
            return tn_split_factor(M * _ST.fuse["n_mb"], R, C, max_split=min(32, M // 128)), True
        # outside a multi-micro-batch window an unsplit launch writes the bf16
        # gradient itself (wgrad_into / _multi_wgrad_into): no fp32 partials
        return tn_split_factor(M, R, C, direct=not (_ST.fuse["on"] and _ST.fuse["multi"])), True
    return split_k_factor(M, R, C), False


def wgrad_partials(a: torch.Tensor, b: torch.Tensor, s: int, out=None, accumulate: bool = False,
                   own: bool | None = None) -> torch.Tensor:
    """fp32 [s, R, C] split-K partials of a^T b (a [T, R], b [T, C]); into /
    onto `out` when given.  own: use the TN kernel (default: wgrad_splits'
    choice)."""
    from . import hip

    M = a.shape[0]
    if own is None:
        own = wgrad_splits(a, b)[1]
    if own and s <= M // 128:
        if out is None:
            return hip.ops().gemm_tn([a], [b], s)
        hip.ops().gemm_tn_([a], [b], out, accumulate)
        return out
    a3, b3 = a.view(s, M // s, a.shape[1]).transpose(1, 2), b.view(s, M // s, b.shape[1])
    if out is None:
        return torch.bmm(a3, b3, out_dtype=torch.float32)
    if accumulate:
        torch.baddbmm(out, a3, b3, out_dtype=torch.float32, out=out)
    else:
        torch.bmm(a3, b3, out_dtype=torch.float32, out=out)
    return out


def _fuse_target(w) -> bool:
    return (_ST.fuse["on"] and isinstance(w, torch.nn.Parameter) and w.requires_grad and w.is_cuda
            and w.dtype == torch.bfloat16 and w.is_contiguous())


# --------------------------------------------- deferred small partial reductions
# Bias / norm-parameter gradients arrive as fp32 partial stacks [P, n] (one row
# per block of the producing kernel: 25 residual+norm boundaries, the c_attn
# and MLP biases of GPT-2 -- ~43 per micro-batch).  Reducing each one as it
# arrives costs a ~9 us latency-bound launch apiece; inside a window of several
# micro-batches the stacks are kept instead and every key is reduced ONCE per
# optimizer step (one launch over the concatenated stacks), i.e. 1/GA of the
# launches.  Only small stacks are deferred (<= _DEFER_MAX_PART bytes each,
# _DEFER_CAP in total; GPT-2 keeps ~1.7 GB across 8 micro-batches).
_DEFER_MAX_PART = 64 << 20
_DEFER_CAP = 8 << 30
_DEFER: dict = {}  # key -> [deposit fn, [part stacks]]
_DEFER_BYTES = [0]


def defer_partials(key, part2d: torch.Tensor, fn) -> bool:
    """Keep ``part2d`` for ``fn(concatenated stacks)`` at the window's end.
    False (nothing kept) outside a multi-micro-batch window or over budget:
    the caller then deposits now."""
    if not (_ST.fuse["on"] and _ST.fuse["multi"]):
        return False
    nb = part2d.numel() * part2d.element_size()
    if nb > _DEFER_MAX_PART or _DEFER_BYTES[0] + nb > _DEFER_CAP:
        return False
    ent = _DEFER.get(key)
    if ent is None:
        ent = _DEFER[key] = [fn, []]
    elif ent[1] and ent[1][0].shape[1:] != part2d.shape[1:]:
        return False
    ent[1].append(part2d)
    _DEFER_BYTES[0] += nb
    return True


class PartList:
    """The kept per-micro-batch partial stacks of one deferred key, reduced
    together by one multi-stack kernel (``sum_partials_multi_``) instead of
    being concatenated first (the concatenations were ~1 ms per GPT-2 step).
    Supports the column slices the deposit functions take."""

    def __init__(self, parts):
        self.parts = parts

    def __getitem__(self, idx):
        return PartList([p[idx] for p in self.parts])

    @property
    def shape(self):
        return (sum(p.shape[0] for p in self.parts),) + tuple(self.parts[0].shape[1:])


def sum_partials_into(part, out=None, accumulate: bool = False) -> torch.Tensor:
    """bf16 column sums of fp32 partials (a [S, n] tensor, row-strided OK, or a
    PartList), written to / added onto `out` (new [n] tensor if None)."""
    from . import hip

    if out is None:
        n = part.shape[1]
        dev = part.parts[0].device if isinstance(part, PartList) else part.device
        if not isinstance(part, PartList):
            return hip.ops().sum_partials(part)
        out = torch.empty(n, dtype=torch.bfloat16, device=dev)
        accumulate = False
    if isinstance(part, PartList):
        hip.ops().sum_partials_multi_(part.parts, out, accumulate)
    elif accumulate:
        hip.ops().sum_partials_acc_(part, out)
    else:
        out.copy_(hip.ops().sum_partials(part).view_as(out))
    return out


def flush_deferred_partials() -> None:
    items = list(_DEFER.values())
    _clear_deferred()
    for fn, parts in items:
        if len(parts) == 1:
            fn(parts[0])
        elif len(parts) <= 16:
            fn(PartList(parts))
        else:
            fn(torch.cat(parts, 0))


def _clear_deferred() -> None:
    _DEFER.clear()
    _DEFER_BYTES[0] = 0


def deposit_grad(param: torch.nn.Parameter, part2d: torch.Tensor, defer: bool = True) -> None:
    """param.grad (+)= column sums of fp32 partials [S, numel] (row-strided OK),
    in one kernel: the reduction adds the running gradient in the same pass.
    Inside a multi-micro-batch window small stacks are reduced at its end."""
    from . import hip

    if defer and defer_partials(("g", id(param)), part2d, lambda pc: deposit_grad(param, pc, defer=False)):
        return
    g = param.grad
    if g is None or not (g.is_contiguous() and g.dtype == param.dtype):
        fresh = sum_partials_into(part2d).view_as(param)
        param.grad = fresh if g is None else g + fresh
    else:
        sum_partials_into(part2d, g.view(-1), accumulate=True)


def _colsum_parts(rows: int) -> int:
    return max(1, min(1024, rows // 16))


def bias_grad(dy: torch.Tensor, b, fuse: bool):
    """Bias gradient = column sums of dy [M, N]; deposited into b.grad when fused
    (returns None then).  One streaming kernel + a tall partial sum instead of
    ATen's column reduction (~2x slower at [20480, 2304])."""
    from . import hip

    if dy.is_cuda and dy.dtype == torch.bfloat16 and dy.shape[1] % 8 == 0 and hip.available():
        part = hip.ops().colsum_partials(dy, _colsum_parts(dy.shape[0]))
        if fuse:
            deposit_grad(b, part)
            return None
        return hip.ops().sum_partials(part)
    return dy.sum(0)


def split_k_factor(M: int, K: int, N: int) -> int:
    tiles = math.ceil(K / 256) * math.ceil(N / 256)
    if tiles >= 160:
        return 1
    s = 2 ** int(round(math.log2(160.0 / tiles)))
    s = max(1, min(16, s))
    while s > 1 and M % s:
        s //= 2
    return s


def _wgrad_via_transposes(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, accumulate: bool) -> bool:
    """out (+)= a^T b as hipBLASLt's NT form (both operands contraction-
    contiguous, its fastest layout: 1.5-1.6 PF/s at Llama-3-8B shapes against
    1.1-1.3 for the TN forms) on token-contiguous copies a^T, b^T made by the
    LDS-tiled transpose kernel -- the copies cost about a fifth of the GEMM
    at gate_up / down_proj and the sum still wins there
    (tools/r5/bench_wgrad_lt.py, profiles/r5/wgrad_tt_c27.txt)."""
    from . import hip

    at, bt = _transposed(a), _transposed(b)
    ok = hip.ops().lt_gemm_nt_acc(at, bt, out, accumulate)
    del at, bt
    return ok


# Token-contiguous copies written by the producing kernels themselves (the
# SwiGLU backward's dgu^T, the SwiGLU forward's h^T: one extra write instead of
# a transpose pass that reads the operand again), offered to the
# transposed-copy weight gradients.  An entry holds the original too, so its
# address cannot be reused while the entry lives; entries die when consumed,
# at the window's end, or past _TCOPY_MAX (oldest first).
_TCOPY: dict = {}  # data_ptr -> (tensor, its transposed copy)
_TCOPY_MAX = 160
_TT_A: set = set()  # (rows, cols) of a-operands (dY) whose weight gradient picked "lt_tt"
_TT_B: set = set()  # (rows, cols) of b-operands (X)



def want_transposed_copy(rows: int, cols: int, operand: str = "a") -> bool:
    """Should a producer of a [rows, cols] weight-gradient operand (a = the
    output gradient, b = the layer input) also write its transpose?  Never
    inside an activation-checkpointed window: an input's copy would be kept
    from the forward to the backward; and never in a multi-micro-batch window,
    whose weight gradients are deferred to its exit or summed in the split-K
    accumulators (the transposed-copy form only runs outside one: a copy
    would only pin memory and cost a write)."""
    if _ST.fuse["on"] and _ST.fuse["multi"]:
        return False
    if operand == "b" and (_ST.fuse["nodefer"] or not _ST.fuse["on"]):
        return False
    return (int(rows), int(cols)) in (_TT_A if operand == "a" else _TT_B)


def register_transposed(t: torch.Tensor, tt: torch.Tensor) -> None:
    while len(_TCOPY) >= _TCOPY_MAX:
        _TCOPY.pop(next(iter(_TCOPY)))
    _TCOPY[t.data_ptr()] = (t, tt)


def _transposed(t: torch.Tensor) -> torch.Tensor:
    ent = _TCOPY.pop(t.data_ptr(), None)
    if ent is not None and _same_view(ent[0], t):
        return ent[1]
    return fast_transpose(t)


def _same_view(x: torch.Tensor, y: torch.Tensor) -> bool:
    return x.data_ptr() == y.data_ptr() and x.shape == y.shape and x.stride() == y.stride()


def _direct_split_pick(a: torch.Tensor, b: torch.Tensor, s: int, own: bool) -> bool:
    """A split own-TN weight gradient outside a multi-micro-batch window goes
    through _unsplit_wgrad's per-shape timing instead (the split launch is one
    of its candidates): hipBLASLt's TN form is faster at some shapes
    (Llama-3-8B q/k/v: 352 vs 399 us, profiles/r5/wgrad_lt_c20.txt)."""
    M, K = a.shape
    return (own and s > 1 and not (_ST.fuse["on"] and _ST.fuse["multi"]) and a.dtype == torch.bfloat16
            and _tunable(a, M, b.shape[1], K))


def _unsplit_wgrad(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, accumulate: bool, split: int = 1) -> None:
    """out [K, N] bf16 (+)= a^T b: the own TN kernel's unsplit bf16 epilogue,
    hipBLASLt's TN GEMM (ATen's heuristic or the searched algorithm; beta = 1 to
    accumulate), or (split > 1) the own kernel's split-K partials + one reduction
    pass, whichever the per-shape timing (see gemm_fwd) finds fastest.  All
    round the fp32 sum (+ out) once."""
    from . import hip

    M, K = a.shape
    N = b.shape[1]
    out2 = out.view(K, N)
    if _tunable(a, M, N, K):
        key = ("wgrad", M, K, N, a.stride(0), b.stride(0), split)
        name = _GEMM_PICK.get(key)
        if name is None:
            scratch = torch.empty(K, N, dtype=out.dtype, device=out.device)
            cands = {"tn": lambda: hip.ops().gemm_tn_([a], [b], scratch, False),
                     "blas": lambda: torch.mm(a.t(), b, out=scratch)}
            if split > 1:
                cands["split"] = lambda: hip.ops().sum_partials_multi_(
                    [hip.ops().gemm_tn([a], [b], split).view(split, K * N)], scratch.view(-1), False)
            if _lt_nn_ok(a, b):  # hipBLASLt's TN form with the searched algorithm
                cands["lt"] = lambda: hip.ops().lt_gemm_tn(a, b, scratch, False) or torch.mm(a.t(), b, out=scratch)
                cands["lt_tt"] = lambda: (_wgrad_via_transposes(a, b, scratch, False)
                                          or torch.mm(a.t(), b, out=scratch))
            name = _pick(key, cands)
            if name == "lt_tt":
                _TT_A.add((M, K))
                _TT_B.add((M, N))
            del scratch
        if name == "lt" and hip.ops().lt_gemm_tn(a, b, out2, accumulate):
            return
        if name == "lt_tt" and _wgrad_via_transposes(a, b, out2, accumulate):
            return
        if name == "split":
            hip.ops().sum_partials_multi_([hip.ops().gemm_tn([a], [b], split).view(split, K * N)], out2.view(-1),
                                          accumulate)
            return
        if name in ("blas", "lt", "lt_tt"):
            if accumulate:
                out2.addmm_(a.t(), b)
            else:
                torch.mm(a.t(), b, out=out2)
            return
    hip.ops().gemm_tn_([a], [b], out, accumulate)


def wgrad_into(a: torch.Tensor, b: torch.Tensor, w: torch.nn.Parameter) -> None:
    """w.grad (+)= a^T @ b, deposited in place (a [M, K], b [M, N], w [K, N])."""
    g = w.grad
    M, K = a.shape
    N = b.shape[1]
    s, own = wgrad_splits(a, b)
    grad_ok = g is None or (g.is_contiguous() and g.dtype == w.dtype)
    if (s > 1 or own) and (K * N) % 4 == 0 and grad_ok and (own or M % s == 0):  # own kernel: uneven splits OK
        from . import hip

        if hip.available():
            timed = w.dtype == torch.bfloat16 and _direct_split_pick(a, b, s, own)
            if _ST.fuse["on"] and not timed and ((own and _defer_wgrad([w], [(0, K * N)], a, b, s))
                                                 or _acc_gemm([w], [(0, K * N)], a, b, s)):
                return  # reduced into w.grad when the accumulation window closes
            g = w.grad  # _acc_gemm may have flushed earlier partials into it
            grad_ok = g is None or (g.is_contiguous() and g.dtype == w.dtype)
            if grad_ok and own and (s == 1 or timed) and w.dtype == torch.bfloat16:
                # unsplit: the TN kernel writes (adds onto) the bf16 gradient itself
                if g is None:
                    w.grad = g = torch.empty_like(w, memory_format=torch.contiguous_format)
                    _unsplit_wgrad(a, b, g, False, s)
                else:
                    _unsplit_wgrad(a, b, g, True, s)
                return
            if grad_ok:
                part = wgrad_partials(a, b, s).view(s, K * N)
                if g is None:
                    w.grad = hip.ops().sum_partials(part).view_as(w)
                else:
                    hip.ops().sum_partials_acc_(part, g)
                return
    if not grad_ok or g is None:
        fresh = wgrad(a, b)
        w.grad = fresh if g is None else g + fresh
        return
    g.addmm_(a.t(), b)


def wgrad(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a^T @ b for a [M, K], b [M, N] (-> [K, N]) with token-axis split-K."""
    M, K = a.shape
    N = b.shape[1]
    if not (a.is_cuda and a.dtype in (torch.bfloat16, torch.float16)):
        return a.t() @ b
    s, own = wgrad_splits(a, b)
    if (s == 1 and not own) or (M % s and not own):
        return a.t() @ b
    if own and s == 1 and a.dtype == torch.bfloat16:
        from . import hip

        out = torch.empty(K, N, dtype=a.dtype, device=a.device)
        hip.ops().gemm_tn_([a], [b], out, False)  # bf16 straight from the accumulators
        return out
    part = wgrad_partials(a, b, s)
    if a.dtype == torch.bfloat16 and (K * N) % 4 == 0:
        from . import hip

        if hip.available():
            return hip.ops().sum_partials(part.view(s, K * N)).view(K, N)  # one pass: fp32 sum -> bf16
    return part.sum(0).to(a.dtype)


# ------------------------------------------------------ transposed weight cache
# hipBLASLt runs the forward GEMM of an HF Conv1D ([K, N] weight) ~8 % faster
# with the weight in [N, K] ("NT": both operands K-contiguous; measured with
# tools/bench_gemm.py, e.g. GPT-2 qkv 73.6 -> 68.5 us, fc 97.4 -> 89.1 us at
# 20480 tokens).  Weights change once per optimizer step while every
# micro-batch reuses them, so a transposed copy is made once per step.  The
# Lion kernels update weights through raw pointers (no autograd version
# bump), hence the explicit generation counter bumped by Lion.step; any other
# in-place update (AdamW, load_state_dict) bumps the tensor's _version.
_WEIGHT_GEN = [0]
_WT_CACHE: dict = {}  # (id(w), tag) -> (weakref(w), key, derived tensor); entries die with w


def bump_weight_generation() -> None:
    _WEIGHT_GEN[0] += 1


def cached_derived(w: torch.Tensor, tag: str, fn) -> torch.Tensor:
    """fn(w.detach()) cached until w changes (in place or via the next Lion
    step).  Used for per-step weight layouts (transposed, vocab-padded)."""
    import weakref

    key = (w._version, _WEIGHT_GEN[0] if w.requires_grad else -1, w.data_ptr())  # frozen: see cat_weights
    ck = (id(w), tag)
    hit = _WT_CACHE.get(ck)
    if hit is not None and hit[0]() is w and hit[1] == key:
        return hit[2]
    with torch.no_grad():
        out = fn(w.detach())
    if hit is None or hit[0]() is not w:
        weakref.finalize(w, _WT_CACHE.pop, ck, None)
    _WT_CACHE[ck] = (weakref.ref(w), key, out)
    return out




def fast_transpose(t: torch.Tensor, rows_out: int | None = None) -> torch.Tensor:
    """t.t().contiguous() (zero-padded to ``rows_out`` columns if given) -- the
    LDS-tiled gfx950 kernel for 16-bit GPU matrices (ATen's strided copy ran
    the GPT-2 per-step weight transposes at 0.2-0.6 TB/s), ATen otherwise."""
    from . import hip

    rp = t.shape[0] if rows_out is None else rows_out
    if (t.is_cuda and t.dim() == 2 and t.element_size() == 2 and t.stride(1) == 1 and t.stride(0) % 8 == 0
            and rp % 8 == 0 and t.data_ptr() % 16 == 0 and hip.available()):
        return hip.ops().transpose_pad(t, rp)
    out = t.t().contiguous()
    if rp != t.shape[0]:
        out = torch.cat([out, out.new_zeros(out.shape[0], rp - t.shape[0])], 1)
    return out


def transposed_weight(w: torch.Tensor) -> torch.Tensor:
    """Contiguous w.t() cached until w changes (next optimizer step)."""
    return cached_derived(w, "t", lambda t: fast_transpose(t))


# ------------------------------------------------ per-shape GEMM choice (Llama sizes)
# hipBLASLt's first heuristic (what ATen calls) is not the fastest option for
# every Llama projection, and the input gradient dX = dY.W runs in the NN
# layout, slower than the NT form against a cached W^T.  Measured at the
# Llama-2-7B SFT micro-batch (4096 tokens, tools/bench_gemm_llama.py): q/k/v
# forward 342 (ATen) vs 303 us (own NT), gate/up forward 644 vs 559 (own),
# q/k/v dgrad 367 (NN) vs 258 (NT), gate/up dgrad 542 vs 471, down dgrad 362
# vs 272 (own NT) -- ~0.4 ms per layer per micro-batch.  Large GEMMs (>= 2^34
# FLOP) therefore time their candidates once per shape on first use and keep
# the fastest.  The NT input-gradient forms need W^T: cached for good for a
# frozen weight (LoRA bases), rebuilt once per optimizer step for a trainable
# one -- whose candidates are timed with that transpose included, so they win
# only if they pay for it within one micro-batch.  DLION_GEMM_AUTOTUNE=0 keeps
# ATen's choice everywhere.
_AUTOTUNE = os.environ.get("DLION_GEMM_AUTOTUNE", "1") != "0"
_TUNE_MIN_FLOP = float(2 ** 34)
_GEMM_PICK: dict = {}  # key -> candidate name
_OWN_MARGIN = 0.05


def _own_nt_ok(a: torch.Tensor, b_nk: torch.Tensor) -> bool:
    return (a.dim() == 2 and b_nk.dim() == 2 and a.shape[1] == b_nk.shape[1] and a.shape[1] % 128 == 0
            and b_nk.shape[0] % 8 == 0 and a.stride(1) == 1 and a.stride(0) % 8 == 0 and b_nk.is_contiguous()
            and a.data_ptr() % 16 == 0 and b_nk.data_ptr() % 16 == 0 and a.shape[0] * a.stride(0) < 2 ** 31
            and b_nk.numel() < 2 ** 31)


def _nt_candidates(a: torch.Tensor, b_nk: torch.Tensor, prefix: str, bias=None) -> dict:
    """a @ b_nk^T (+ bias) implementations (bf16, a [M, K], b_nk [N, K])."""
    from . import hip

    F = torch.nn.functional
    c = {prefix + "aten": lambda: F.linear(a, b_nk, bias)}
    bias_ok = bias is None or (bias.is_contiguous() and bias.dtype == a.dtype and bias.data_ptr() % 16 == 0)
    if _own_nt_ok(a, b_nk) and bias_ok:
        c[prefix + "own"] = lambda: hip.ops().gemm_nt(a, b_nk, bias)

    def lt():
        out = torch.empty(a.shape[0], b_nk.shape[0], dtype=a.dtype, device=a.device)
        if not hip.ops().lt_gemm_nt(a, b_nk, bias, 0 if bias is None else 1, out):
            return F.linear(a, b_nk, bias)
        return out

    if a.stride(1) == 1 and b_nk.is_contiguous() and bias_ok:
        c[prefix + "lt"] = lt
    return c


def _pick(key, cands: dict, rounds: int = 3, reps: int = 3) -> str:
    """Measured-fastest candidate for ``key``, cached: ``rounds`` interleaved
    rounds of ``reps`` calls each, the best round per candidate (a single
    3-call sample let clock ramps / interference flip the choice between runs)."""
    name = _GEMM_PICK.get(key)
    if name is not None and name in cands:
        return name
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    live = {}
    for n, fn in cands.items():
        try:
            fn()  # warm-up (also tunes lt_gemm's algorithm for the shape)
            live[n] = float("inf")
        except RuntimeError:
            continue
    for _ in range(rounds):
        for n in list(live):
            try:
                ev0.record()
                for _ in range(reps):
                    cands[n]()
                ev1.record()
                ev1.synchronize()
            except RuntimeError:
                del live[n]
                continue
            live[n] = min(live[n], ev0.elapsed_time(ev1))
    # nothing ran: the first candidate (ATen) raises its own error when called
    best = min(live, key=live.get) if live else next(iter(cands))
    others = [n for n in live if not n.endswith("own")]
    if best.endswith("own") and others:
        # in the training step the own kernel does worse than its isolated timing
        # says (GPT-2's N = 768 input gradients: picked on that timing, the step
        # ran 0.3-0.5 % slower than with hipBLASLt -- profiles/r3/misc_ab.txt),
        # so it has to win by a margin
        alt = min(others, key=live.get)
        if live[best] > live[alt] * (1.0 - _OWN_MARGIN):
            best = alt
    _GEMM_PICK[key] = best
    return best


def _tunable(a: torch.Tensor, M: int, N: int, K: int) -> bool:
    from . import hip

    return (_AUTOTUNE and a.is_cuda and a.dtype == torch.bfloat16 and 2.0 * M * N * K >= _TUNE_MIN_FLOP
            and not torch.cuda.is_current_stream_capturing() and hip.available())


def gemm_fwd(x2d: torch.Tensor, w: torch.Tensor, bias=None) -> torch.Tensor:
    """x2d @ w^T (+ bias) (w [N, K], nn.Linear layout; also any NT product,
    e.g. an HF Conv1D input gradient dy @ W^T): ATen, or the measured-fastest of
    ATen / own NT / tuned hipBLASLt for large bf16 shapes."""
    M, K = x2d.shape
    N = w.shape[0]
    if not (_tunable(x2d, M, N, K) and w.dtype == torch.bfloat16 and w.dim() == 2):
        return torch.nn.functional.linear(x2d, w, bias)
    cands = _nt_candidates(x2d, w, "", bias)
    key = ("fwd", M, N, K, x2d.stride(0), w.stride(0), bias is not None)
    return cands[_pick(key, cands)]()



def _lt_nn(dy: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """dy @ w (w [N, K] row-major) through hipBLASLt's NN form with the tuned
    algorithm (csrc/lt_gemm.cpp): no W^T copy."""
    from . import hip

    out = torch.empty(dy.shape[0], w.shape[1], dtype=dy.dtype, device=dy.device)
    if not hip.ops().lt_gemm_nn(dy, w, out):
        return dy @ w
    return out


def _lt_nn_ok(dy: torch.Tensor, w: torch.Tensor) -> bool:
    return (dy.dim() == 2 and w.dim() == 2 and dy.stride(1) == 1 and dy.stride(0) % 8 == 0 and w.stride(1) == 1
            and w.stride(0) % 8 == 0 and dy.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0)


def gemm_dgrad(dy: torch.Tensor, w: torch.Tensor, frozen: bool) -> torch.Tensor:
    """dy @ w (w [N, K]): the NN product (ATen, or hipBLASLt's NN form with the
    searched algorithm), or the measured-fastest NT form against a w^T [K, N]
    (cached for good for frozen weights, rebuilt per optimizer step otherwise)."""
    M, N = dy.shape
    K = w.shape[1]
    if not (_tunable(dy, M, N, K) and w.dtype == torch.bfloat16 and w.dim() == 2):
        return dy @ w
    key = ("dgrad", M, N, K, dy.stride(0), frozen)
    name = _GEMM_PICK.get(key)
    if name == "nn":
        return dy @ w
    if name == "lt_nn":
        return _lt_nn(dy, w)
    if name is None:
        # time the NT forms with the transpose included for a trainable weight (its W^T is
        # rebuilt once per optimizer step, i.e. at most once per micro-batch)
        timed = {"nn": lambda: dy @ w}
        if _lt_nn_ok(dy, w):
            timed["lt_nn"] = lambda: _lt_nn(dy, w)
        wt_t = cached_derived(w, "t", lambda t: fast_transpose(t)) if frozen else None
        probe = _nt_candidates(dy, wt_t if frozen else fast_transpose(w), "nt_")
        for n in probe:
            timed[n] = probe[n] if frozen else (lambda n=n: _nt_candidates(dy, fast_transpose(w), "nt_")[n]())
        name = _pick(key, timed)
        if name == "nn":
            return dy @ w
        if name == "lt_nn":
            return _lt_nn(dy, w)
    wt = cached_derived(w, "t", lambda t: fast_transpose(t))  # frozen: for good; trainable: per step
    return _nt_candidates(dy, wt, "nt_")[name]()


class _LinearKN(torch.autograd.Function):
    """y = x @ W + b with W stored [K, N] (HF Conv1D layout)."""

    @staticmethod
    def forward(ctx, x2d, w, b):
        ctx.save_for_backward(x2d, w)
        ctx.has_b = b is not None
        ctx.fuse = _fuse_target(w)
        ctx.param = w if ctx.fuse else None
        ctx.fuse_b = b is not None and _fuse_target(b)
        ctx.bias = b if ctx.fuse_b else None
        if isinstance(w, torch.nn.Parameter) and x2d.dtype in (torch.bfloat16, torch.float16):
            return gemm_fwd(x2d, transposed_weight(w), b)
        return torch.addmm(b, x2d, w) if b is not None else x2d @ w

    @staticmethod
    def backward(ctx, dy):
        x2d, w = ctx.saved_tensors
        dy = dy.contiguous()
        dx = gemm_fwd(dy, w) if ctx.needs_input_grad[0] else None  # dy @ W^T, W [K, N]: an NT product
        dw = None
        if ctx.needs_input_grad[1]:
            if ctx.fuse:
                wgrad_into(x2d, dy, ctx.param)
            else:
                dw = wgrad(x2d, dy)
        db = bias_grad(dy, ctx.bias, ctx.fuse_b) if ctx.has_b and ctx.needs_input_grad[2] else None
        return dx, dw, db


class _LinearNK(torch.autograd.Function):
    """y = x @ W^T + b with W stored [N, K] (nn.Linear layout)."""

    @staticmethod
    def forward(ctx, x2d, w, b):
        ctx.save_for_backward(x2d, w)
        ctx.has_b = b is not None
        ctx.fuse = _fuse_target(w)
        ctx.param = w if ctx.fuse else None
        ctx.fuse_b = b is not None and _fuse_target(b)
        ctx.bias = b if ctx.fuse_b else None
        ctx.w = w  # the weight object itself (the W^T cache key; saved_tensors may be an alias)
        if b is None:
            return gemm_fwd(x2d, w)
        return torch.nn.functional.linear(x2d, w, b)

    @staticmethod
    def backward(ctx, dy):
        x2d, w = ctx.saved_tensors
        dy = dy.contiguous()
        dx = gemm_dgrad(dy, ctx.w, not ctx.w.requires_grad) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            if ctx.fuse:
                wgrad_into(dy, x2d, ctx.param)
            else:
                dw = wgrad(dy, x2d)
        db = bias_grad(dy, ctx.bias, ctx.fuse_b) if ctx.has_b and ctx.needs_input_grad[2] else None
        return dx, dw, db


# ------------------------------------------------- fused projections (one GEMM)
_CAT_CACHE: dict = {}  # tuple(id(w)) -> (weakrefs, key, concatenated weight)


def cat_weights(ws) -> torch.Tensor:
    """[W1; W2; ...] along the output dim, cached until any of them changes
    (in place, or via the next Lion step: see bump_weight_generation).  When
    the weights are consecutive row blocks of one buffer (pack_projections)
    the result is that buffer's view -- no copy at all."""
    import weakref

    if len(ws) == 1:
        return ws[0]
    ck = tuple(id(w) for w in ws)
    adj = _adjacent_rows([w.detach() for w in ws])
    if adj is not None:
        # one stable view object per weight set (the W^T cache is keyed by it)
        hit = _CAT_CACHE.get(ck)
        if (hit is not None and all(r() is w for r, w in zip(hit[0], ws)) and hit[1] == "adjacent"
                and hit[2].data_ptr() == adj.data_ptr() and hit[2].shape == adj.shape):
            return hit[2]
        if hit is None:
            weakref.finalize(ws[0], _CAT_CACHE.pop, ck, None)
        _CAT_CACHE[ck] = ([weakref.ref(w) for w in ws], "adjacent", adj)
        return adj
    # the optimizer's kernels write trainable weights through raw pointers (no
    # _version bump): those are re-concatenated after every step; frozen ones
    # (LoRA base weights, a DPO reference model) stay cached -- the re-cat of a
    # Llama-2-7B layer's q/k/v + gate/up weights was ~2.7 % of a LoRA SFT step
    gen = _WEIGHT_GEN[0] if any(w.requires_grad for w in ws) else -1
    key = (gen,) + tuple((w._version, w.data_ptr()) for w in ws)
    hit = _CAT_CACHE.get(ck)
    same = hit is not None and all(r() is w for r, w in zip(hit[0], ws))
    if same and hit[1] == key:
        return hit[2]
    with torch.no_grad():
        old = hit[2] if same and hit[1] != "adjacent" else None
        if (old is not None and old.dtype == ws[0].dtype and old.shape[0] == sum(w.shape[0] for w in ws)
                and old.shape[1:] == ws[0].shape[1:]):
            # refreshed in place after an optimizer step (trainable Llama q/k/v, gate/up):
            # one contiguous device copy per weight into the kept buffer -- no reallocation, and
            # ~2x the rate of the cat kernel (Llama-3-8B: 64 cats per step, ~6.6 ms)
            off = 0
            for w in ws:
                old[off:off + w.shape[0]].copy_(w.detach())
                off += w.shape[0]
            _CAT_CACHE[ck] = (hit[0], key, old)
            return old
        out = torch.cat([w.detach() for w in ws], 0)
    if hit is None:
        weakref.finalize(ws[0], _CAT_CACHE.pop, ck, None)
    _CAT_CACHE[ck] = ([weakref.ref(w) for w in ws], key, out)
    return out


def _adjacent_views(ts):
    """If ts are consecutive column blocks of one row-major buffer (e.g. the
    fused SwiGLU backward's [dgate | dup]), return that [..., sum n] view."""
    t0 = ts[0]
    if any(t is None for t in ts) or t0.dim() < 2 or t0.stride(-1) != 1:
        return None
    n = sum(t.shape[-1] for t in ts)
    off = 0
    for t in ts:
        if (t.shape[:-1] != t0.shape[:-1] or t.stride() != t0.stride() or t.dtype != t0.dtype
                or t.data_ptr() != t0.data_ptr() + off * t0.element_size()
                or t.untyped_storage().data_ptr() != t0.untyped_storage().data_ptr()):
            return None
        off += t.shape[-1]
    if t0.stride(-2) != n:
        return None
    return t0.as_strided(t0.shape[:-1] + (n,), t0.stride())


class _LinearMultiNK(torch.autograd.Function):
    """[y1 | y2 | ...] = x @ [W1; W2; ...]^T as ONE GEMM for projections that
    share their input (Llama q/k/v, gate/up); the outputs are column views of
    the fused result.  Backward: one input-gradient GEMM on the concatenated
    output gradient (zero-copy when the consumers wrote it as one buffer) and
    one weight-gradient GEMM whose row blocks are the per-weight gradients.
    Measured at Llama-3-8B shapes (tools/bench_fused_proj.py): q/k/v fwd+dgrad+
    wgrad 1155 -> 958 us, gate/up 4590 -> 4242 us per layer -- the k/v
    projections alone (1024 outputs) fill only half of the 256 CUs."""

    @staticmethod
    def forward(ctx, x2d, *ws):
        sizes = [w.shape[0] for w in ws]
        y = gemm_fwd(x2d, cat_weights(ws))
        ctx.save_for_backward(x2d, *ws)
        ctx.ws = ws  # the weight objects (cat / W^T cache keys; saved_tensors may be aliases)
        ctx.sizes = sizes
        ctx.fuse = [_fuse_target(w) for w in ws]
        ctx.params = [w if f else None for w, f in zip(ws, ctx.fuse)]
        return tuple(y.split(sizes, dim=-1))

    @staticmethod
    def backward(ctx, *grads):
        x2d, *ws = ctx.saved_tensors
        grads = [torch.zeros(x2d.shape[0], n, dtype=x2d.dtype, device=x2d.device) if g is None else g
                 for g, n in zip(grads, ctx.sizes)]
        dy = _adjacent_views(grads)
        if dy is None:
            dy = torch.cat([g.reshape(-1, g.shape[-1]) for g in grads], -1)
        dy = dy.reshape(-1, dy.shape[-1])
        dx = None
        if ctx.needs_input_grad[0]:
            dx = gemm_dgrad(dy, cat_weights(ctx.ws), not any(w.requires_grad for w in ctx.ws))
        dws = [None] * len(ws)
        want = [ctx.needs_input_grad[1 + i] for i in range(len(ws))]
        if any(want):
            if all(ctx.fuse) and all(want):
                _multi_wgrad_into(dy, x2d, ctx.params, ctx.sizes)
            else:
                dwc = wgrad(dy, x2d)  # [sum n, K]; its row blocks are contiguous
                off = 0
                for i, n in enumerate(ctx.sizes):
                    if want[i]:
                        blk = dwc[off:off + n]
                        if ctx.fuse[i]:
                            p = ctx.params[i]
                            p.grad = blk if p.grad is None else p.grad.add_(blk)
                        else:
                            dws[i] = blk
                    off += n
        return (dx, *dws)


def _multi_wgrad_into(dy, x2d, params, sizes) -> None:
    """params[i].grad (+)= (dy[:, block i])^T x2d for every block, one GEMM."""
    M, N = dy.shape
    K = x2d.shape[1]
    s, own = wgrad_splits(dy, x2d)
    if (s > 1 or own) and (N * K) % 4 == 0 and (own or M % s == 0):
        from . import hip

        if hip.available():
            cols, off = [], 0
            for n in sizes:
                cols.append((off * K, n * K))
                off += n
            bf = all(p.dtype == torch.bfloat16 for p in params)
            gs = [p.grad for p in params]
            base = _adjacent_rows(gs) if all(g is not None for g in gs) else None
            timed = (bf and _direct_split_pick(dy, x2d, s, own)
                     and (all(g is None for g in gs) or (base is not None and base.is_contiguous())))
            if _ST.fuse["on"] and not timed and ((own and _defer_wgrad(list(params), cols, dy, x2d, s))
                                                 or _acc_gemm(list(params), cols, dy, x2d, s)):
                return  # reduced into each params[i].grad when the window closes
            if own and (s == 1 or timed) and bf:
                gs = [p.grad for p in params]
                if all(g is None for g in gs):  # one buffer; each grad is a row block of it
                    buf = torch.empty(N, K, dtype=torch.bfloat16, device=dy.device)
                    _unsplit_wgrad(dy, x2d, buf, False, s)
                    off = 0
                    for p, n in zip(params, sizes):
                        p.grad = buf[off:off + n].view_as(p)
                        off += n
                    return
                base = _adjacent_rows(gs) if all(g is not None for g in gs) else None
                if base is not None and base.dtype == torch.bfloat16 and base.is_contiguous():
                    _unsplit_wgrad(dy, x2d, base, True, s)
                    return
            flat = wgrad_partials(dy, x2d, s).view(s, N * K)
            off = 0
            for p, n in zip(params, sizes):
                deposit_grad(p, flat[:, off * K:(off + n) * K])
                off += n
            return
    gs = [p.grad for p in params]
    base = _adjacent_rows(gs) if all(g is not None for g in gs) else None
    if base is not None:  # every grad is a row block of one buffer (the first micro-batch made it)
        base.addmm_(dy.t(), x2d)
        return
    dwc = dy.t() @ x2d
    off = 0
    for p, n in zip(params, sizes):
        blk = dwc[off:off + n]
        p.grad = blk if p.grad is None else p.grad.add_(blk)
        off += n


def _adjacent_rows(ts):
    t0 = ts[0]
    if not all(t.is_contiguous() and t.dtype == t0.dtype and t.shape[1:] == t0.shape[1:] for t in ts):
        return None
    off = 0
    for t in ts:
        if (t.data_ptr() != t0.data_ptr() + off * t0.stride(0) * t0.element_size()
                or t.untyped_storage().data_ptr() != t0.untyped_storage().data_ptr()):
            return None
        off += t.shape[0]
    return t0.as_strided((off,) + tuple(t0.shape[1:]), t0.stride())


_PACK_PROJ = os.environ.get("DLION_PACK_PROJ", "1") != "0"  # A/B switch for pack_projections


def pack_projections(ws) -> bool:
    """Re-point trainable weights that one fused GEMM uses together (Llama
    q/k/v, gate/up) at consecutive row blocks of ONE buffer, so that their
    concatenation is a view instead of a per-step copy (Llama-3-8B: 64 copies,
    ~3.5 ms per step).  Done once, on first fused use on the GPU (after
    `.to(device)`; a later `.to()` that moves them apart just brings the copy
    back).  Safe for the optimizers (the Lion pointer tables follow data_ptr,
    others hold the Parameter objects), for load_state_dict (copies in place)
    and for save_pretrained (disjoint views of one storage are cloned on save).
    Returns True when the weights are (now) adjacent."""
    if _adjacent_rows([w.detach() for w in ws]) is not None:
        return True
    if torch.is_inference_mode_enabled():  # the new buffer would be an inference tensor, unusable for training
        return False
    if not (_PACK_PROJ and len(ws) > 1 and all(isinstance(w, torch.nn.Parameter) and w.requires_grad and w.is_cuda
                                                and w.is_contiguous() for w in ws)
            and len({(w.dtype, w.device, tuple(w.shape[1:])) for w in ws}) == 1):
        return False
    with torch.no_grad():
        buf = torch.cat([w.detach() for w in ws], 0)
        off = 0
        for w in ws:
            w.data = buf[off:off + w.shape[0]]
            off += w.shape[0]
    return True


def linear_multi_nk(x: torch.Tensor, ws) -> tuple:
    """(x @ W1^T, x @ W2^T, ...) for nn.Linear-layout weights sharing the input
    x, as one fused GEMM (CUDA) -- outputs are column views of one buffer."""
    x2d = x.reshape(-1, x.shape[-1])
    lead = x.shape[:-1]
    if not x.is_cuda:
        return tuple(torch.nn.functional.linear(x2d, w).view(lead + (w.shape[0],)) for w in ws)
    pack_projections(ws)
    x2d, *ws = autocast_inputs(x2d, *ws)
    with torch.autocast("cuda", enabled=False):
        outs = _LinearMultiNK.apply(x2d, *ws)
    return tuple(o.view(lead + (o.shape[-1],)) for o in outs)


def autocast_inputs(*ts):
    """Under autocast (HF ``--bf16``/``--fp16``), cast the floating inputs of a
    custom op to the autocast dtype with differentiable casts, so the op itself
    runs with autocast disabled and sees one dtype (e.g. LayerNorm outputs are
    fp32 under autocast while the GEMM computes in bf16)."""
    if not torch.is_autocast_enabled("cuda"):
        return ts
    dt = torch.get_autocast_dtype("cuda")
    return tuple(t.to(dt) if t is not None and t.is_floating_point() and t.dtype != dt else t for t in ts)


def linear_kn(x: torch.Tensor, w: torch.Tensor, b=None) -> torch.Tensor:
    shp = x.shape[:-1] + (w.shape[1],)
    x2d = x.reshape(-1, x.shape[-1])
    if not x.is_cuda:
        y = torch.addmm(b, x2d, w) if b is not None else x2d @ w
    else:
        x2d, w, b = autocast_inputs(x2d, w, b)
        with torch.autocast("cuda", enabled=False):
            y = _LinearKN.apply(x2d, w, b)
    return y.view(shp)


def linear_nk(x: torch.Tensor, w: torch.Tensor, b=None) -> torch.Tensor:
    shp = x.shape[:-1] + (w.shape[0],)
    x2d = x.reshape(-1, x.shape[-1])
    if not x.is_cuda:
        y = torch.nn.functional.linear(x2d, w, b)
    else:
        x2d, w, b = autocast_inputs(x2d, w, b)
        with torch.autocast("cuda", enabled=False):
            y = _LinearNK.apply(x2d, w, b)
    return y.view(shp)
