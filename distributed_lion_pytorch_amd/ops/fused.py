"""Fused model ops with a gfx950 fast path and a PyTorch fallback.

Every function here is the single entry point the native models use; the
implementation is chosen per call:

* on a GPU tensor the hand-written HIP kernels from ``_dlion_C.so`` run (the
  extension is *required* on a GPU box -- see ops/hip.py);
* on CPU tensors (unit tests, gloo runs) a plain PyTorch composition with the
  same semantics runs.

``set_impl("torch")`` forces the PyTorch path everywhere (A/B benchmarks).
"""
from __future__ import annotations



import torch
import torch.nn.functional as F

from . import hip
from .linear import gemm_fwd

_IMPL = {"mode": "auto"}  # auto | torch | hip (set_impl)


def set_impl(mode: str) -> None:
    if mode not in ("auto", "torch", "hip"):
        raise ValueError(mode)
    _IMPL["mode"] = mode


def get_impl() -> str:
    return _IMPL["mode"]


def _use_hip(t: torch.Tensor) -> bool:
    mode = _IMPL["mode"]
    if mode == "torch" or not t.is_cuda:
        return False
    if mode == "hip" or not hip.fallback_allowed():
        hip.require()
        return True
    return hip.available()


# ---------------------------------------------------------------- layer norm
def layer_norm(x: torch.Tensor, ln: torch.nn.LayerNorm) -> torch.Tensor:
    return F.layer_norm(x, ln.normalized_shape, ln.weight, ln.bias, ln.eps)


def rms_norm(x: torch.Tensor, weight: torch.Tensor, eps: float) -> torch.Tensor:
    """Llama RMSNorm (HF semantics: normalise in fp32, cast back, then scale)."""
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return weight * y.to(x.dtype)


# ---------------------------------------------------------- rotary / SwiGLU
def rope_reference(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """x [B, T, H, D]; cos/sin [T, D]; HF rotate-half convention (ATen chain)."""
    d2 = x.shape[-1] // 2
    x1, x2 = x[..., :d2], x[..., d2:]
    rot = torch.cat([-x2, x1], dim=-1)
    T = x.shape[1]
    return x * cos[None, :T, None, :] + rot * sin[None, :T, None, :]


class _Rope(torch.autograd.Function):
    """One gfx950 kernel each way (csrc/elementwise_kernels.hip rope_kernel);
    the backward is the inverse rotation."""

    @staticmethod
    def forward(ctx, x, cos, sin):
        ctx.save_for_backward(cos, sin)
        return hip.ops().rope(x, cos, sin, False)

    @staticmethod
    def backward(ctx, dy):
        cos, sin = ctx.saved_tensors
        return hip.ops().rope(dy.contiguous(), cos, sin, True), None, None


def _token_strided_ok(x: torch.Tensor) -> bool:
    """[B, T, H, D] with contiguous heads and one 16-byte aligned token stride
    (a q / k column slice of a fused projection output): the kernel reads it
    in place."""
    B, T, H, D = x.shape
    return (x.stride(3) == 1 and x.stride(2) == D and (B == 1 or x.stride(0) == T * x.stride(1))
            and x.stride(1) % 8 == 0 and x.data_ptr() % 16 == 0)


def rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """x [B, T, H, D]; cos/sin [>=T, D]; HF rotate-half convention."""
    if (x.dtype == torch.bfloat16 and cos.dtype == torch.bfloat16 and sin.dtype == torch.bfloat16
            and x.shape[-1] % 8 == 0 and _use_hip(x)):
        if not _token_strided_ok(x):
            x = x.contiguous()
        with torch.autocast("cuda", enabled=False):
            return _Rope.apply(x, cos.contiguous(), sin.contiguous())
    return rope_reference(x, cos, sin)


class _SwiGLU(torch.autograd.Function):
    """gate / up may be the two column halves of one fused projection output
    (row stride 2F): read in place, and the backward then writes [dgate | dup]
    as one buffer, which the fused projection's backward takes without a copy."""

    @staticmethod
    def forward(ctx, gate, up, want_t):
        from . import linear

        ctx.save_for_backward(gate, up)
        F_ = gate.shape[-1]
        rows = gate.numel() // F_
        if want_t and rows % 64 == 0 and F_ % 64 == 0 and linear.want_transposed_copy(rows, F_, "b"):
            # the down projection's weight gradient runs on token-contiguous copies: write h^T now
            h, ht = hip.ops().swiglu_fwd_t(gate, up)
            linear.register_transposed(h.view(rows, F_), ht)
            return h
        return hip.ops().swiglu_fwd(gate, up)

    @staticmethod
    def backward(ctx, dh):
        gate, up = ctx.saved_tensors
        F_ = gate.shape[-1]
        if (gate.stride(-2) == 2 * F_ and up.data_ptr() == gate.data_ptr() + F_ * gate.element_size()
                and up.stride() == gate.stride()):
            from . import linear

            rows = gate.numel() // F_
            if rows % 64 == 0 and F_ % 64 == 0 and linear.want_transposed_copy(rows, 2 * F_):
                # the gate/up weight gradient runs on token-contiguous copies: write dgu^T here
                dgu, dgut = hip.ops().swiglu_bwd_fused_t(dh.contiguous(), gate, up)
                linear.register_transposed(dgu.view(rows, 2 * F_), dgut)
            else:
                dgu = hip.ops().swiglu_bwd_fused(dh.contiguous(), gate, up)
            return dgu[..., :F_], dgu[..., F_:], None
        dg, du = hip.ops().swiglu_bwd(dh.contiguous(), gate, up)
        return dg, du, None


def swiglu(gate: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    """silu(gate) * up (Llama MLP); one fused kernel each way on the GPU."""
    if gate.is_cuda:
        from .linear import autocast_inputs

        gate, up = autocast_inputs(gate, up)
    if (gate.dtype == torch.bfloat16 and up.dtype == torch.bfloat16 and gate.shape == up.shape
            and gate.shape[-1] % 8 == 0 and _use_hip(gate)):
        if not (_rows_ok(gate) and up.stride() == gate.stride()):
            gate, up = gate.contiguous(), up.contiguous()
        # h^T is written only when a backward will consume it: never under
        # no_grad (a frozen reference model's forward) or for frozen inputs
        want_t = torch.is_grad_enabled() and (gate.requires_grad or up.requires_grad)
        with torch.autocast("cuda", enabled=False):
            return _SwiGLU.apply(gate, up, want_t)
    return F.silu(gate) * up


def _rows_ok(t: torch.Tensor) -> bool:
    """[..., F] whose leading dims collapse to rows of one 16-byte aligned stride."""
    if t.dim() < 2 or t.stride(-1) != 1 or t.stride(-2) % 8 or t.data_ptr() % 16:
        return False
    return all(t.shape[i] == 1 or t.stride(i) == t.stride(i + 1) * t.shape[i + 1] for i in range(t.dim() - 2))


# ------------------------------------------------------------- dropout + add
def dropout_add(y: torch.Tensor, residual: torch.Tensor, p: float) -> torch.Tensor:
    if p > 0.0:
        y = F.dropout(y, p, True)
    return residual + y


# --------------------------------------- fused residual + dropout + LN / RMSNorm
_NORM_BWD_ROWS = 4  # rows per backward block-iteration for C <= 1024 (csrc/norm_kernels.hip RowGroup)
_NORM_PARTS_CAP = 512


def _norm_parts(rows: int, C: int) -> int:
    # blocks of 4 waves, one fp32 partial row triple per block: enough waves to
    # cover the CUs a few times over while the partial stack stays a small
    # fraction of the row traffic (tools/bench_norm.py: 512 best at 20480x768).
    # C <= 1024: 4 rows per block-iteration, wider: 1 (4-wave rows)
    rows_per_iter = _NORM_BWD_ROWS if C <= 1024 else 1
    return max(1, min(_NORM_PARTS_CAP, rows // (4 * rows_per_iter)))


def _sum_rows(part: torch.Tensor) -> torch.Tensor:
    """[P, ...] fp32 partials -> bf16 sums in one kernel (row-parallel for tall stacks)."""
    return hip.ops().sum_partials(part)


def _fused_params(*params):
    """Which of (gamma, beta, bias) get their gradient deposited in place
    (gradient-accumulation fusion, ops/linear.py); None entries are not fused."""
    from .linear import _fuse_target

    return tuple(p if p is not None and _fuse_target(p) else None for p in params)


def _param_grads(part2d, C, fused, present):
    """(dgamma, dbeta, dbias) from the [S, 3C] partials: fused parameters get
    their .grad accumulated in place (returned as None), the rest come back as
    bf16 gradients."""
    from .linear import deposit_grad

    out = [None, None, None]
    need = [i for i in range(3) if present[i] and fused[i] is None]
    if len(need) == 3 or (len(need) >= 1 and all(f is None for f in fused)):
        sums = _sum_rows(part2d)
        for i in need:
            out[i] = sums[i * C:(i + 1) * C]
    else:
        for i in need:
            out[i] = _sum_rows(part2d[:, i * C:(i + 1) * C])
    dep = [i for i in range(3) if present[i] and fused[i] is not None]
    if len(dep) > 1 and dep == list(range(dep[0], dep[0] + len(dep))):
        from .linear import defer_partials

        params = [fused[i] for i in dep]
        sub = part2d[:, dep[0] * C:(dep[-1] + 1) * C]
        if defer_partials(("joint",) + tuple(id(p) for p in params), sub,
                          lambda pc: _deposit_joint_or_each(params, pc, C)):
            return tuple(out)
        if _deposit_joint(params, sub, C):
            return tuple(out)
    for i in dep:
        deposit_grad(fused[i], part2d[:, i * C:(i + 1) * C])
    return tuple(out)


def _deposit_joint_or_each(params, part2d, C) -> None:
    from .linear import deposit_grad

    if not _deposit_joint(params, part2d, C):
        for j, p in enumerate(params):
            deposit_grad(p, part2d[:, j * C:(j + 1) * C], defer=False)


def _deposit_joint(params, part2d, C) -> bool:
    """(gamma, beta, bias).grad (+)= column sums of their adjacent partial
    blocks in ONE reduction launch: the gradients live as consecutive views of
    one buffer (allocated that way on the step's first deposit).  GPT-2 has 25
    such boundaries per micro-batch: 50 fewer ~9 us launches."""
    gs = [p.grad for p in params]
    if all(g is None for g in gs):
        from .linear import sum_partials_into

        buf = sum_partials_into(part2d)  # bf16 [k*C], fresh
        for j, p in enumerate(params):
            p.grad = buf[j * C:(j + 1) * C].view_as(p)
        return True
    if any(g is None or not g.is_contiguous() or g.dtype != params[0].dtype for g in gs):
        return False
    g0 = gs[0]
    for j, g in enumerate(gs):
        if (g.data_ptr() != g0.data_ptr() + j * C * g0.element_size()
                or g.untyped_storage().data_ptr() != g0.untyped_storage().data_ptr()):
            return False
    from .linear import sum_partials_into

    sum_partials_into(part2d, g0.as_strided((len(gs) * C,), (1,)), accumulate=True)
    return True


class _AddNorm(torch.autograd.Function):
    """(xo, h) = (x + dropout(y + bias), Norm(xo)) in one gfx950 kernel each way;
    gamma / beta / bias gradients come out of the backward kernel as partials."""

    @staticmethod
    def forward(ctx, y, x, bias, gamma, beta, eps, rms, p, seed):
        xo, h, mean, rstd = hip.ops().add_norm_fwd(x, y, bias, gamma, beta, eps, rms, p, seed)
        ctx.save_for_backward(xo, gamma, mean, rstd)
        ctx.rms, ctx.p, ctx.seed = rms, p, seed
        ctx.has_beta, ctx.has_bias = beta is not None, bias is not None
        ctx.fused_params = _fused_params(gamma, beta, bias)
        return xo, h

    @staticmethod
    def backward(ctx, dxo, dh):
        xo, gamma, mean, rstd = ctx.saved_tensors
        C = xo.shape[-1]
        rows = xo.numel() // C
        if dh is None:
            dh = torch.zeros_like(xo)
        parts = _norm_parts(rows, C)
        need = ctx.needs_input_grad
        # without dropout (Llama) and with no bias gradient to sum, the branch gradient IS the
        # residual one: return dx for both instead of writing an identical copy (one stream of
        # the backward's five; autograd aliases grads the same way for an add)
        alias = ctx.p == 0.0 and not (ctx.has_bias and need[2])
        dx, dy, part = hip.ops().add_norm_bwd(dh.contiguous(), None if dxo is None else dxo.contiguous(), xo, gamma,
                                              mean, rstd, ctx.rms, ctx.p, ctx.seed, not alias, parts)
        if alias:
            dy = dx
        dgamma, dbeta, dbias = _param_grads(part.view(-1, 3 * C), C, ctx.fused_params,
                                            (need[3], ctx.has_beta and need[4], ctx.has_bias and need[2]))
        return dy, dx, dbias, dgamma, dbeta, None, None, None, None


class _Norm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, eps, rms):
        _, h, mean, rstd = hip.ops().add_norm_fwd(x, None, None, gamma, beta, eps, rms, 0.0, 0)
        ctx.save_for_backward(x, gamma, mean, rstd)
        ctx.rms, ctx.has_beta = rms, beta is not None
        ctx.fused_params = _fused_params(gamma, beta, None)
        return h

    @staticmethod
    def backward(ctx, dh):
        x, gamma, mean, rstd = ctx.saved_tensors
        C = x.shape[-1]
        parts = _norm_parts(x.numel() // C, C)
        dx, _, part = hip.ops().add_norm_bwd(dh.contiguous(), None, x, gamma, mean, rstd, ctx.rms, 0.0, 0, False,
                                             parts)
        need = ctx.needs_input_grad
        dgamma, dbeta, _ = _param_grads(part.view(-1, 3 * C), C, ctx.fused_params,
                                        (need[1], ctx.has_beta and need[2], False))
        return dx, dgamma, dbeta, None, None


NORM_WIDTHS = (256, 512, 768, 1024, 2048, 3072, 4096, 5120, 6144, 8192)  # csrc/norm_kernels.hip NORM_DISPATCH


def _norm_ok(x: torch.Tensor, gamma: torch.Tensor) -> bool:
    # the kernels hold a whole row in registers: one wave per row up to 1024,
    # one 4-wave block per row for the Llama widths
    return (x.dtype == torch.bfloat16 and gamma.dtype == torch.bfloat16 and x.shape[-1] in NORM_WIDTHS
            and _use_hip(x))


def dropout_add_norm(y: torch.Tensor, x: torch.Tensor, gamma: torch.Tensor, beta, eps: float, p: float,
                     rms: bool = False, bias=None):
    """Returns (x + dropout(y + bias), Norm(...)) -- the residual stream and the
    next sub-block's normalised input."""
    if y.is_cuda:
        from .linear import autocast_inputs

        y, x, bias = autocast_inputs(y, x, bias)
    if _norm_ok(x, gamma) and y.dtype == x.dtype and (bias is None or bias.dtype == x.dtype):
        with torch.autocast("cuda", enabled=False):
            return _AddNorm.apply(y.contiguous(), x.contiguous(), bias, gamma, beta, float(eps), bool(rms),
                                  float(p), _new_seed())
    if bias is not None:
        y = y + bias
    xo = dropout_add(y, x, p)
    if rms:
        return xo, rms_norm(xo, gamma, eps)
    return xo, F.layer_norm(xo, (x.shape[-1],), gamma, beta, eps)


class _BiasGelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, b, exact):
        ctx.save_for_backward(z, b)
        ctx.exact = exact
        ctx.fused_b = _fused_params(b)[0]
        return hip.ops().bias_gelu_fwd(z, b, exact)

    @staticmethod
    def backward(ctx, dh):
        z, b = ctx.saved_tensors
        rows = z.numel() // z.shape[-1]
        parts = max(1, min(1024, rows // 8))  # tools/bench_norm.py sweep: 1024 best at GPT-2 shape
        dz, part = hip.ops().bias_gelu_bwd(dh.contiguous(), z, b, ctx.exact, parts)
        if ctx.fused_b is not None:
            from .linear import deposit_grad

            deposit_grad(ctx.fused_b, part)
            return dz, None, None
        return dz, _sum_rows(part), None


def bias_gelu(z: torch.Tensor, b: torch.Tensor, exact: bool = False) -> torch.Tensor:
    """gelu(z + b) (tanh approximation unless exact); fused kernel on the GPU."""
    if z.is_cuda:
        from .linear import autocast_inputs

        z, b = autocast_inputs(z, b)
        if z.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and z.shape[-1] % 8 == 0 and _use_hip(z):
            with torch.autocast("cuda", enabled=False):
                return _BiasGelu.apply(z.contiguous(), b, bool(exact))
    return F.gelu(z + b, approximate="none" if exact else "tanh")


def norm(x: torch.Tensor, gamma: torch.Tensor, beta, eps: float, rms: bool = False) -> torch.Tensor:
    if _norm_ok(x, gamma):
        with torch.autocast("cuda", enabled=False):
            return _Norm.apply(x.contiguous(), gamma, beta, float(eps), bool(rms))
    if rms:
        return rms_norm(x, gamma, eps)
    return F.layer_norm(x, (x.shape[-1],), gamma, beta, eps)


def norm_dropout_keep(rows: int, C: int, p: float, seed: int, device=None) -> torch.Tensor:
    """bool keep-mask [rows, C] exactly as norm_kernels.hip draws it."""
    th = min(65535, int(round(p * 65536)))
    idx = torch.arange(rows * C, device=device, dtype=torch.int64)
    x = (seed & _M32) ^ (((idx >> 1) * 0x9E3779B1) & _M32) ^ ((idx >> 33) & _M32)
    u16 = (_lowbias32(x) >> ((idx & 1) * 16)) & 0xFFFF
    return (u16 >= th).view(rows, C)


# --------------------------------------------------------------- bias + GELU
def linear_gelu(x2d: torch.Tensor, w_in_out: torch.Tensor, bias: torch.Tensor, exact: bool = False):
    """gelu(x @ W + b) with HF Conv1D's [in, out] weight layout.  Training: GEMM
    without bias, then one bias+GELU kernel whose backward also yields the
    bias grad.  Without autograd (evaluation, frozen models): one hipBLASLt
    GEMM with the bias+GELU epilogue (csrc/lt_gemm.cpp; tanh GELU only)."""
    from .linear import autocast_inputs, linear_kn, transposed_weight

    if (not exact and not torch.is_grad_enabled() and x2d.is_cuda and _use_hip(x2d)
            and x2d.dim() == 2 and x2d.stride(1) == 1 and x2d.stride(0) % 8 == 0):
        xa, wa, ba = autocast_inputs(x2d, w_in_out, bias)
        if xa.dtype == wa.dtype == ba.dtype == torch.bfloat16 and ba.is_contiguous() and xa.data_ptr() % 16 == 0:
            wt = transposed_weight(wa)  # [out, in], cached until the next optimizer step
            out = torch.empty(xa.shape[0], wt.shape[0], dtype=xa.dtype, device=xa.device)
            if hip.ops().lt_gemm_nt(xa, wt, ba, 2, out):
                return out
    return bias_gelu(linear_kn(x2d, w_in_out, None), bias, exact)


# unfused paths kept as test references (tests/test_dgelu_gpu.py toggles these)
_DGELU_FUSED = True  # DGELU backward in the own NT GEMM's epilogue
_GELU_FUSED = True  # bias + GELU forward in the own NT GEMM's epilogue
_GELU_DSTORE = True  # store gelu'(z) instead of z


def _own_gemm_ok(a: torch.Tensor, b_nk: torch.Tensor) -> bool:
    """Shapes the own NT GEMM (csrc/gemm.hip) takes: a [M, K], b [N, K]."""
    return (a.dim() == 2 and b_nk.dim() == 2 and a.shape[1] == b_nk.shape[1] and a.shape[1] % 128 == 0
            and b_nk.shape[0] % 8 == 0 and a.stride(1) == 1 and a.stride(0) % 8 == 0 and b_nk.is_contiguous()
            and a.data_ptr() % 16 == 0 and a.shape[0] * a.stride(0) < 2 ** 31)


class _MLP(torch.autograd.Function):
    """y = gelu(x @ Wfc + b) @ Wproj for the GPT-2 MLP (both weights in HF
    Conv1D [in, out] layout, no output bias: the caller's residual+norm kernel
    adds it).  Measured at the bench shape (20480 tokens, C 768, 4C 3072;
    tools/bench_dgelu.py), per layer:

    * forward: the own NT GEMM with the bias+GELU epilogue writes h and the
      pre-activation z in one pass -- 129 us against hipBLASLt + the separate
      bias+GELU kernel's 140 us;
    * backward: the down-projection's input gradient and the bias+GELU
      backward are ONE kernel -- the own GEMM's DGELU epilogue rounds
      g = dy . Wproj^T to bf16 like the unfused GEMM, multiplies by gelu'(z+b)
      in its drain and emits per-wave column sums for the bias gradient
      (144 us against hipBLASLt + bias_gelu_bwd's 177 us).

    Weight gradients are split-K GEMMs deposited straight into .grad inside a
    gradient-accumulation fusion window (ops/linear.py), like every linear."""

    @staticmethod
    def forward(ctx, x, w_fc, b_fc, w_proj, exact):
        from .linear import _fuse_target, transposed_weight

        wfc_t = transposed_weight(w_fc) if isinstance(w_fc, torch.nn.Parameter) else w_fc.t().contiguous()
        # the backward's fused DGELU GEMM will run (dy [M, C] against w_proj [4C, C]):
        # store gelu'(z + b) instead of z (EPI 6/7 -> EPI 8, one multiply per element
        # in the backward drain instead of a GELU derivative)
        bwd_own = (_DGELU_FUSED and w_proj.is_contiguous() and w_proj.shape[1] % 128 == 0
                   and w_proj.shape[0] % 8 == 0 and x.shape[0] * w_proj.shape[1] < 2 ** 31)
        ctx.dstored = False
        if _GELU_FUSED and _own_gemm_ok(x, wfc_t):
            if bwd_own and _GELU_DSTORE:
                h, z = hip.ops().gemm_nt_gelu_d(x, wfc_t, b_fc, exact)  # z <- gelu'(z + b)
                ctx.dstored = True
            else:
                h, z = hip.ops().gemm_nt_gelu(x, wfc_t, b_fc, exact)
        else:
            z = F.linear(x, wfc_t)
            h = hip.ops().bias_gelu_fwd(z, b_fc, exact)
        ctx.save_for_backward(x, z, h, w_fc, b_fc, w_proj)
        ctx.exact = exact
        ctx.fuse = (_fuse_target(w_fc), _fuse_target(w_proj))
        # deposit targets: the Parameter objects themselves -- under non-reentrant
        # activation checkpointing ctx.saved_tensors hands back recomputed
        # aliases, and a .grad set on an alias is lost
        ctx.wparams = (w_fc, w_proj)
        ctx.fused_b = _fused_params(b_fc)[0]
        wp_t = transposed_weight(w_proj) if isinstance(w_proj, torch.nn.Parameter) else w_proj.t()
        return gemm_fwd(h, wp_t)

    @staticmethod
    def backward(ctx, dy):
        from .linear import deposit_grad, wgrad, wgrad_into

        x, z, h, w_fc, b_fc, w_proj = ctx.saved_tensors
        dy = dy.contiguous()
        if ctx.dstored:  # z holds gelu'(z + b)
            assert _own_gemm_ok(dy, w_proj)
            dz, part = hip.ops().gemm_nt_dmul(dy, w_proj, z)
        elif _DGELU_FUSED and _own_gemm_ok(dy, w_proj):
            dz, part = hip.ops().gemm_nt_dgelu(dy, w_proj, b_fc, z, ctx.exact)
        else:
            dz, part = hip.ops().bias_gelu_bwd(dy @ w_proj.t(), z, b_fc, ctx.exact, max(1, min(1024, z.shape[0] // 8)))
        grads = [None] * 5
        if ctx.needs_input_grad[0]:
            grads[0] = gemm_fwd(dz, w_fc)  # dx = dz . Wfc^T, Wfc stored [C, 4C]
        for i, (w, a, g) in ((1, (ctx.wparams[0], x, dz)), (3, (ctx.wparams[1], h, dy))):
            if ctx.needs_input_grad[i]:
                if ctx.fuse[(i - 1) // 2]:
                    wgrad_into(a, g, w)
                else:
                    grads[i] = wgrad(a, g)
        if ctx.needs_input_grad[2]:
            if ctx.fused_b is not None:
                deposit_grad(ctx.fused_b, part)
            else:
                grads[2] = _sum_rows(part)
        return tuple(grads)


def mlp_gelu(x: torch.Tensor, w_fc: torch.Tensor, b_fc: torch.Tensor, w_proj: torch.Tensor,
             exact: bool = False) -> torch.Tensor:
    """gelu(x @ Wfc + b) @ Wproj (weights stored [in, out]) with the fused
    GEMM epilogues of :class:`_MLP`; plain PyTorch off the GPU path."""
    shp = x.shape[:-1] + (w_proj.shape[1],)
    x2 = x.reshape(-1, x.shape[-1])
    if x2.is_cuda and _use_hip(x2):
        from .linear import autocast_inputs

        x2, w_fc, b_fc, w_proj = autocast_inputs(x2, w_fc, b_fc, w_proj)
        if (x2.dtype == w_fc.dtype == b_fc.dtype == w_proj.dtype == torch.bfloat16 and w_fc.shape[1] % 8 == 0
                and b_fc.is_contiguous() and w_fc.is_contiguous() and w_proj.is_contiguous()):
            with torch.autocast("cuda", enabled=False):
                return _MLP.apply(x2.contiguous(), w_fc, b_fc, w_proj, bool(exact)).view(shp)
    h = F.gelu(x2 @ w_fc + b_fc, approximate="none" if exact else "tanh")
    return (h @ w_proj).view(shp)


# ------------------------------------------------------------ index errors
# Out-of-range token ids / labels are an error, as in ATen's embedding and
# cross-entropy, not a silent clamp: the embedding kernel and a label check
# OR a bit into a per-device int32 flag, which check_index_errors() reads
# once per optimizer step without stalling the stream (one step late) or, at
# the end of a run, synchronously.
_IDX_EMBED, _IDX_LABEL = 1, 2
_IDX_FLAGS: dict = {}  # device -> [flag int32[1] (device), pinned host mirror, copy-done event]


def _index_flag(dev: torch.device) -> torch.Tensor:
    st = _IDX_FLAGS.get(dev)
    if st is None:
        st = _IDX_FLAGS[dev] = [torch.zeros(1, dtype=torch.int32, device=dev),
                                torch.zeros(1, dtype=torch.int32).pin_memory(), None]
    return st[0]


def _index_error(code: int, where: str):
    msgs = []
    if code & _IDX_EMBED:
        msgs.append("a token id is outside the embedding table [0, vocab_size) -- is the tokenizer larger than "
                    "the model vocabulary? (run_clm resizes the embeddings for that)")
    if code & _IDX_LABEL:
        msgs.append("a label is outside [0, vocab_size) and is not the ignore index -100")
    return ValueError(f"dlion ({where}): " + "; ".join(msgs))


def check_labels(labels1d: torch.Tensor, v: int) -> None:
    """Labels must be in [0, v) or -100 (ATen cross-entropy's contract)."""
    if labels1d.is_cuda and hip.available():
        hip.ops().index_check_(labels1d.contiguous(), int(v), -100, _index_flag(labels1d.device), _IDX_LABEL)
    elif not labels1d.is_cuda:
        bad = ((labels1d < 0) & (labels1d != -100)) | (labels1d >= v)
        if bool(bad.any()):
            raise _index_error(_IDX_LABEL, "labels")


def check_index_errors(blocking: bool = False) -> None:
    """Raise ValueError if a kernel flagged an out-of-range id or label.
    Non-blocking (the per-step call): reads the flag copied at the previous
    call if that copy has landed, then starts the next asynchronous copy.
    ``blocking``: reads the flag now (end of a run, tests)."""
    for dev, st in _IDX_FLAGS.items():
        flag, host, ev = st
        if blocking:
            code = int(flag.item())
        else:
            code = 0
            if ev is not None:
                if not ev.query():
                    continue  # the previous copy is still in flight
                code = int(host[0])
            host.copy_(flag, non_blocking=True)
            st[2] = torch.cuda.Event()
            st[2].record()
        if code:
            flag.zero_()
            st[2] = None
            raise _index_error(code, str(dev))


# ------------------------------------------------------------ token embedding
class _Embed(torch.autograd.Function):
    """x = dropout(wte[ids] + wpe[t]) for ids [B, T] (csrc/embedding.hip).
    Backward: the token gradient is a deterministic segmented sum over the
    stably sorted ids, added in place into wte.grad inside a fusion window
    (GPT-2's tied wte already holds the LM head's gradient there), instead of
    ATen's dense [V, C] embedding gradient + AccumulateGrad pass."""

    @staticmethod
    def forward(ctx, ids, wte, wpe, p, seed):
        from .linear import _fuse_target

        out = hip.ops().embed_fwd(ids, wte, wpe, p, seed, _index_flag(ids.device))
        ctx.save_for_backward(ids)
        ctx.p, ctx.seed = p, seed
        ctx.wte = wte if _fuse_target(wte) else None
        ctx.wpe = wpe if _fuse_target(wpe) else None
        ctx.shapes = (wte.shape, wpe.shape)
        return out

    @staticmethod
    def backward(ctx, dout):
        (ids,) = ctx.saved_tensors
        T = ids.shape[1]
        dx = dout.contiguous()
        ops = hip.ops()
        gw = gp = None
        sid = perm = dwte = dwpe = None
        pos_acc = False

        def target(param, shape, dev, dtype):
            if param is not None:
                if param.grad is None:
                    param.grad = torch.zeros(shape, dtype=dtype, device=dev)
                if param.grad.is_contiguous() and param.grad.dtype == dtype:
                    return param.grad, None
            buf = torch.zeros(shape, dtype=dtype, device=dev)
            return buf, buf

        if ctx.needs_input_grad[1]:
            sid, perm = torch.sort(ids.reshape(-1), stable=True)
            dwte, gw = target(ctx.wte, ctx.shapes[0], dx.device, dx.dtype)
        if ctx.needs_input_grad[2]:
            dwpe, gp = target(ctx.wpe, ctx.shapes[1], dx.device, dx.dtype)
            pos_acc = True  # rows >= T stay as they are (zeros when fresh)
        ops.embed_bwd_(dx, sid, perm, dwte, dwpe, T, pos_acc, ctx.p, ctx.seed)
        return None, gw, gp, None, None




def embed(ids: torch.Tensor, wte: torch.Tensor, wpe: torch.Tensor, p: float) -> torch.Tensor:
    """dropout(wte[ids] + wpe[arange(T)]) for ids [B, T]: one kernel each way on
    the GPU (bf16), the ATen chain elsewhere."""
    T = ids.shape[1]
    if (ids.is_cuda and wte.dtype == torch.bfloat16 and wpe.dtype == torch.bfloat16 and wte.shape[1] % 8 == 0
            and wte.is_contiguous() and wpe.is_contiguous() and T <= wpe.shape[0] and _use_hip(wte)):
        with torch.autocast("cuda", enabled=False):
            return _Embed.apply(ids.contiguous(), wte, wpe, float(p), _new_seed() if p > 0 else 0)
    x = F.embedding(ids, wte) + F.embedding(torch.arange(T, device=ids.device), wpe)[None]
    return F.dropout(x, p, True) if p > 0 else x


# ------------------------------------------------------------------ attention
def _attn_ok(x: torch.Tensor, T: int, D: int, window: int = 0) -> bool:
    """The gfx950 flash kernels take any sequence length (tail tiles are
    masked in-kernel) at head_dim 64 / 128 -- every GPT-2 and Llama-2/3 size;
    a sliding window (< T) at head_dim 128 (csrc/attention.hip window_of)."""
    return (x.dtype == torch.bfloat16 and D in (64, 128) and T >= 1 and _use_hip(x)
            and (_eff_window(window, T) == 0 or D == 128))


def _eff_window(window, T: int) -> int:
    """A sliding window that covers the whole sequence is plain causal: 0."""
    return int(window) if window and int(window) < T else 0


_MATH_WARNED = set()


def _sdpa_math(q, k, v, dropout_p: float, window: int = 0) -> torch.Tensor:
    """Fallback for what the flash kernels do not cover (head_dim not in {64,
    128}, fp32/fp16 inputs, no extension): PyTorch's *math* SDPA backend only
    -- matmul + softmax ATen ops (hipBLASLt GEMMs) -- never the flash /
    memory-efficient backends, which on ROCm are Triton-built (aotriton).
    O(T^2) memory; a one-time warning names the shape."""
    from torch.nn.attention import SDPBackend, sdpa_kernel

    key = (tuple(q.shape[-2:]), q.dtype, q.device.type)
    if q.is_cuda and key not in _MATH_WARNED:
        _MATH_WARNED.add(key)
        import warnings

        warnings.warn(f"dlion attention: no gfx950 flash kernel for head_dim={q.shape[-1]} / {q.dtype}; "
                      "using the math SDPA backend (O(T^2) memory)")
    T = q.shape[-2]
    window = _eff_window(window, T)
    with sdpa_kernel([SDPBackend.MATH]):
        if window:  # HF's sliding-window mask: key k visible to query q iff q - window < k <= q
            i = torch.arange(T, device=q.device)
            d = i[:, None] - i[None, :]
            return F.scaled_dot_product_attention(q, k, v, attn_mask=(d >= 0) & (d < window), dropout_p=dropout_p)
        return F.scaled_dot_product_attention(q, k, v, dropout_p=dropout_p, is_causal=True)


def _new_seed() -> int:
    return int(torch.randint(0, 2**31 - 1, (1,)).item())


class _FlashAttnPacked(torch.autograd.Function):
    """Causal attention on packed qkv [B,T,3,H,D]; dqkv is written in place of
    the q/k/v gradients (no stack/cat) by the gfx950 kernels."""

    @staticmethod
    def forward(ctx, qkv, p, seed):
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        out, lse = hip.ops().attn_fwd(q, k, v, p, seed)
        ctx.save_for_backward(qkv, out, lse)
        ctx.p, ctx.seed = p, seed
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        dout = dout.contiguous()
        dqkv = torch.empty_like(qkv)
        hip.ops().attn_bwd(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], out, dout, lse, ctx.p, ctx.seed,
                           dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2])
        return dqkv, None, None


class _FlashAttn(torch.autograd.Function):
    """Causal (GQA) attention on separate q [B,T,H,D], k/v [B,T,Hkv,D]."""

    @staticmethod
    def forward(ctx, q, k, v, p, seed, window=0):
        out, lse = hip.ops().attn_fwd(q, k, v, p, seed, window)
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.p, ctx.seed, ctx.window = p, seed, window
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, lse = ctx.saved_tensors
        dout = dout.contiguous()
        dq = torch.empty(q.shape, dtype=q.dtype, device=q.device)
        dkv = torch.empty((2,) + tuple(k.shape), dtype=k.dtype, device=k.device)
        hip.ops().attn_bwd(q, k, v, out, dout, lse, ctx.p, ctx.seed, dq, dkv[0], dkv[1], None, None, None,
                           ctx.window)
        return dq, dkv[0], dkv[1], None, None, None


def causal_attention(qkv: torch.Tensor, dropout_p: float) -> torch.Tensor:
    """qkv: [B, T, 3, H, D] -> causal softmax attention output [B, T, H*D]."""
    B, T, _, H, D = qkv.shape
    if qkv.is_cuda:
        from .linear import autocast_inputs

        (qkv,) = autocast_inputs(qkv)
    if _attn_ok(qkv, T, D):
        with torch.autocast("cuda", enabled=False):
            return _FlashAttnPacked.apply(qkv, float(dropout_p), _new_seed()).view(B, T, H * D)
    q, k, v = qkv.permute(2, 0, 3, 1, 4).unbind(0)  # [B, H, T, D] views
    y = _sdpa_math(q, k, v, dropout_p)
    return y.transpose(1, 2).reshape(B, T, H * D)


class _QKVAttention(torch.autograd.Function):
    """y = causal_attention(x @ Wqkv + b) for GPT-2's packed c_attn projection
    (Wqkv in HF Conv1D [C, 3C] layout).  One op so that the backward can take
    the c_attn bias gradient from the attention kernels themselves: the dQ /
    dKV kernels emit per-32-row column sums of the dq | dk | dv values they
    store (csrc/attention.hip), replacing a column-sum pass over the [tokens,
    3C] gradient."""

    @staticmethod
    def forward(ctx, x2d, w, b, B, T, H, p, seed):
        from .linear import _fuse_target, transposed_weight

        C3 = w.shape[1]
        D = C3 // (3 * H)
        wt = transposed_weight(w) if isinstance(w, torch.nn.Parameter) else w.t()
        qkv = gemm_fwd(x2d, wt, b).view(B, T, 3, H, D)
        out, lse = hip.ops().attn_fwd(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], p, seed)
        ctx.save_for_backward(x2d, w, qkv, out, lse)
        ctx.p, ctx.seed = p, seed
        ctx.fuse = _fuse_target(w)
        ctx.wparam = w  # deposit target (see _MLP: saved tensors may be checkpoint aliases)
        ctx.fused_b = _fused_params(b)[0]
        return out.view(B, T, H * D)

    @staticmethod
    def backward(ctx, dy):
        from .linear import deposit_grad, wgrad, wgrad_into

        x2d, w, qkv, out, lse = ctx.saved_tensors
        B, T = qkv.shape[:2]
        dout = dy.reshape(out.shape).contiguous()
        dqkv = torch.empty_like(qkv)
        part = torch.empty(B * ((T + 31) // 32), w.shape[1], dtype=torch.float32, device=qkv.device)
        hip.ops().attn_bwd(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], out, dout, lse, ctx.p, ctx.seed,
                           dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2], part)
        g = dqkv.view(B * T, -1)
        dx = gemm_fwd(g, w) if ctx.needs_input_grad[0] else None  # g @ W^T, W [C, 3C]
        dw = db = None
        if ctx.needs_input_grad[1]:
            if ctx.fuse:
                wgrad_into(x2d, g, ctx.wparam)
            else:
                dw = wgrad(x2d, g)
        if ctx.needs_input_grad[2]:
            if ctx.fused_b is not None:
                deposit_grad(ctx.fused_b, part)
            else:
                db = _sum_rows(part)
        return dx, dw, db, None, None, None, None, None




def qkv_attention(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, n_head: int, dropout_p: float) -> torch.Tensor:
    """GPT-2 attention core: causal_attention((x @ Wqkv + b).view(B, T, 3, H, D))
    -> [B, T, C], as one op on the GPU path (see _QKVAttention)."""
    from .linear import autocast_inputs, linear_kn

    B, T, C = x.shape
    D = w.shape[1] // (3 * n_head)
    if x.is_cuda:
        x, w, b = autocast_inputs(x, w, b)
    if (b is not None and x.is_cuda and x.dtype == w.dtype == b.dtype == torch.bfloat16
            and _attn_ok(x, T, D)
            and w.is_contiguous() and b.is_contiguous()):
        with torch.autocast("cuda", enabled=False):
            return _QKVAttention.apply(x.reshape(B * T, C).contiguous(), w, b, B, T, n_head, float(dropout_p),
                                       _new_seed())
    qkv = linear_kn(x, w, b).view(B, T, 3, n_head, D)
    return causal_attention(qkv, dropout_p)


def causal_attention_gqa(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, dropout_p: float = 0.0,
                         window: int = 0) -> torch.Tensor:
    """q [B,T,H,D], k/v [B,T,Hkv,D] -> [B,T,H*D] (grouped-query causal attention;
    ``window`` > 0: sliding window, query q sees keys q - window < k <= q)."""
    B, T, H, D = q.shape
    window = _eff_window(window, T)
    if q.is_cuda:
        from .linear import autocast_inputs

        q, k, v = autocast_inputs(q, k, v)
    if _attn_ok(q, T, D, window):
        with torch.autocast("cuda", enabled=False):
            return _FlashAttn.apply(q, k, v, float(dropout_p), _new_seed(), window).view(B, T, H * D)
    rep = H // k.shape[2]
    qh, kh, vh = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
    if rep > 1:
        kh = kh.repeat_interleave(rep, dim=1)
        vh = vh.repeat_interleave(rep, dim=1)
    y = _sdpa_math(qh, kh, vh, dropout_p, window)
    return y.transpose(1, 2).reshape(B, T, H * D)




def _adjacent_heads(q: torch.Tensor, k: torch.Tensor):
    """[B, T, Hq + Hk, D] view over q [B, T, Hq, D] and k when k's heads follow
    q's in memory with the same token stride (the fused q|k|v output), else None."""
    B, T, Hq, D = q.shape
    if (k.shape[0] != B or k.shape[1] != T or k.shape[3] != D or q.stride() != k.stride() or q.stride(2) != D
            or q.stride(3) != 1 or k.data_ptr() != q.data_ptr() + Hq * D * q.element_size()
            or k.untyped_storage().data_ptr() != q.untyped_storage().data_ptr()):
        return None
    return q.as_strided((B, T, Hq + k.shape[2], D), q.stride())


class _RopeAttention(torch.autograd.Function):
    """Llama attention core: causal GQA attention on rope(q), rope(k), v where
    q / k / v are column views of the fused q|k|v projection output.  The
    backward writes dq | dk | dv into ONE packed buffer (attention kernels
    into its column slices, the inverse rotation in place), so the fused
    projection's backward takes the three gradients as adjacent views of one
    [tokens, (H + 2 Hkv) D] matrix -- no concatenation copy (it was ~4 % of the
    Llama-2-7B LoRA SFT step)."""

    @staticmethod
    def forward(ctx, q, k, v, cos, sin, p, seed, window=0):
        ops = hip.ops()
        H = q.shape[2]
        qk = _adjacent_heads(q, k)
        if qk is not None:  # q | k adjacent column blocks of the projection output: one rotation launch
            r = ops.rope(qk, cos, sin, False)
            qr, kr = r[:, :, :H], r[:, :, H:]
        else:
            qr = ops.rope(q, cos, sin, False)
            kr = ops.rope(k, cos, sin, False)
        out, lse = ops.attn_fwd(qr, kr, v, p, seed, window)
        ctx.save_for_backward(qr, kr, v, out, lse, cos, sin)
        ctx.p, ctx.seed, ctx.window = p, seed, window
        return out

    @staticmethod
    def backward(ctx, dout):
        qr, kr, v, out, lse, cos, sin = ctx.saved_tensors
        B, T, H, D = qr.shape
        Hkv = kr.shape[2]
        buf = torch.empty(B, T, H + 2 * Hkv, D, dtype=qr.dtype, device=qr.device)
        dq, dk, dv = buf[:, :, :H], buf[:, :, H:H + Hkv], buf[:, :, H + Hkv:]
        ops = hip.ops()
        if _ROPE_BWD_FUSED and cos.shape[-1] == D:
            # the kernels store dq / dk through the inverse rotation (no extra pass)
            ops.attn_bwd(qr, kr, v, out, dout.contiguous(), lse, ctx.p, ctx.seed, dq, dk, dv, None,
                         cos.reshape(-1, D), sin.reshape(-1, D), ctx.window)
            return dq, dk, dv, None, None, None, None, None
        ops.attn_bwd(qr, kr, v, out, dout.contiguous(), lse, ctx.p, ctx.seed, dq, dk, dv, None, None, None,
                     ctx.window)
        ops.rope_(buf[:, :, :H + Hkv], cos, sin, True)  # dq | dk: one in-place inverse rotation
        return dq, dk, dv, None, None, None, None, None


_ROPE_BWD_FUSED = True  # inverse rotation in the bwd kernels' stores (tests compare the separate pass)


def rope_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor,
                   dropout_p: float = 0.0, window: int = 0) -> torch.Tensor:
    """causal_attention_gqa(rope(q), rope(k), v, window) -> [B, T, H*D]; q [B,T,H,D],
    k / v [B,T,Hkv,D] (views of a fused projection output are read in place)."""
    B, T, H, D = q.shape
    window = _eff_window(window, T)
    if q.is_cuda:
        from .linear import autocast_inputs

        q, k, v = autocast_inputs(q, k, v)
    if (_attn_ok(q, T, D, window) and cos.dtype == sin.dtype == torch.bfloat16
            and k.dtype == v.dtype == torch.bfloat16 and all(_token_strided_ok(t) for t in (q, k, v))):
        with torch.autocast("cuda", enabled=False):
            out = _RopeAttention.apply(q, k, v, cos.contiguous(), sin.contiguous(), float(dropout_p), _new_seed(),
                                       window)
        return out.view(B, T, H * D)
    return causal_attention_gqa(rope(q, cos, sin), rope(k, cos, sin), v, dropout_p, window)


# ------------------------------------------------------------------- LoRA
def _lora_rows_ok(t: torch.Tensor) -> bool:
    return (t.dim() == 2 and t.dtype == torch.bfloat16 and t.stride(1) == 1 and t.stride(0) % 8 == 0
            and t.shape[1] % 8 == 0 and t.data_ptr() % 16 == 0)


def _lora_weight_grad(param, part2d: torch.Tensor, fuse: bool):
    """Deposit (fusion window) or return the column sums of fp32 partials."""
    from .linear import deposit_grad

    if fuse:
        deposit_grad(param, part2d, defer=False)  # MB-sized stacks: nothing to gain from deferral
        return None
    return hip.ops().sum_partials(part2d).view_as(param)


class _LoraAdd(torch.autograd.Function):
    """out = o + s * (drop(x) A^T) B^T with the csrc/lora.hip streams: the
    forward reads x once (dropout from the stateless hash, never stored) and
    o once; the backward reads dout twice (du, dB) and x once (dA and dx in
    the same pass).  o's gradient is dout itself, so a fused projection's
    packed gradient buffer stays packed."""

    @staticmethod
    def forward(ctx, o, x, a, b, s, p, seed):
        from .linear import _fuse_target

        ops = hip.ops()
        u = ops.lora_rows(x, a, 1.0, p, seed)
        out = ops.lora_up(o, u, b, s)
        ctx.save_for_backward(x, u, a, b)
        ctx.s, ctx.p, ctx.seed = s, p, seed
        ctx.fuse = (_fuse_target(a), _fuse_target(b))
        ctx.abparams = (a, b)  # deposit targets (see _MLP: saved tensors may be checkpoint aliases)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, u, a, b = ctx.saved_tensors
        if not _lora_rows_ok(dout):
            dout = dout.contiguous()
        ops = hip.ops()
        ga = gb = dx = None
        if ctx.needs_input_grad[3]:
            part_b, _ = ops.lora_cols(dout, u, None, ctx.s, 0.0, 0)
            gb = _lora_weight_grad(ctx.abparams[1], part_b.view(part_b.shape[0], -1), ctx.fuse[1])
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            du = ops.lora_rows(dout, b.t().contiguous(), ctx.s, 0.0, 0)
            part_a, dx = ops.lora_cols(x, du, a, 1.0, ctx.p, ctx.seed)
            if ctx.needs_input_grad[2]:
                ga = _lora_weight_grad(ctx.abparams[0], part_a.view(part_a.shape[0], -1), ctx.fuse[0])
        return dout if ctx.needs_input_grad[0] else None, dx, ga, gb, None, None, None


_LORA_FUSED = True  # fused LoRA kernels (tests compare the unfused chain)


def lora_add(o: torch.Tensor, x: torch.Tensor, a: torch.Tensor, b: torch.Tensor, scaling: float,
             p: float) -> torch.Tensor:
    """o + dropout(x, p) A^T B^T * scaling (peft's LoRA output, A [r, K],
    B [N, r]); the fused HIP path for bf16 GPU tensors with r in {8, 16}."""
    r = a.shape[0]
    if _LORA_FUSED and x.is_cuda and r in (8, 16) and _use_hip(x):
        from .linear import autocast_inputs

        o_, x_, a_, b_ = autocast_inputs(o, x, a, b)
        if x_.dtype == o_.dtype == a_.dtype == b_.dtype == torch.bfloat16 and a_.is_contiguous() and b_.is_contiguous():
            x2 = x_.reshape(-1, x_.shape[-1])
            o2 = o_.reshape(-1, o_.shape[-1])
            if not _lora_rows_ok(x2):
                x2 = x2.contiguous()
            if (_lora_rows_ok(o2) and _lora_rows_ok(x2) and a_.shape[1] == x2.shape[1] and b_.shape[0] == o2.shape[1]
                    and x2.shape[1] % 32 == 0 and o2.shape[1] % 32 == 0):
                with torch.autocast("cuda", enabled=False):
                    out = _LoraAdd.apply(o2, x2, a_, b_, float(scaling), float(p), _new_seed() if p > 0 else 0)
                return out.view(o.shape)
    xd = F.dropout(x, p, True) if p > 0 else x
    return o + F.linear(F.linear(xd, a), b) * scaling


_M32 = 0xFFFFFFFF


def _lowbias32(x: torch.Tensor) -> torch.Tensor:
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    return x ^ (x >> 16)


def attention_dropout_keep(B: int, H: int, T: int, p: float, seed: int, device=None) -> torch.Tensor:
    """bool keep-mask [B, H, T(q), T(key)] exactly as the HIP kernels draw it
    (csrc/attention.hip, drop hash v3): one 32-bit hash per (row, key pair),
    the low half for the even key; a key is kept iff its half, read as a
    signed 16-bit value, is >= thresh16 - 32768.  The hash of pair jj (0..15)
    of 32-key tile kt in row (bh, q) is mix1(base + jj * kKeyMul) with a
    per-(row, tile) base mix1(rotr(arow, 8 (kt mod 4)) ^ kt * kTileMul).  v2's
    base was linear in the tile (arow + 16 kt kKeyMul): the rows' masks were
    windows of ONE fixed sequence, rows whose arow differed by a small multiple
    of kKeyMul held shifted copies of each other's masks, and since
    mix1 reads 24 bits, rows agreeing in arow's low 24 bits (a 2^-24 birthday
    rate: ~4 pairs among a GPT-2 layer's 12k rows per batch row) had identical
    masks.  The rotation gives each tile a different 24-bit view of the
    32-bit row key, so two rows coincide in every tile only if their full
    keys do."""
    th = min(65535, int(round(p * 65536)))
    bh = torch.arange(B * H, device=device, dtype=torch.int64).view(B * H, 1, 1)
    q = torch.arange(T, device=device, dtype=torch.int64).view(1, T, 1)
    key = torch.arange(T, device=device, dtype=torch.int64).view(1, 1, T)

    def mix1(x):  # v_mul_u32_u24 + xor-shift
        x = ((x & 0xFFFFFF) * 0x9E3779) & _M32
        return x ^ (x >> 16)

    arow = _lowbias32(((bh * 0x9E3779B9) & _M32) ^ ((q * 0x85EBCA6B) & _M32) ^ (seed & _M32))
    rot = ((key >> 5) & 3) * 8
    arot = ((arow >> rot) | (arow << ((32 - rot) & 31))) & _M32
    base = mix1(arot ^ (((key >> 5) * 0x27D4EB2F) & _M32))
    x = mix1((base + (((key >> 1) & 15) * 0xC2B2AE35)) & _M32)
    u16 = (x >> ((key & 1) * 16)) & 0xFFFF
    s16 = u16 - ((u16 >> 15) << 16)
    return (s16 >= th - 32768).view(B, H, T, T)


def reference_attention(q, k, v, dropout_p: float = 0.0, seed: int = 0, window: int = 0) -> torch.Tensor:
    """fp32 math reference with the kernels' dropout mask: q [B,T,H,D], k/v [B,T,Hkv,D]
    (``window`` > 0: keys q - window < k <= q only)."""
    B, T, H, D = q.shape
    rep = H // k.shape[2]
    qh = q.float().transpose(1, 2)
    kh = k.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    vh = v.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    s = (qh @ kh.transpose(-1, -2)) / (D ** 0.5)
    causal = torch.ones(T, T, dtype=torch.bool, device=q.device).tril()
    if window:
        causal &= ~torch.ones(T, T, dtype=torch.bool, device=q.device).tril(-window)
    s = s.masked_fill(~causal, float("-inf"))
    pr = torch.softmax(s, dim=-1)
    if dropout_p > 0:
        th = min(65535, int(round(dropout_p * 65536)))
        keep = attention_dropout_keep(B, H, T, dropout_p, seed, q.device)
        pr = pr * keep * (65536.0 / (65536.0 - th))
    return (pr @ vh).transpose(1, 2).reshape(B, T, H * D)


# ------------------------------------------------- LM head + cross-entropy
def _pad_rows(w: torch.Tensor, mult: int = 64) -> torch.Tensor:
    """Vocabulary rows padded to a multiple of 64, cached per optimizer step
    for parameters (the same padded copy serves every micro-batch)."""
    v = w.shape[0]
    vp = (v + mult - 1) // mult * mult
    if vp == v:
        return w
    if isinstance(w, torch.nn.Parameter):
        from .linear import cached_derived

        return cached_derived(w, "pad_rows", lambda t: torch.cat([t, t.new_zeros(vp - v, t.shape[1])], 0))
    return torch.cat([w, w.new_zeros(vp - v, w.shape[1])], 0)


def _lm_dgrad(g: torch.Tensor, weight: torch.Tensor, wp: torch.Tensor) -> torch.Tensor:
    """g [N, Vp] @ wp [Vp, C]: the LM head's input gradient, K = vocab.  When
    the output has fewer 256x256 tiles than the chip has CUs (GPT-2: 20480 x 768
    = 240 tiles, each with a 50304-long K loop) the own gfx950 NT GEMM
    (csrc/gemm.hip) against a per-step cached wp^T beats hipBLASLt: 1589 ->
    1169 us (tools/bench_lmhead.py), same-box bench A/B 859k -> 880k tok/s.
    At Llama-3-8B's 8192 x 4096 (512 tiles) hipBLASLt stays ahead (22.6k vs
    22.1k tok/s with the own kernel), so larger outputs keep it."""
    vp = wp.shape[0]
    tiles = -(-g.shape[0] // 256) * -(-wp.shape[1] // 256)
    if (tiles < 256 and isinstance(weight, torch.nn.Parameter) and g.is_cuda
            and g.dtype == torch.bfloat16 and vp % 128 == 0 and vp >= 8192 and g.is_contiguous()
            and g.numel() < 2**31 and hip.available()):
        from .linear import cached_derived

        from .linear import fast_transpose

        wpt = cached_derived(weight, "pad_t", lambda t: fast_transpose(t, vp))  # [C, Vp], zero vocab padding
        return hip.ops().gemm_nt(g, wpt, None)
    return g @ wp


_LM_DEFER = True  # LM-head weight gradient in the window-level TN GEMM (tests compare per micro-batch)


def _lm_wgrad_partials(g: torch.Tensor, h2d: torch.Tensor, v: int):
    """The LM head's weight gradient g^T h (g = softmax - onehot [N, Vp]) as
    fp32 split partials [S, v*C] from the own TN kernel (csrc/gemm_tn.hip), or
    None when not applicable.  GPT-2: 591 output tiles -> 3 splits (7 short
    waves instead of 3 long ones); the backward reduces, scales by the loss
    gradient and deposits them in one pass.  Measured 1.62 ms (hipBLASLt) vs
    ~1.3 ms + 0.15 ms of partial traffic (tools/bench_wgrad.py)."""
    from .linear import _tn_eligible, tn_split_factor

    if not (g.shape[1] % 8 == 0 and _tn_eligible(g, h2d) and hip.available()):
        return None
    s = tn_split_factor(g.shape[0], g.shape[1], h2d.shape[1])
    part = hip.ops().gemm_tn([g], [h2d], s)  # [S, Vp, C]
    return part.view(s, -1)[:, : v * h2d.shape[1]]


class _LMHeadCE(torch.autograd.Function):
    """loss = mean_{labels != -100} CE(h @ W^T, labels), gradients computed in
    the forward pass (the loss gradient is a scalar multiple of
    softmax - onehot), so the [N, V] logits never persist and never exist in
    fp32.  The vocabulary is padded to a multiple of 64 for aligned rows and
    well-shaped GEMMs; padded columns are masked out of the softmax."""

    @staticmethod
    def forward(ctx, h2d, weight, labels1d, normalizer=None):
        v = weight.shape[0]
        need_grad = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
        wp = _pad_rows(weight)
        logits = gemm_fwd(h2d, wp)  # [N, Vp] in the compute dtype
        if normalizer is None:
            n_valid = (labels1d != -100).sum().clamp_min(1).to(torch.float32)
        else:
            n_valid = torch.as_tensor(normalizer, dtype=torch.float32, device=h2d.device).clamp_min(1)
        check_labels(labels1d, v)
        if _use_hip(logits):
            row_loss = hip.ops().softmax_xent_(logits, labels1d, v)  # logits <- softmax - onehot (in place)
        else:
            row_loss = _softmax_xent_torch_(logits, labels1d, v)
        loss = row_loss.sum() / n_valid
        if need_grad:
            dh = _lm_dgrad(logits, weight, wp)  # [N, C]
            dw = None
            ctx.dw_parts = False
            ctx.defer = ctx.needs_input_grad[1] and _lm_defer_ok(weight, logits, h2d)
            if ctx.defer:
                # the weight gradient joins the fusion window: the backward scales h by
                # the loss gradient and hands (softmax - onehot, s * h) to the window's
                # single TN GEMM over all micro-batches (ops/linear.py deferral)
                ctx.save_for_backward(dh, logits, n_valid, h2d)
                ctx.has_dw = True
                ctx.weight = weight
                return loss
            if ctx.needs_input_grad[1] and _lm_late_ok(weight, logits, h2d, v):
                # unsplit (Llama-sized head): the backward runs one TN GEMM of
                # (softmax - onehot) against s * h writing the bf16 gradient itself --
                # no fp32 [Vp, C] partials between the passes, no reduction pass
                ctx.save_for_backward(dh, logits, n_valid, h2d)
                ctx.late = True
                ctx.v = v
                from .linear import _fuse_target

                ctx.weight = weight if _fuse_target(weight) else None
                return loss
            if ctx.needs_input_grad[1]:
                dw = _lm_wgrad_partials(logits, h2d, v)
                ctx.dw_parts = dw is not None
                if dw is None:
                    dw = (logits.t() @ h2d)[:v]
            ctx.save_for_backward(dh, dw if dw is not None else dh.new_empty(0), n_valid)
            ctx.has_dw = dw is not None
            from .linear import _fuse_target

            ctx.weight = weight if dw is not None and _fuse_target(weight) else None
        del logits
        return loss

    @staticmethod
    def backward(ctx, g):
        if getattr(ctx, "defer", False):
            return _LMHeadCE._backward_deferred(ctx, g)
        if getattr(ctx, "late", False):
            return _LMHeadCE._backward_late(ctx, g)
        dh, dw, n_valid = ctx.saved_tensors
        if not (dh.is_cuda and dh.dtype == torch.bfloat16 and _use_hip(dh)):
            scale = (g / n_valid).to(dh.dtype)
            gh = dh * scale if ctx.needs_input_grad[0] else None
            gw = dw * scale if ctx.has_dw and ctx.needs_input_grad[1] else None
            return gh, gw, None, None
        # one pass each: bf16(x * bf16(g / n)) with the scale on the device; the
        # weight gradient is added straight into .grad inside a fusion window
        # (tied GPT-2 wte: the embedding backward then adds its rows in place)
        s = (g.float() / n_valid).reshape(1)
        ops = hip.ops()
        gh = gw = None
        if ctx.needs_input_grad[0]:
            gh = torch.empty_like(dh)
            ops.scale_acc_(dh, s, gh, False)
        if ctx.has_dw and ctx.needs_input_grad[1] and ctx.dw_parts:
            # fp32 split partials [S, v*C] (row-strided): reduce + scale + deposit in one pass
            w = ctx.weight
            if w is not None and w.grad is not None and w.grad.is_contiguous() and w.grad.dtype == dh.dtype:
                ops.sum_partials_scaled_(dw, s, w.grad, True)
            else:
                out = torch.empty(dw.shape[1] // dh.shape[1], dh.shape[1], dtype=dh.dtype, device=dh.device)
                ops.sum_partials_scaled_(dw, s, out, False)
                if w is not None:
                    w.grad = out if w.grad is None else w.grad + out
                else:
                    gw = out
        elif ctx.has_dw and ctx.needs_input_grad[1]:
            w = ctx.weight
            if w is not None and w.grad is not None and w.grad.is_contiguous() and w.grad.dtype == dw.dtype:
                ops.scale_acc_(dw, s, w.grad, True)
            else:
                out = torch.empty_like(dw)
                ops.scale_acc_(dw, s, out, False)
                if w is not None:
                    w.grad = out if w.grad is None else w.grad + out
                else:
                    gw = out
        return gh, gw, None, None

    @staticmethod
    def _backward_deferred(ctx, g):
        """Backward of a head whose weight gradient joined the fusion window."""
        from . import linear

        dh, logits, n_valid, h2d = ctx.saved_tensors
        s = (g.float() / n_valid).reshape(1)
        ops = hip.ops()
        gh = None
        if ctx.needs_input_grad[0]:
            gh = torch.empty_like(dh)
            ops.scale_acc_(dh, s, gh, False)
        w = ctx.weight
        v, c = w.shape
        hs = torch.empty_like(h2d)  # s * h: the per-micro-batch loss scale rides on the small operand
        ops.scale_acc_(h2d.contiguous(), s, hs, False)
        split = linear.tn_split_factor(logits.shape[0], logits.shape[1], c)
        if not linear._defer_wgrad([w], [(0, v * c)], logits, hs, split):
            part = ops.gemm_tn([logits], [hs], split)  # over budget / window closed: now
            linear.deposit_grad(w, part.view(split, -1)[:, : v * c], defer=False)
        return gh, None, None, None


    @staticmethod
    def _backward_late(ctx, g):
        """Backward of an unsplit head: w.grad (+)= bf16((softmax - onehot)^T (s h))
        from the TN kernel's bf16 epilogue (the window path's operand scaling)."""
        dh, logits, n_valid, h2d = ctx.saved_tensors
        s = (g.float() / n_valid).reshape(1)
        ops = hip.ops()
        gh = gw = None
        if ctx.needs_input_grad[0]:
            gh = torch.empty_like(dh)
            ops.scale_acc_(dh, s, gh, False)
        hs = torch.empty_like(h2d)
        ops.scale_acc_(h2d.contiguous(), s, hs, False)
        lv = logits[:, : ctx.v]  # row stride Vp: the vocabulary padding is never read
        w = ctx.weight
        if w is not None and w.grad is not None and w.grad.is_contiguous() and w.grad.dtype == torch.bfloat16:
            ops.gemm_tn_([lv], [hs], w.grad, True)
        else:
            out = torch.empty(ctx.v, h2d.shape[1], dtype=torch.bfloat16, device=h2d.device)
            ops.gemm_tn_([lv], [hs], out, False)
            if w is not None:
                w.grad = out if w.grad is None else w.grad + out
            else:
                gw = out
        return gh, gw, None, None


def _lm_late_ok(weight, logits, h2d, v) -> bool:
    """The head's weight gradient runs unsplit in the backward (bf16 straight
    from the TN kernel): a bf16 weight, v % 8 == 0 (the kernel reads the
    unpadded columns of the padded logits), TN-eligible operands, and the split
    model choosing one split for the unsplit launch (Llama-3-8B's 128256 x 4096:
    7.4 ms GEMM + 0.6 ms partial reduction before)."""
    from . import linear

    if not (logits.is_cuda and weight.dtype == torch.bfloat16 and v % 8 == 0
            and hip.available()):
        return False
    lv = logits[:, :v]
    return (linear._tn_eligible(lv, h2d)
            and linear.tn_split_factor(logits.shape[0], v, h2d.shape[1], direct=True) == 1)


def _lm_defer_ok(weight, logits, h2d) -> bool:
    """The LM head's weight gradient can join the window-level TN GEMM: a
    multi-micro-batch fusion window, a fusable bf16 weight, TN-eligible operands."""
    from . import linear

    return (_LM_DEFER and logits.is_cuda and linear._WDEFER_ON and linear._ST.fuse["on"]
            and linear._ST.fuse["multi"] and not linear._ST.fuse["nodefer"] and linear._fuse_target(weight)
            and logits.shape[1] % 8 == 0 and linear._tn_eligible(logits, h2d) and hip.available())




def _softmax_xent_torch_(logits: torch.Tensor, labels: torch.Tensor, v: int) -> torch.Tensor:
    """In-place reference of the HIP kernel: logits[:, :v] <- softmax - onehot
    (zero rows for ignored labels, zero padded columns); returns fp32 row loss."""
    x = logits[:, :v].float()
    lse = torch.logsumexp(x, dim=1)
    valid = labels != -100
    safe = labels.clamp_min(0)
    tgt = x.gather(1, safe[:, None]).squeeze(1)
    row_loss = torch.where(valid, lse - tgt, torch.zeros_like(lse))
    prob = torch.exp(x - lse[:, None])
    prob.scatter_add_(1, safe[:, None], -torch.ones_like(tgt)[:, None])
    prob[~valid] = 0.0
    logits[:, :v] = prob.to(logits.dtype)
    if logits.shape[1] > v:
        logits[:, v:] = 0
    return row_loss


class _TokenLogp(torch.autograd.Function):
    """Per-token log p(label) of ``h @ W^T`` (0 for labels == -100) through the
    same fused softmax-xent kernel: the [N, V] logits are turned into
    softmax - onehot in place; forward-only callers (the frozen DPO reference
    model) keep nothing, training callers keep that bf16 matrix for the two
    backward GEMMs (the row weights differ per sequence, so the gradients
    cannot be pre-contracted in the forward as in _LMHeadCE)."""

    @staticmethod
    def forward(ctx, h2d, weight, labels1d):
        v = weight.shape[0]
        wp = _pad_rows(weight)
        logits = h2d @ wp.t()
        check_labels(labels1d, v)
        if _use_hip(logits):
            row_loss = hip.ops().softmax_xent_(logits, labels1d, v)
        else:
            row_loss = _softmax_xent_torch_(logits, labels1d, v)
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            ctx.save_for_backward(h2d, wp, logits)
            ctx.v = v
            ctx.weight = weight
        return -row_loss

    @staticmethod
    def backward(ctx, g):
        h2d, wp, pm = ctx.saved_tensors  # pm = softmax - onehot
        d = pm * (-g).to(pm.dtype)[:, None]  # d logp / d logits = -(softmax - onehot)
        dh = _lm_dgrad(d, ctx.weight, wp) if ctx.needs_input_grad[0] else None
        dw = (d.t() @ h2d)[: ctx.v] if ctx.needs_input_grad[1] else None
        return dh, dw, None


def token_logps(h: torch.Tensor, weight: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """log p(labels) per position of h [..., C] under the LM head (0 where -100)."""
    h2d = h.reshape(-1, h.shape[-1])
    lab = labels.reshape(-1)
    if h2d.is_cuda:
        from .linear import autocast_inputs

        h2d, weight = autocast_inputs(h2d.contiguous(), weight)
        with torch.autocast("cuda", enabled=False):
            return _TokenLogp.apply(h2d, weight, lab).view(labels.shape)
    if h2d.dtype != weight.dtype:
        h2d = h2d.to(weight.dtype)
    return _TokenLogp.apply(h2d.contiguous(), weight, lab).view(labels.shape)


def lm_head_cross_entropy(h: torch.Tensor, weight: torch.Tensor, labels: torch.Tensor,
                          normalizer=None) -> torch.Tensor:
    """Token cross-entropy of ``h @ weight.T`` against ``labels`` (-100 ignored):
    mean over valid tokens, or sum / ``normalizer`` (HF ``num_items_in_batch``)."""
    h2d = h.reshape(-1, h.shape[-1])
    if h2d.is_cuda:
        from .linear import autocast_inputs

        h2d, weight = autocast_inputs(h2d, weight)
        with torch.autocast("cuda", enabled=False):
            return _LMHeadCE.apply(h2d, weight, labels.reshape(-1), normalizer)
    if h2d.dtype != weight.dtype:
        h2d = h2d.to(weight.dtype)
    return _LMHeadCE.apply(h2d, weight, labels.reshape(-1), normalizer)


def shift_labels(labels: torch.Tensor) -> torch.Tensor:
    """HF causal-LM label shift without slicing the hidden states: position t
    is scored against labels[t + 1]; the last position gets -100 (ignored).
    The LM head then runs on the whole [B, T] hidden-state block in place --
    no [B, T-1] copy of h forward, no scatter of its gradient backward, and
    M = B * T keeps the GEMMs tile-aligned."""
    out = torch.full_like(labels, -100)
    out[..., :-1] = labels[..., 1:]
    return out


def causal_lm_loss(h: torch.Tensor, weight: torch.Tensor, labels: torch.Tensor, normalizer=None) -> torch.Tensor:
    """Shifted next-token cross-entropy of the LM head on h [B, T, C]."""
    return lm_head_cross_entropy(h, weight, shift_labels(labels), normalizer=normalizer)


def reference_lm_loss(h, weight, labels):
    """Unfused reference (HF semantics) used by tests."""
    logits = (h.reshape(-1, h.shape[-1]) @ weight.t()).float()
    return F.cross_entropy(logits, labels.reshape(-1), ignore_index=-100)


