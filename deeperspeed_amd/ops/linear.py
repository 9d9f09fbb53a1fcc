"""Linear layers whose weight-gradient GEMM accumulates straight into the bound gradient.

The engine binds `p.grad` of every ZeRO-managed parameter to a view of a flat gradient
arena (ZeRO-0/1, single-rank ZeRO-3) or of a unit's gathered gradient bucket (ZeRO-3).
Stock autograd then forms each weight gradient in a fresh [out, in] buffer and
`AccumulateGrad` adds it into the bound view: one extra read + write of the full gradient
per micro-batch (an elementwise add over every weight; 2.5 % of a 20B step on MI355X).

Here the wgrad is one hipBLASLt GEMM with beta = 1 (`grad.addmm_(dy^T, x)`), which reads
the bound gradient in the epilogue and accumulates in fp32 before rounding once.  The
backward returns None for that parameter; autograd's AccumulateGrad node still runs and fires
the parameter's post-accumulate-grad hooks (the ZeRO bucket bookkeeping) in the usual order.
When no gradient is bound (first use, ZeRO-2 buckets that steal `p.grad`, plain torch
training), the layer returns the gradient to autograd as usual.

Reference counterpart: the weight-gradient GEMMs of `csrc/transformer/ds_transformer_cuda.cpp`
(`_ff1.Backward`, `_ff2.Backward`, `_attn_out_linear.Backward`, `_qkv_linear.Backward`,
`ds_transformer_cuda.cpp:370-540`), which write into the parameter's `.grad` storage.

Reduction-contiguous wgrad operands (GPU tensors): hipBLASLt on
gfx950 runs dW = dy^T x at ~1.1 PF/s with the token-major operands autograd holds, and at
~1.45 PF/s when both operands are contiguous along the token (reduction) dimension
(profiles/aux/wgrad_dgrad_variants_neox20b.jsonl).  The HIP transpose kernel
(ops/csrc/kernels/transpose.hip) makes dy^T and x^T first; the transpose of dy also produces
the bias gradient (its column sum) from the same read.
"""

from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import lt_tune
from . import wgrad_batch as _wb

FUSE_WGRAD = True
WGRAD_NT = True
# smallest out*in weight that takes the transposed path (the transposes move ~4*M*(out+in)
# bytes; below this the GEMM saving does not pay for them)
WGRAD_NT_MIN_NUMEL = 10_000_000
# cap on the transient transposed copies (bytes of dy^T + x^T): the LM head's dlogits at 16k
# tokens (1.65 GB) keeps the token-major formulation instead of adding its copy to the peak
WGRAD_NT_MAX_BYTES = 1_200_000_000
# input gradient dx = dy W from W^T [in, out] (reduction-contiguous, one HIP transpose of the
# weight per use): hipBLASLt ~1.45 vs ~1.28 PF/s at the GPT-NeoX-20B shapes, 1.05-1.2 vs
# 0.98-1.03 PF/s at BERT-Large's (profiles/r2m_gemm_shapes_bert_neox.md)
DGRAD_NT = True
DGRAD_NT_MIN_NUMEL = 1_000_000
# split-K weight gradient for small weights over many tokens: [out, in] gives too few 256x256
# output tiles to fill 256 CUs (BERT-Large: 16-64 tiles at 8k tokens, 300-800 TF/s), so the
# tokens are cut into WGRAD_SPLIT batches of one strided-batched GEMM whose partial products
# are summed in fp32 (1.25-1.6x at the BERT-Large shapes, same profile).
WGRAD_SPLIT = 4
WGRAD_SPLIT_MAX_TILES = 128
WGRAD_SPLIT_MIN_TOKENS = 4096


_count = [0]  # in-place accumulations performed (tests / diagnostics)
_nt_count = [0]  # wgrads formed from transposed operands


def fused_wgrad_count() -> int:
    return _count[0]


def nt_wgrad_count() -> int:
    return _nt_count[0]


def _bound_grad(p: torch.Tensor):
    if (torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
            and not getattr(p, "_dsa_persistent_grad", False)):
        # a HIP-graph capture may only bake in gradient buffers that outlive the step
        # (make_graphed_encoder's persistent .grad, zeroed in place by the optimizer)
        return None
    g = p.grad
    if g is None or g.shape != p.shape or g.dtype != p.dtype or g.device != p.device:
        return None
    return g


# Pre-transposed operands: a tensor recorded together with its contiguous transpose, consumed
# by the next weight gradient that reads that same tensor -- du and du^T written in one pass by
# the bias+GeLU backward (fc1's wgrad), and the block-output gradient that the parallel-residual
# branches share (fc2's wgrad transposes it, the attention output projection reuses it).  Each
# entry holds the tensor itself, so its storage cannot be recycled for another tensor while the
# entry exists (no false address matches); at most _PRE_T_SLOTS entries are kept.
_pre_t = []
_PRE_T_SLOTS = 2


def offer_transposed(t: torch.Tensor, t_t: torch.Tensor):
    """Record t_t = t^T (contiguous) for a later weight gradient that reads t."""
    _pre_t.append((t, t_t))
    if len(_pre_t) > _PRE_T_SLOTS:
        del _pre_t[0]


def clear_transposed():
    _pre_t.clear()


def _take_transposed(x2: torch.Tensor):
    for i, (t, t_t) in enumerate(_pre_t):
        if (t.data_ptr() == x2.data_ptr() and t.numel() == x2.numel() and x2.dim() == 2
                and tuple(t_t.shape) == (x2.size(1), x2.size(0)) and x2.is_contiguous()):
            del _pre_t[i]
            return t_t
    return None


def _t_operand(x2, colsum_out=None, offer=False):
    """x2^T contiguous (x2 [M, K]): free when x2 is a column-major view or its transpose was
    offered by the kernel that wrote it, else one HIP transpose (which also folds
    colsum_out += sum(x2) into the same read; with `offer` the result is kept for the next
    weight gradient of the same x2)."""
    from . import native
    pre = x2.t() if (x2.t().is_contiguous() and x2.stride(1) != 1) else _take_transposed(x2)
    if pre is not None:
        if colsum_out is not None:
            native.colsum(x2, colsum_out, accumulate=True)
        return pre
    if native.transpose_supported(x2):
        xt = native.transpose2d(x2, colsum_out, accum=colsum_out is not None)
        if offer and SHARE_GRAD_T:
            offer_transposed(x2, xt)
        return xt
    return None


# one transpose of a shared output gradient serves both weight gradients that read it
SHARE_GRAD_T = True


def nt_wgrad_planned(M: int, out_features: int, in_features: int, elem_size: int = 2, g_ready: bool = False,
                     x_ready: bool = False) -> bool:
    """Whether the weight gradient of a [out, in] linear over M tokens takes the
    reduction-contiguous (transposed-operand) path -- the predicate producers of pre-transposed
    operands check before offering one.  g_ready / x_ready: that operand is already available
    transposed, so it adds no transient copy."""
    if not WGRAD_NT or out_features * in_features < WGRAD_NT_MIN_NUMEL:
        return False
    if (WGRAD_SPLIT > 1 and M >= WGRAD_SPLIT_MIN_TOKENS and M % WGRAD_SPLIT == 0
            and -(-out_features // 256) * -(-in_features // 256) <= WGRAD_SPLIT_MAX_TILES):
        return False  # split-K path (_split_k)
    copies = (0 if g_ready else M * out_features) + (0 if x_ready else M * in_features)
    return copies * elem_size <= WGRAD_NT_MAX_BYTES


def _nt_operands(g2, x2, bias_grad, offer_gt=False):
    """(dy^T, x^T) contiguous along the tokens, with bias_grad (+)= sum(dy) folded into the
    transpose of dy; None when the path does not apply."""
    x_ready = x2.t().is_contiguous() and x2.stride(1) != 1
    g_ready = any(t.data_ptr() == g2.data_ptr() for t, _ in _pre_t)
    if not (g2.is_cuda and g2.dtype == x2.dtype
            and nt_wgrad_planned(g2.size(0), g2.size(1), x2.size(1), g2.element_size(), g_ready, x_ready)):
        return None
    if bias_grad is not None and (bias_grad.dtype != g2.dtype or not bias_grad.is_contiguous()):
        return None
    from . import native
    if not ((g_ready or native.transpose_supported(g2)) and (x_ready or native.transpose_supported(x2))):
        return None
    xt = _t_operand(x2)
    if xt is None:
        return None
    gt = _t_operand(g2, bias_grad, offer=offer_gt)
    if gt is None:
        return None
    _nt_count[0] += 1
    return gt, xt


def _split_k(g2, x2):
    """Number of token batches for the split-K weight gradient (1 = one plain GEMM)."""
    M, out, inp = g2.size(0), g2.size(1), x2.size(1)
    if (WGRAD_SPLIT <= 1 or not g2.is_cuda or M < WGRAD_SPLIT_MIN_TOKENS or M % WGRAD_SPLIT
            or not g2.is_contiguous() or not x2.is_contiguous()):
        return 1
    tiles = -(-out // 256) * -(-inp // 256)
    return WGRAD_SPLIT if tiles <= WGRAD_SPLIT_MAX_TILES else 1


def _wgrad_split(g2, x2, s, out=None):
    """dy^T x as s strided-batched partial GEMMs over token slices.  The partials are written
    in fp32 (hipBLASLt accumulates in fp32 and stores it: no bf16 rounding per partial) and
    folded by one HIP pass into `out` (accumulated: the bound gradient) or a fresh tensor."""
    M = g2.size(0)
    part = torch.bmm(g2.view(s, M // s, g2.size(1)).transpose(1, 2), x2.view(s, M // s, x2.size(1)),
                     out_dtype=torch.float32)
    from . import native
    if out is not None:
        return native.hip_ops().sum_slices(part, out, True)
    return native.hip_ops().sum_slices(part, torch.empty(part.shape[1:], dtype=g2.dtype, device=part.device),
                                       False)


def end_backward_pass():
    clear_transposed()


def input_grad(g2: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """dx = g2 @ W for g2 = dy [M, out], W [out, in]: from W^T [in, out] (one HIP transpose of the
    weight per use, reduction-contiguous operands for hipBLASLt) where that pays."""
    if (DGRAD_NT and g2.is_cuda and g2.dtype == weight.dtype and weight.numel() >= DGRAD_NT_MIN_NUMEL
            and g2.size(0) >= 1024):
        from . import native
        if native.transpose_supported(weight):
            return g2 @ native.transpose2d(weight).t()
    return g2 @ weight


def accumulate_param_grads(g2: torch.Tensor, x2: torch.Tensor, weight: torch.Tensor, bias, need_w: bool,
                           need_b: bool, offer_gt: bool = False):
    """Weight/bias gradients of y = x W^T (+ b) for flattened g2 = dy [M, out], x2 = x [M, in].
    offer_gt: another linear's weight gradient reads the same dy (parallel-residual branch
    outputs), so a transpose of dy made here is kept for it.

    Returns (dw, db) for autograd, or None entries for parameters whose gradient was
    accumulated in place."""
    dw = db = None
    has_b = bias is not None and need_b
    fuse = FUSE_WGRAD and need_w and (not has_b or _bound_grad(bias) is not None)
    gw = _bound_grad(weight) if fuse else None
    if (gw is not None and _wb.state.defer and (not has_b or bias.grad.is_contiguous()) and _wb.deferrable(g2, x2, gw)
            and _wb.in_slab(x2)):
        # run at the end of the backward, batched with the other layers' (ops/wgrad_batch.py)
        _wb.record(g2, x2, gw)
        if has_b:
            from . import native
            native.colsum(g2, bias.grad, accumulate=True)
        _count[0] += 1
        return None, None
    split = _split_k(g2, x2) if need_w else 1
    if split > 1:
        from . import native
        if gw is not None and gw.is_contiguous() and (not has_b or bias.grad.is_contiguous()):
            _wgrad_split(g2, x2, split, out=gw)
            if has_b:
                native.colsum(g2, bias.grad, accumulate=True)
            _count[0] += 1
            return None, None
        return _wgrad_split(g2, x2, split), (native.colsum(g2) if has_b else None)
    if gw is not None and gw.is_contiguous():
        nt = _nt_operands(g2, x2, bias.grad if has_b else None, offer_gt)
        if nt is not None:
            gw.addmm_(nt[0], nt[1].t())
        else:
            gw.addmm_(g2.t(), x2)
            if has_b:
                bias.grad.add_(g2.sum(0))
        _count[0] += 1
        # returning None still runs the leaf's AccumulateGrad node, which leaves the bound
        # gradient untouched and fires its post-accumulate hooks (ZeRO bucket bookkeeping)
        return None, None
    if need_w:
        db = torch.zeros(g2.size(1), dtype=g2.dtype, device=g2.device) if has_b else None
        nt = _nt_operands(g2, x2, db, offer_gt)
        if nt is not None:
            return nt[0] @ nt[1].t(), db
        dw = g2.t() @ x2
    if has_b:
        db = g2.sum(0)
    return dw, db


def wgrad_into(g2: torch.Tensor, x2: torch.Tensor, gw: torch.Tensor):
    """gw += g2^T x2 by the path accumulate_param_grads takes for a bound gradient without bias
    (split-K, a measured NT solution, transposed operands or one GEMM)."""
    split = _split_k(g2, x2)
    if split > 1 and gw.is_contiguous():
        _wgrad_split(g2, x2, split, out=gw)
    else:
        nt = _nt_operands(g2, x2, None) if gw.is_contiguous() else None
        if nt is None:
            gw.addmm_(g2.t(), x2)
        else:
            gw.addmm_(nt[0], nt[1].t())


def _lt_ops():
    """The HIP extension with the measured hipBLASLt solutions registered (ops/lt_tune.py)."""
    from . import lt_tune, native
    ops = native.hip_ops()
    lt_tune.register(ops)
    return ops


def _lt_ok(*ts) -> bool:
    return all(t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous() for t in ts)


def forward_gemm(x, weight, bias=None):
    """y = x W^T + b; through the hipBLASLt wrapper when the measured-solution table covers the
    problem (ops/lt_tune.py), else torch's F.linear."""
    if lt_tune.FWD and x.dim() >= 2 and _lt_ok(x, weight) and (bias is None or _lt_ok(bias)):
        M = x.numel() // x.shape[-1]
        if M > 0 and lt_tune.use_fwd(M, weight.shape[0], weight.shape[1], bias is not None):
            y = _lt_ops().linear_lt(x.view(M, x.shape[-1]), weight, bias, None, False, None)
            return y.view(*x.shape[:-1], weight.shape[0])
    return F.linear(x, weight, bias)


def _linear_backward(ctx, g):
    x, weight = ctx.saved_tensors
    bias = ctx.bias
    g2 = g.reshape(-1, g.shape[-1])
    x2 = x.reshape(-1, x.shape[-1])
    need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
    need_b = bias is not None and ctx.needs_input_grad[2]
    dx = input_grad(g2, weight).view(x.shape) if need_x else None
    dw, db = accumulate_param_grads(g2, x2, weight, bias, need_w, need_b, ctx.share_gt)
    return dx, dw, db, None


class _AccumLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, share_gt=False):
        ctx.save_for_backward(x, weight)
        ctx.bias = bias
        ctx.share_gt = share_gt
        return forward_gemm(x, weight, bias)

    @staticmethod
    def backward(ctx, g):
        return _linear_backward(ctx, g)


_ZERO = {}


def zero_placeholder(like: torch.Tensor, shape) -> torch.Tensor:
    """A zero-stride view of one cached zero element (per dtype / device) expanded to `shape`:
    the value of an output nobody reads.  Reusing the element avoids a one-element fill kernel
    per call (~600 launches per 20B step from the recompute's gradient-only ops)."""
    key = (like.dtype, like.device)
    z = _ZERO.get(key)
    if z is None:
        z = _ZERO[key] = torch.zeros(1, dtype=like.dtype, device=like.device)
    return z.expand(*shape)


class _GradOnlyLinear(torch.autograd.Function):
    """y = x W^T + b whose VALUE is never read: forward returns a zero-stride placeholder and
    costs nothing; backward produces the exact input / weight / bias gradients."""

    @staticmethod
    def forward(ctx, x, weight, bias, share_gt=False):
        ctx.save_for_backward(x, weight)
        ctx.bias = bias
        ctx.share_gt = share_gt
        return zero_placeholder(x, (*x.shape[:-1], weight.shape[0]))

    @staticmethod
    def backward(ctx, g):
        return _linear_backward(ctx, g)


def linear(x, weight, bias=None, share_grad_t=False):
    """F.linear whose weight gradient accumulates in place when a gradient is bound.
    share_grad_t: the output gradient is also another linear's (see accumulate_param_grads)."""
    if torch.is_grad_enabled() and weight.requires_grad:
        return _AccumLinear.apply(x, weight, bias, share_grad_t)
    return forward_gemm(x, weight, bias)


def grad_only_linear(x, weight, bias=None, share_grad_t=False):
    return _GradOnlyLinear.apply(x, weight, bias, share_grad_t)


class Linear(nn.Linear):
    """nn.Linear with in-place weight-gradient accumulation (state-dict compatible).

    `grad_only_next = True` makes the next call a gradient-only linear (its value is never
    read: selective recompute hands the consumer a kept copy of the output)."""

    grad_only_next = False

    def forward(self, x):
        if self.grad_only_next:
            self.grad_only_next = False
            return grad_only_linear(x, self.weight, self.bias)
        return linear(x, self.weight, self.bias)
