"""Python entry points for the native (HIP / C++) kernels.

Every GPU hot op in the framework goes through this module.  On a GPU tensor the HIP
extension is mandatory: if it cannot be built or imported the call raises (no silent
eager fallback).  CPU tensors (unit tests on the CPU-only CI host) use a PyTorch reference
implementation of the same math; that path is never taken for tensors on the MI355X.
"""

from __future__ import annotations

import math
from typing import Optional, Tuple

import torch

from . import builder

_hip = None
_flop_sink = None  # set by the FLOPs profiler while it is active: callable(macs)


def _macs(n):
    if _flop_sink is not None:
        _flop_sink(float(n))


def hip_ops():
    """The `_hip_ops` extension module (built in-tree on first use)."""
    global _hip
    if _hip is None:
        _hip = builder.load("_hip_ops")
    return _hip


_PIN_CODES = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.int16: 3, torch.int64: 4}


def pinned_zeros(numel: int, dtype=torch.float32) -> torch.Tensor:
    """Zero-filled page-locked host tensor of exactly `numel` elements (hipHostMalloc through the
    extension; torch's caching host allocator would round a 111 GB request up to 128 GiB).  A
    plain CPU tensor when no GPU is visible."""
    if not torch.cuda.is_available():
        return torch.zeros(numel, dtype=dtype)
    if numel * torch.empty(0, dtype=dtype).element_size() < (64 << 20) or dtype not in _PIN_CODES:
        return torch.zeros(numel, dtype=dtype, pin_memory=True)  # small: the caching allocator is fine
    return hip_ops().pinned_zeros(int(numel), _PIN_CODES[dtype])


def on_gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


# --------------------------------------------------------------------------- LayerNorm
def _ln_ref(x, gamma, beta, eps):
    xf = x.float()
    mean = xf.mean(-1, keepdim=True)
    var = (xf - mean).pow(2).mean(-1, keepdim=True)
    rstd = torch.rsqrt(var + eps)
    y = (xf - mean) * rstd * gamma.float()
    if beta is not None:
        y = y + beta.float()
    return y.to(x.dtype), mean.reshape(-1), rstd.reshape(-1)


def _ln_param_acc(ctx):
    """(gamma.grad, beta.grad) when both are bound gradient buffers the LN-backward column sums
    can accumulate into (the engine's p.grad views; ops/linear.py does the same for weights):
    autograd then gets None for them and its AccumulateGrad add over the parameter disappears."""
    from .linear import FUSE_WGRAD, _bound_grad
    g, b = ctx.params
    if not (FUSE_WGRAD and ctx.needs_input_grad[1]) or (b is not None and not ctx.needs_input_grad[2]):
        return None
    gg = _bound_grad(g)
    gb = _bound_grad(b) if b is not None else None
    if gg is None or not gg.is_contiguous() or (b is not None and (gb is None or not gb.is_contiguous())):
        return None
    return gg, gb


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, eps):
        x = x.contiguous()
        _macs(5 * x.numel())
        if x.is_cuda:
            y, mean, rstd, _ = hip_ops().ln_fwd(x, gamma, beta, eps, None, None)
        else:
            y, mean, rstd = _ln_ref(x, gamma, beta, eps)
        ctx.save_for_backward(x, gamma, mean, rstd)
        ctx.has_beta = beta is not None
        ctx.params = (gamma, beta)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, gamma, mean, rstd = ctx.saved_tensors
        dy = dy.contiguous()
        acc = _ln_param_acc(ctx) if x.is_cuda else None
        if acc is not None:
            dx, _, _ = hip_ops().ln_bwd(dy, x, gamma, mean, rstd, ctx.has_beta, None, acc[0], acc[1])
            return dx, None, None, None
        if x.is_cuda:
            dx, dg, db = hip_ops().ln_bwd(dy, x, gamma, mean, rstd, ctx.has_beta, None)
        else:
            H = x.shape[-1]
            xf = x.float().reshape(-1, H)
            g = dy.float().reshape(-1, H)
            xh = (xf - mean[:, None]) * rstd[:, None]
            dxh = g * gamma.float()
            dx = rstd[:, None] * (dxh - dxh.mean(-1, keepdim=True) - xh * (dxh * xh).mean(-1, keepdim=True))
            dx = dx.reshape(x.shape).to(x.dtype)
            dg = (g * xh).sum(0).to(gamma.dtype)
            db = g.sum(0).to(gamma.dtype) if ctx.has_beta else None
        return dx, dg, (db if ctx.has_beta else None), None


def _slab(spec, like, backward=False):
    """A layer slot of ops/wgrad_batch's stacked buffers for this output (spec = (kind, layer,
    layers)), or None for ordinary memory."""
    if spec is None or not like.is_cuda:
        return None
    from . import wgrad_batch
    return wgrad_batch.view(spec[0], spec[1], spec[2], like, backward)


def layer_norm(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], eps: float = 1e-5):
    return _LayerNormFn.apply(x, weight, bias, eps)


class _LayerNormResidualFn(torch.autograd.Function):
    """(LayerNorm(x), x) for a pre-LN block whose input also feeds the residual add: the second
    output is x itself, so the residual branch's gradient reaches this node and the LN-backward
    kernel adds it into dx in the same pass (reference LayerNormBackward*_fused_add,
    normalize_kernels.cu:1350-1790) instead of autograd summing the two branches separately."""

    @staticmethod
    def forward(ctx, x, gamma, beta, eps, y_slab=None):
        x = x.contiguous()
        _macs(5 * x.numel())
        if x.is_cuda:
            y, mean, rstd, _ = hip_ops().ln_fwd(x, gamma, beta, eps, None, None, _slab(y_slab, x))
        else:
            y, mean, rstd = _ln_ref(x, gamma, beta, eps)
        ctx.save_for_backward(x, gamma, mean, rstd)
        ctx.has_beta = beta is not None
        ctx.params = (gamma, beta)
        return y, x

    @staticmethod
    def backward(ctx, dy, dres):
        x, gamma, mean, rstd = ctx.saved_tensors
        if not x.is_cuda:
            dx, dg, db, _ = _LayerNormFn.backward(ctx, dy)
            return (dx if dres is None else dx + dres), dg, db, None, None
        dres = None if dres is None else dres.contiguous()
        acc = _ln_param_acc(ctx)
        if acc is not None:
            dx, _, _ = hip_ops().ln_bwd(dy.contiguous(), x, gamma, mean, rstd, ctx.has_beta, dres, acc[0], acc[1])
            return dx, None, None, None, None
        dx, dg, db = hip_ops().ln_bwd(dy.contiguous(), x, gamma, mean, rstd, ctx.has_beta, dres)
        return dx, dg, (db if ctx.has_beta else None), None, None


def layer_norm_residual(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], eps: float = 1e-5,
                        y_slab=None):
    """(LayerNorm(x), x): use the second output for the residual path (fused backward add).
    y_slab: (kind, layer, layers) slot of ops/wgrad_batch for the normalised output."""
    return _LayerNormResidualFn.apply(x, weight, bias, eps, y_slab)


class _InvertibleLayerNormFn(torch.autograd.Function):
    """LayerNorm that keeps only its OUTPUT for backward (reference `normalize_invertible`,
    csrc/transformer/normalize_kernels.cu invertible variants): x_hat = (y - beta) / gamma is
    recovered from y, so the layer input is not stored -- when y is saved anyway by the next
    GEMM, one [tokens, hidden] activation per LayerNorm less is held until backward.  The
    backward is the regular fused LN backward on x_hat (mean 0, rstd 1) scaled by the saved
    per-row rstd.  Needs gamma != 0 (as the reference)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, eps):
        x = x.contiguous()
        if x.is_cuda:
            y, mean, rstd, _ = hip_ops().ln_fwd(x, gamma, beta, eps, None, None)
        else:
            y, mean, rstd = _ln_ref(x, gamma, beta, eps)
        ctx.save_for_backward(y, gamma, beta if beta is not None else gamma.new_zeros(gamma.shape), rstd)
        ctx.has_beta = beta is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        y, gamma, beta, rstd = ctx.saved_tensors
        H = y.shape[-1]
        xhat = ((y.float() - beta.float()) / gamma.float()).to(y.dtype).reshape(-1, H)
        rows = xhat.shape[0]
        zero = torch.zeros(rows, dtype=torch.float32, device=y.device)
        one = torch.ones(rows, dtype=torch.float32, device=y.device)
        dyc = dy.contiguous().reshape(-1, H)
        if y.is_cuda:
            dx, dg, db = hip_ops().ln_bwd(dyc, xhat, gamma, zero, one, ctx.has_beta, None)
        else:
            xf, g = xhat.float(), dyc.float()
            gw = g * gamma.float()
            dx = (gw - gw.mean(-1, keepdim=True) - xf * (gw * xf).mean(-1, keepdim=True)).to(dy.dtype)
            dg = (g * xf).sum(0).to(gamma.dtype)
            db = g.sum(0).to(gamma.dtype) if ctx.has_beta else None
        dx = (dx.float() * rstd.reshape(-1, 1).float()).to(dy.dtype).reshape(dy.shape)
        return dx, dg, (db if ctx.has_beta else None), None


def layer_norm_invertible(x, weight, bias, eps: float = 1e-5):
    return _InvertibleLayerNormFn.apply(x, weight, bias, eps)


class FusedLayerNorm(torch.nn.Module):
    """LayerNorm on the HIP kernel (wave64 row reductions, fp32 statistics)."""

    def __init__(self, hidden: int, eps: float = 1e-5, elementwise_affine: bool = True, dtype=None, device=None):
        super().__init__()
        self.normalized_shape = (hidden,)
        self.eps = eps
        self.weight = torch.nn.Parameter(torch.ones(hidden, dtype=dtype, device=device))
        self.bias = torch.nn.Parameter(torch.zeros(hidden, dtype=dtype, device=device))

    def forward(self, x, residual_out: bool = False):
        """LayerNorm(x); with residual_out, (LayerNorm(x), x) where the second output carries the
        residual branch's gradient into the LN-backward kernel (layer_norm_residual)."""
        if residual_out:
            return layer_norm_residual(x, self.weight, self.bias, self.eps)
        return layer_norm(x, self.weight, self.bias, self.eps)

    def extra_repr(self):
        return f"{self.normalized_shape[0]}, eps={self.eps}"


# --------------------------------------------------------------------------- bias + GeLU
def _gelu_ref(x, approx):
    return torch.nn.functional.gelu(x, approximate="tanh" if approx else "none")


def _gelu_t_ok(x2: torch.Tensor) -> bool:
    """Shapes the transposing bias+GeLU kernels take (transpose.hip tile rules)."""
    return (x2.is_cuda and x2.dim() == 2 and x2.dtype in (torch.bfloat16, torch.float16) and x2.is_contiguous()
            and x2.size(0) % 128 == 0 and x2.size(1) % 64 == 0 and x2.size(0) > 0 and x2.data_ptr() % 16 == 0)


def _gelu_bwd(dy, x, bias, approx, offer_t, dx_out=None, db_acc=None):
    """(dx, db) of y = gelu(x + bias).  With offer_t, on the GPU one pass also writes dx^T and
    hands it to ops.linear as the pre-transposed output gradient of the linear that produced x
    (its weight gradient then skips the transpose of dx)."""
    C = x.shape[-1]
    if offer_t and DUAL_GELU_BWD and _gelu_t_ok(x.view(-1, C)) and dy.is_contiguous() \
            and (bias is None or bias.is_contiguous()):
        dx, dxt, db = hip_ops().bias_gelu_bwd_t(dy.view(-1, C), x.view(-1, C), bias, approx)
        from . import linear as _linear
        _linear.offer_transposed(dx, dxt)
        if db_acc is not None and db is not None:  # db_acc: the caller's bound bias gradient
            db = db_acc.add_(db)
        return dx.view(x.shape), db
    return hip_ops().bias_gelu_bwd(dy, x, bias, approx, dx_out, db_acc)


# the bias+GeLU backward also writes dx^T for the linear's weight gradient (False: dx only)
DUAL_GELU_BWD = True


class _BiasGeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, approx, offer_t=False, slabs=None):
        x = x.contiguous()
        _macs(2 * x.numel())
        if x.is_cuda:
            y = hip_ops().bias_gelu_fwd(x, bias, approx, _slab(slabs and slabs[0], x))
        else:
            y = _gelu_ref((x.float() + (bias.float() if bias is not None else 0)), approx).to(x.dtype)
        ctx.save_for_backward(x, bias)
        ctx.approx = approx
        ctx.offer_t = offer_t
        ctx.has_bias = bias is not None
        ctx.dx_slab = slabs and slabs[1]
        return y

    @staticmethod
    def backward(ctx, dy):
        x, bias = ctx.saved_tensors
        dy = dy.contiguous()
        if x.is_cuda:
            # a bound bias gradient (persistent, ops/wgrad_batch.py stacks) takes the column sums in place
            from .linear import FUSE_WGRAD, _bound_grad
            bacc = _bound_grad(bias) if (bias is not None and FUSE_WGRAD and ctx.needs_input_grad[1]) else None
            if bacc is not None and not bacc.is_contiguous():
                bacc = None
            dx, db = _gelu_bwd(dy, x, bias, ctx.approx, ctx.offer_t, _slab(ctx.dx_slab, x, backward=True), bacc)
            if bacc is not None:
                db = None
        else:
            with torch.enable_grad():
                xi = (x.float() + (bias.float() if bias is not None else 0)).detach().requires_grad_(True)
                y = _gelu_ref(xi, ctx.approx)
                (g,) = torch.autograd.grad(y, xi, dy.float())
            dx = g.to(x.dtype)
            db = g.reshape(-1, g.shape[-1]).sum(0).to(bias.dtype) if bias is not None else None
        return dx, (db if ctx.has_bias else None), None, None, None


def bias_gelu(x: torch.Tensor, bias: Optional[torch.Tensor], approximate: bool = False, offer_t: bool = False,
              slabs=None):
    """gelu(x + bias).  offer_t: x is the output of an ops.linear whose weight gradient takes
    the reduction-contiguous path -- the backward then also forms dx^T for it in the same pass.
    slabs: (y spec, dx spec) layer slots of ops/wgrad_batch for the output and its input gradient."""
    return _BiasGeluFn.apply(x, bias, approximate, offer_t, slabs)


class _BiasGeluTFn(torch.autograd.Function):
    """gelu(x + bias) returned TRANSPOSED, [C, M] for x [M, C] (one tiled HIP pass)."""

    @staticmethod
    def forward(ctx, x2, bias, approx):
        _macs(2 * x2.numel())
        yt = hip_ops().bias_gelu_fwd_t(x2, bias, approx)
        ctx.save_for_backward(x2, bias)
        ctx.approx = approx
        ctx.has_bias = bias is not None
        return yt

    @staticmethod
    def backward(ctx, dyt):
        x2, bias = ctx.saved_tensors
        dx, db = _gelu_bwd(dyt.t().contiguous(), x2, bias, ctx.approx, True)
        return dx, (db if ctx.has_bias else None), None


def bias_gelu_t_supported(x: torch.Tensor) -> bool:
    return _gelu_t_ok(x.reshape(-1, x.shape[-1])) if x.is_cuda and x.is_contiguous() else False


def bias_gelu_colmajor(x: torch.Tensor, bias: Optional[torch.Tensor], approximate: bool = False) -> torch.Tensor:
    """gelu(x + bias) with the value of bias_gelu but stored column-major: a [..., C] view of a
    contiguous [C, M] tensor.  For a consumer that only needs y^T -- the gradient-only fc2 of an
    activation recompute, whose weight gradient reads its input transposed -- this saves the
    separate transpose.  (Any reader of y gets the right values, only slower.)"""
    C = x.shape[-1]
    yt = _BiasGeluTFn.apply(x.reshape(-1, C), bias, approximate)
    return yt.t().view(*x.shape[:-1], C)


class _Add3Fn(torch.autograd.Function):
    """a + b (+ c) in one HIP pass (residual sums); the gradient passes to every summand."""

    @staticmethod
    def forward(ctx, a, b, c):
        ctx.n = 2 if c is None else 3
        return hip_ops().add3(a.contiguous(), b.contiguous(), None if c is None else c.contiguous())

    @staticmethod
    def backward(ctx, g):
        return (g, g, g if ctx.n == 3 else None)


def add3(a: torch.Tensor, b: torch.Tensor, c: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Fused residual sum on the GPU (one read of each input, one write); plain adds elsewhere."""
    vn = 4 if a.dtype == torch.float32 else 8
    if (a.is_cuda and a.shape == b.shape and a.dtype == b.dtype and a.numel() % vn == 0
            and (c is None or (c.shape == a.shape and c.dtype == a.dtype))):
        return _Add3Fn.apply(a, b, c)
    return a + b if c is None else a + b + c


# --------------------------------------------------------------------------- reductions
_WS = {}


def _workspace(device, n=2048):
    key = (device, n)
    ws = _WS.get(key)
    if ws is None:
        ws = torch.empty(n, dtype=torch.float32, device=device)
        _WS[key] = ws
    return ws


_SUMSQ_CHUNK = 65536
_sumsq_meta = {}


def sumsq_multi_(tensors, out: torch.Tensor):
    """out[0] += sum of squares of every tensor (one dtype, one device, contiguous) in two HIP
    launches (multi-tensor partials + finish); CPU tensors fall back to torch."""
    tensors = [t for t in tensors if t.numel() > 0]
    if not tensors:
        return out
    t0 = tensors[0]
    if not t0.is_cuda:
        for t in tensors:
            out += t.float().square().sum()
        return out
    code = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}[t0.dtype]
    key = tuple(t.data_ptr() for t in tensors) + tuple(t.numel() for t in tensors)
    hit = _sumsq_meta.get(key)
    if hit is None:
        numels = [t.numel() for t in tensors]
        pref = [0]
        for n in numels:
            pref.append(pref[-1] + (n + _SUMSQ_CHUNK - 1) // _SUMSQ_CHUNK)
        rows = [t.data_ptr() for t in tensors] + numels + pref
        # pinned staging + async copy (a pageable H2D copy would wait for the stream)
        meta = torch.tensor(rows, dtype=torch.int64).pin_memory().to(t0.device, non_blocking=True)
        hit = (meta, len(tensors), pref[-1], torch.empty(pref[-1], dtype=torch.float32, device=t0.device))
        if len(_sumsq_meta) > 64:
            _sumsq_meta.clear()
        _sumsq_meta[key] = hit
    meta, nt, total, partial = hit
    # the cache may drop these on a later call while this stream still reads them: tie their
    # reuse to the stream that consumes them (the norm can run on an overlap / side stream)
    cur = torch.cuda.current_stream(t0.device)
    meta.record_stream(cur)
    partial.record_stream(cur)
    hip_ops().sumsq_multi(meta, nt, total, _SUMSQ_CHUNK, code, partial, out)
    return out


def sumsq_accumulate(x: torch.Tensor, out: torch.Tensor):
    """out[0] += sum(x.float()**2) without a host sync (HIP on GPU)."""
    if x.numel() == 0:
        return out
    if x.is_cuda:
        if x.data_ptr() % 16 != 0 or not x.is_contiguous():
            out.add_(x.float().pow(2).sum())
        else:
            hip_ops().sumsq_accum(x, _workspace(x.device), out)
    else:
        out.add_(x.float().pow(2).sum())
    return out


def colsum(x: torch.Tensor, out: Optional[torch.Tensor] = None, accumulate: bool = False) -> torch.Tensor:
    """Column sums of x [..., C] (fp32 accumulation) into a fresh [C] tensor, or into `out`
    (added to it when `accumulate`)."""
    if x.is_cuda:
        return hip_ops().colsum(x.contiguous(), out, accumulate)
    r = x.reshape(-1, x.shape[-1]).float().sum(0)
    if out is None:
        return r.to(x.dtype)
    if accumulate:
        r += out.float()
    return out.copy_(r)


def transpose_supported(x: torch.Tensor) -> bool:
    """Shapes/layouts the HIP transpose takes: 2-D 16-bit, rows % 128, cols % 64, unit column
    stride, 16-byte aligned rows."""
    return (x.dim() == 2 and x.dtype in (torch.bfloat16, torch.float16) and x.size(0) % 128 == 0
            and x.size(1) % 64 == 0 and x.size(0) > 0 and x.size(1) > 0 and x.stride(1) == 1
            and x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0)


def transpose2d(x: torch.Tensor, colsum_out: Optional[torch.Tensor] = None, accum: bool = False,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """x [R, C] -> contiguous x^T [C, R] (into `out` when given); optionally colsum_out (+)= x.sum(0)
    from the same read (the bias gradient of a linear whose output gradient is x)."""
    if x.is_cuda:
        return hip_ops().transpose2d(x, colsum_out, accum, out)
    y = x.t().contiguous() if out is None else out.copy_(x.t())
    if colsum_out is not None:
        s = x.float().sum(0)
        if accum:
            s += colsum_out.float()
        colsum_out.copy_(s)
    return y


# --------------------------------------------------------------------------- Adam
def adam_flat_(w, g, m, v, out, lr, beta1, beta2, eps, weight_decay, step, bias_correction, grad_scale, adamw):
    """In-place Adam/AdamW on flat tensors.  `w` is the fp32 master (or the param itself),
    `out` an optional low-precision model copy refreshed in the same pass."""
    bc1 = 1.0 - beta1 ** step if bias_correction else 1.0
    bc2 = 1.0 - beta2 ** step if bias_correction else 1.0
    if w.is_cuda:
        hip_ops().adam_flat(w, g, m, v, out, lr, beta1, beta2, eps, weight_decay, bc1, bc2, grad_scale, adamw)
        return
    # CPU reference (tests on CPU CI): identical math in fp32
    gf = g.float() * grad_scale
    wf = w.float()
    if not adamw and weight_decay != 0:
        gf = gf + weight_decay * wf
    m.mul_(beta1).add_(gf, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(gf, gf, value=1 - beta2)
    upd = (m / bc1) / ((v / bc2).sqrt() + eps)
    if adamw and weight_decay != 0:
        upd = upd + weight_decay * wf
    wf = wf - lr * upd
    w.copy_(wf)
    if out is not None:
        out.copy_(wf)


def adam_compact_(hi, res, g, m, v, lr, beta1, beta2, eps, weight_decay, step, bias_correction, grad_scale, adamw):
    """Adam/AdamW on a compact master: `hi` (bf16 model weights) + `res` (int16 residual) hold
    the exact fp32 master (runtime/zero/compact_master.py); both are updated in place."""
    bc1 = 1.0 - beta1 ** step if bias_correction else 1.0
    bc2 = 1.0 - beta2 ** step if bias_correction else 1.0
    if hi.is_cuda:
        hip_ops().adam_compact(hi, res, g, m, v, lr, beta1, beta2, eps, weight_decay, bc1, bc2, grad_scale, adamw)
        return
    from ..runtime.zero import compact_master as cm
    w = cm.decode(hi, res)
    adam_flat_(w, g, m, v, None, lr, beta1, beta2, eps, weight_decay, step, bias_correction, grad_scale, adamw)
    h, r = cm.encode(w)
    hi.copy_(h)
    res.copy_(r)


def copy_narrow_(dst: torch.Tensor, src: torch.Tensor, wgs: int = 16):
    """dst <- src on `wgs` workgroups (HBM -> pinned host at the PCIe rate without a workgroup on
    every CU); falls back to copy_ for unaligned tensors."""
    if (dst.data_ptr() | src.data_ptr()) & 15:
        return dst.copy_(src, non_blocking=True)
    hip_ops().copy_narrow(dst, src, wgs)
    return dst


def copy_nocu_(dst: torch.Tensor, src: torch.Tensor, kind: int = -1):
    """dst <- src (same bytes; device or pinned host tensors) on the current stream with one
    hipMemcpyAsync of the given hipMemcpyKind (default -1: hipMemcpyDeviceToDeviceNoCU, a DMA
    engine instead of a copy kernel)."""
    hip_ops().copy_nocu(dst, src, kind)
    return dst


def scale_copy_(x: torch.Tensor, y: torch.Tensor, scale: float = 1.0, scale_tensor: Optional[torch.Tensor] = None,
                accumulate: bool = False):
    """y = x * scale (accumulate: y += x * scale), one pass for any dtype pair."""
    if x.is_cuda and x.data_ptr() % (x.element_size() * 4) == 0 and y.data_ptr() % (y.element_size() * 4) == 0:
        hip_ops().scale_copy(x, y, scale_tensor, scale, accumulate)
    else:
        s = scale if scale_tensor is None else scale * scale_tensor.float()
        if accumulate:
            y.add_((x.float() * s).to(y.dtype))
        else:
            y.copy_(x.float() * s)
    return y


# --------------------------------------------------------------------------- flash attention
def has_flash_attention(q: torch.Tensor) -> bool:
    """True when the fused MFMA attention kernel supports this problem."""
    if not q.is_cuda or q.dtype not in (torch.bfloat16, torch.float16):
        return False
    mod = hip_ops()
    return hasattr(mod, "flash_attn_fwd") and q.shape[-1] in (64, 96, 128)


class _FlashAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale, out_bshd):
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        B, H, S, D = q.shape
        _macs(2 * B * H * S * S * D * (0.5 if causal else 1.0))
        o, lse = hip_ops().flash_attn_fwd(q, k, v, causal, scale, out_bshd)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.scale, ctx.out_bshd = causal, scale, out_bshd
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        dq, dk, dv = hip_ops().flash_attn_bwd(do.contiguous(), q, k, v, o, lse, ctx.causal, ctx.scale, ctx.out_bshd)
        return dq, dk, dv, None, None, None


class _StashedFlashAttnFn(_FlashAttnFn):
    """Recompute-time stand-in: (o, lse) kept from the first forward; backward unchanged."""

    @staticmethod
    def forward(ctx, q, k, v, causal, scale, out_bshd, stash):
        o, lse = stash
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.scale, ctx.out_bshd = causal, scale, out_bshd
        return o

    @staticmethod
    def backward(ctx, do):
        return _FlashAttnFn.backward(ctx, do) + (None,)


def flash_attention(q, k, v, causal=True, scale=1.0, out_layout="bhsd", stash=None):
    """q, k, v [B, H, S, D] -> o [B, H, S, D] (out_layout "bhsd") or [B, S, H, D] ("bshd": the
    token-major layout the output projection reads, written directly by the kernel).
    stash: (o, lse) from flash_attention_fwd_lse of the same inputs (selective recompute)."""
    assert out_layout in ("bhsd", "bshd")
    if stash is not None:
        return _StashedFlashAttnFn.apply(q, k, v, causal, scale, out_layout == "bshd", tuple(stash))
    return _FlashAttnFn.apply(q, k, v, causal, scale, out_layout == "bshd")


class _FlashAttnExFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, kbias, scale, p, seed, out_bshd):
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        B, H, S, D = q.shape
        _macs(2 * B * H * S * S * D)
        o, lse = hip_ops().flash_attn_fwd_ex(q, k, v, kbias, scale, p, seed, out_bshd)
        ctx.save_for_backward(q, k, v, o, lse, kbias)
        ctx.scale, ctx.p, ctx.seed, ctx.out_bshd = scale, p, seed, out_bshd
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, kbias = ctx.saved_tensors
        dq, dk, dv = hip_ops().flash_attn_bwd_ex(do.contiguous(), q, k, v, o, lse, kbias, ctx.scale, ctx.p, ctx.seed,
                                                 ctx.out_bshd)
        return dq, dk, dv, None, None, None, None, None


def encoder_flash_supported(q: torch.Tensor, key_bias_ok: bool = True) -> bool:
    """Shapes the encoder flash kernel (key bias + in-kernel dropout) handles."""
    return (key_bias_ok and q.is_cuda and q.dtype in (torch.bfloat16, torch.float16) and q.dim() == 4
            and q.shape[-1] in (64, 128) and q.shape[2] % 8 == 0)


def flash_attention_encoder(q, k, v, key_bias=None, scale=1.0, dropout_p=0.0, training=True, generator=None,
                            out_layout="bhsd"):
    """Non-causal attention softmax(scale * q k^T + key_bias[b, None, :]) with dropout on the
    probabilities, fused in one MFMA kernel per direction (no S x S tensor is stored; the keep mask
    is a hash of (seed, head, query, key) regenerated in backward).  q, k, v [B, H, S, D];
    key_bias [B, S] (any float dtype; the reference's additive [B,1,1,S] mask squeezed)."""
    assert out_layout in ("bhsd", "bshd")
    p = float(dropout_p) if training else 0.0
    if key_bias is not None:
        key_bias = key_bias.reshape(q.shape[0], q.shape[2]).float().contiguous()
    if key_bias is None and p <= 0.0:
        return flash_attention(q, k, v, False, scale, out_layout)
    seed = _draw_seed(generator) if p > 0.0 else 0
    return _FlashAttnExFn.apply(q, k, v, key_bias, float(scale), p, int(seed) & ((1 << 63) - 1),
                                out_layout == "bshd")


class _FlashAttnQkvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv5, kbias, scale, p, seed, rng=None, slabs=None):
        B, S, _, H, D = qkv5.shape
        _macs(2 * B * H * S * S * D)
        o_out = _slab(slabs and slabs[0], qkv5[:, :, 0])
        o, lse = hip_ops().flash_attn_qkv_fwd(qkv5, kbias, scale, p, seed, rng, o_out)
        ctx.save_for_backward(qkv5, o, lse, kbias)
        ctx.scale, ctx.p, ctx.seed, ctx.rng = scale, p, seed, rng
        ctx.dqkv_slab = slabs and slabs[1]
        return o

    @staticmethod
    def backward(ctx, do):
        qkv5, o, lse, kbias = ctx.saved_tensors
        dqkv = hip_ops().flash_attn_qkv_bwd(do.contiguous(), qkv5, o, lse, kbias, ctx.scale, ctx.p, ctx.seed,
                                            ctx.rng, _slab(ctx.dqkv_slab, qkv5, backward=True))
        return dqkv, None, None, None, None, None, None


_KB_CACHE = []  # [(source tensor, its key, fp32 [B, S] copy)]: the last conversion


def _fp32_key_bias(key_bias, B, S):
    """key_bias as a contiguous fp32 [B, S]: the conversion of the mask every layer of a forward
    passes is made once and reused while the same (unmodified) tensor comes back -- one launch per
    forward instead of one per layer.  Holding the source keeps its storage from being recycled."""
    if key_bias.dtype == torch.float32 and key_bias.is_contiguous():
        return key_bias.reshape(B, S)
    if key_bias.is_cuda and torch.cuda.is_current_stream_capturing():
        return key_bias.reshape(B, S).float().contiguous()  # a graph may only bake in its own buffers
    # every layer passes a fresh view of the same mask: match on storage, layout and version
    key = (key_bias.data_ptr(), key_bias.dtype, key_bias.device, tuple(key_bias.shape), key_bias.stride(),
           key_bias._version, B, S)
    if _KB_CACHE and _KB_CACHE[0][1] == key:
        return _KB_CACHE[0][2]
    out = key_bias.reshape(B, S).float().contiguous()
    _KB_CACHE[:] = [(key_bias, key, out)]
    return out


def flash_attention_qkv(qkv, num_heads, key_bias=None, scale=1.0, dropout_p=0.0, training=True, generator=None,
                        rng=None, site=0, slabs=None):
    """Encoder attention straight from the fused QKV projection: qkv [B, S, 3*H*D] (q | k | v,
    heads contiguous inside each) -> context [B, S, H*D], same math as flash_attention_encoder
    (same keep mask for the same seed) without the head split / merge copies; the backward
    returns dqkv in the qkv layout."""
    B, S, C = qkv.shape
    D = C // (3 * num_heads)
    p = float(dropout_p) if training else 0.0
    if key_bias is not None:
        key_bias = _fp32_key_bias(key_bias, B, S)
    if rng is not None:  # device [seed, step] (graph-replayable): the host value only names the call site
        seed = site
    else:
        seed = (_draw_seed(generator) if p > 0.0 else 0) & ((1 << 63) - 1)
    o = _FlashAttnQkvFn.apply(qkv.contiguous().view(B, S, 3, num_heads, D), key_bias, float(scale), p, int(seed),
                              rng if p > 0.0 else None, slabs)
    return o.view(B, S, num_heads * D)


def qkv_flash_supported(qkv: torch.Tensor, num_heads: int) -> bool:
    if not (qkv.is_cuda and qkv.dtype in (torch.bfloat16, torch.float16) and qkv.dim() == 3):
        return False
    B, S, C = qkv.shape
    return C % (3 * num_heads) == 0 and C // (3 * num_heads) in (64, 128) and S % 8 == 0


def flash_dropout_keep_mask(B, H, S, p, seed, device=None):
    """Host/torch re-implementation of the kernel's keep mask ([B, H, S, S] bool), for tests."""
    M = 0xFFFFFFFF

    def mix(x):
        x = x ^ (x >> 16)
        x = (x * 0x7FEB352D) & M
        x = x ^ (x >> 15)
        x = (x * 0x846CA68B) & M
        return x ^ (x >> 16)

    s32 = (int(seed) ^ (int(seed) >> 32)) & M
    thresh = min(65536, int(round(p * 65536))) if p > 0 else 0
    bh = torch.arange(B * H, dtype=torch.int64, device=device)
    hb = mix(s32 ^ mix((bh * 0x9E3779B1 + 0x632BE5AB) & M))  # [BH]
    q = torch.arange(S, dtype=torch.int64, device=device)
    j = torch.arange(S // 2, dtype=torch.int64, device=device)
    idx = (q[:, None] * (S // 2) + j[None, :]) & M  # [S, S/2]
    x = mix(((idx * 0x85EBCA6B) & M)[None] ^ hb[:, None, None])  # [BH, S, S/2]
    draws = torch.stack([x & 0xFFFF, x >> 16], dim=-1).reshape(B, H, S, S)
    return draws >= thresh


def flash_attention_fwd_lse(q, k, v, causal=True, scale=1.0, out_layout="bhsd"):
    """Forward only (no autograd): (o, lse) with lse [B*H, S] fp32, for a later stashed backward."""
    q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
    B, H, S, D = q.shape
    _macs(2 * B * H * S * S * D * (0.5 if causal else 1.0))
    return hip_ops().flash_attn_fwd(q, k, v, causal, scale, out_layout == "bshd")


# --------------------------------------------------------------------------- flatten
def _cpu_flatten():
    """(flatten, unflatten) pair: native C++ ops when built, torch._utils otherwise."""
    try:
        mod = builder.load("_cpu_ops")
        if hasattr(mod, "flatten"):
            return mod.flatten, mod.unflatten
    except Exception:
        pass
    from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors
    return _flatten_dense_tensors, _unflatten_dense_tensors


# --------------------------------------------------------------------------- fused LM loss
class _CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, inplace_grad=False):
        ctx.inplace = inplace_grad and logits.is_contiguous()
        x = logits.reshape(-1, logits.shape[-1]).contiguous()
        lab = labels.reshape(-1).contiguous()
        _macs(3 * x.numel())
        rows, lse = hip_ops().xent_fwd(x, lab)
        nvalid = (lab >= 0).sum().clamp_min(1).float()
        ctx.save_for_backward(x, lab, lse, nvalid)
        ctx.shape = logits.shape
        return rows.sum() / nvalid

    @staticmethod
    def backward(ctx, g):
        x, lab, lse, nvalid = ctx.saved_tensors
        # caller-owned logits (inplace_grad: nothing else reads them) are dead once their gradient
        # exists, so it is written over them (one [tokens, vocab] buffer instead of two at the
        # head of backward); the version bump makes a second backward through this graph fail
        # loudly instead of reading gradients as logits
        inplace = XENT_INPLACE and ctx.inplace
        dx = hip_ops().xent_bwd(x, lab, lse, (g.float() / nvalid).reshape(1).contiguous(), inplace)
        if inplace:
            torch.autograd.graph.increment_version(x)
        return dx.view(ctx.shape), None, None


# the cross-entropy backward writes dlogits over the logits (False: into a fresh buffer)
XENT_INPLACE = True


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor, inplace_grad: bool = False) -> torch.Tensor:
    """Mean token cross-entropy (labels < 0 ignored) on 16-bit logits without fp32 copies
    of the [tokens, vocab] tensor; fp32 PyTorch path on CPU / fp32 logits.  inplace_grad: the
    caller guarantees nothing reads `logits` after the backward (an LM head's internal output),
    so their gradient may overwrite them."""
    if logits.is_cuda and logits.dtype in (torch.bfloat16, torch.float16) and logits.shape[-1] % 8 == 0:
        return _CrossEntropyFn.apply(logits, labels, inplace_grad)
    return torch.nn.functional.cross_entropy(logits.float().reshape(-1, logits.shape[-1]), labels.reshape(-1),
                                             ignore_index=-100)


# --------------------------------------------------------------------------- LAMB
def lamb_(w, g, m, v, out, lr, beta1, beta2, eps, weight_decay, step, bias_correction, grad_scale, max_coeff,
          min_coeff, eps_outside_sqrt=True, coeff_out=None):
    """One LAMB step on one tensor (reference semantics, fused_lamb_cuda_kernel.cu:185-310):
    u = m/(sqrt(v)+eps) + wd*w, coeff = clamp(|w|/|u|, min, max) (1 if either norm is 0),
    w -= lr*sqrt(bc2)/bc1 * coeff * u.  Returns the coefficient as a 1-element fp32 tensor
    (device-resident on GPU: no host sync)."""
    bc1 = 1.0 - beta1 ** step if bias_correction else 1.0
    bc2 = 1.0 - beta2 ** step if bias_correction else 1.0
    step_size = lr * math.sqrt(bc2) / bc1
    if coeff_out is None:
        coeff_out = torch.empty(1, dtype=torch.float32, device=w.device)
    if w.is_cuda:
        upd = torch.empty(w.numel(), dtype=torch.float32, device=w.device)
        hip_ops().lamb(w, g, m, v, upd, out, step_size, beta1, beta2, eps, weight_decay, bc1, bc2, grad_scale,
                       max_coeff, min_coeff, bool(eps_outside_sqrt), _workspace(w.device, 4096), coeff_out)
        return coeff_out
    gf = g.float() * grad_scale
    m.mul_(beta1).add_(gf, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(gf, gf, value=1 - beta2)
    denom = v.sqrt().add_(eps) if eps_outside_sqrt else (v + eps).sqrt()
    wf = w.float()
    u = m / denom + weight_decay * wf
    wn, un = wf.norm(), u.norm()
    c = torch.where((wn > 0) & (un > 0), (wn / un).clamp(min_coeff, max_coeff), torch.ones_like(wn))
    w.copy_(wf - step_size * c * u)
    if out is not None:
        out.copy_(w)
    coeff_out.copy_(c.reshape(1))
    return coeff_out


# --------------------------------------------------------------------------- 1-bit compression
_BITW = None


def _packbits(bits: torch.Tensor) -> torch.Tensor:
    global _BITW
    if _BITW is None:
        _BITW = torch.tensor([128, 64, 32, 16, 8, 4, 2, 1], dtype=torch.int32)
    return (bits.view(-1, 8).to(torch.int32) * _BITW.to(bits.device)).sum(1).to(torch.uint8)


def _unpackbits(packed: torch.Tensor) -> torch.Tensor:
    """uint8 [..., nb] -> float +-1 [..., nb*8] (MSB first)."""
    shifts = torch.arange(7, -1, -1, device=packed.device, dtype=torch.int32)
    bits = (packed.to(torch.int32).unsqueeze(-1) >> shifts) & 1
    return bits.reshape(*packed.shape[:-1], -1).float().mul_(2).sub_(1)


def _ef_pack(c: torch.Tensor, err: torch.Tensor):
    scale = c.norm() / math.sqrt(c.numel())
    pos = c >= 0
    err.copy_(c - scale * (pos.float() * 2 - 1))
    return _packbits(pos), scale.reshape(1).float()


def onebit_worker_compress(m: torch.Tensor, err: torch.Tensor):
    """Error-compensated sign compression of `m` (fp32, numel % 8 == 0); updates `err`.
    Returns (packed uint8 [n/8], scale fp32 [1])."""
    if m.is_cuda:
        return tuple(hip_ops().onebit_worker_compress(m, err, _workspace(m.device, 2048)))
    return _ef_pack(m + err, err)


def onebit_server_compress(signs: torch.Tensor, scales: torch.Tensor, server_err: torch.Tensor):
    """Average P received sign chunks (signs uint8 [P*nb], scales [P]) into the server chunk,
    add the server error, re-compress.  Returns (packed [nb], scale [1])."""
    if signs.is_cuda:
        return tuple(hip_ops().onebit_server_compress(signs, scales, server_err, _workspace(signs.device, 2048)))
    P = scales.numel()
    vals = _unpackbits(signs.view(P, -1)) * scales.view(P, 1)
    return _ef_pack(server_err + vals.sum(0) / P, server_err)


def onebit_unpack(signs: torch.Tensor, scales: torch.Tensor, out: torch.Tensor):
    if signs.is_cuda:
        hip_ops().onebit_unpack(signs, scales, out)
        return out
    P = scales.numel()
    out.copy_((_unpackbits(signs.view(P, -1)) * scales.view(P, 1)).view(-1))
    return out


# --------------------------------------------------------------------------- dropout (Philox)
def _draw_seed(generator=None):
    """64-bit seed from a CPU generator (the default one is saved/restored by activation
    checkpointing, so recomputation replays the same masks)."""
    return int(torch.randint(0, 2 ** 62, (1,), generator=generator).item())


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed, rng=None):
        if x.is_cuda:
            y, mask = hip_ops().dropout_fwd(x.contiguous(), p, seed, 0, rng)
        else:
            g = torch.Generator().manual_seed(seed)
            mask = (torch.rand(x.shape, generator=g) >= p).to(torch.uint8)
            y = (x.float() * mask / (1 - p)).to(x.dtype)
        ctx.save_for_backward(mask)
        ctx.p = p
        return y

    @staticmethod
    def backward(ctx, dy):
        (mask,) = ctx.saved_tensors
        if dy.is_cuda:
            return hip_ops().dropout_bwd(dy.contiguous(), mask, ctx.p), None, None, None
        return (dy.float() * mask / (1 - ctx.p)).to(dy.dtype), None, None, None


def dropout(x, p, training=True, generator=None, rng=None, site=0):
    """rng: optional device int64 [seed, step] read by the kernel (graph-replayable masks, see
    DeepSpeedTransformerLayer.enable_device_rng); the host part of the seed is then the
    constant `site`, never a host draw, which a captured graph would freeze."""
    if not training or p <= 0:
        return x
    if rng is not None and x.is_cuda:
        return _DropoutFn.apply(x, float(p), int(site) << 20, rng)
    return _DropoutFn.apply(x, float(p), _draw_seed(generator))


class _DropoutMatmulFn(torch.autograd.Function):
    """out = dropout(probs) @ v without storing the dropped probabilities (reference
    `attn_dropout_checkpoint`, ds_transformer_cuda.cpp:185-193): backward re-applies the saved
    1-byte mask to the saved probs, so one [B, heads, S, S] activation per layer is not held."""

    @staticmethod
    def forward(ctx, probs, v, p, seed):
        if probs.is_cuda:
            pd, mask = hip_ops().dropout_fwd(probs.contiguous(), p, seed, 0)
        else:
            g = torch.Generator().manual_seed(seed)
            mask = (torch.rand(probs.shape, generator=g) >= p).to(torch.uint8)
            pd = (probs.float() * mask / (1 - p)).to(probs.dtype)
        v = v.contiguous()  # a view of a fused qkv buffer would keep all of it alive
        out = torch.matmul(pd, v)
        ctx.save_for_backward(probs, mask, v)
        ctx.p = p
        return out

    @staticmethod
    def backward(ctx, dout):
        probs, mask, v = ctx.saved_tensors
        p = ctx.p
        if probs.is_cuda:  # mask * probs / (1 - p): the dropout-backward kernel applied to probs
            pd = hip_ops().dropout_bwd(probs.contiguous(), mask, p)
        else:
            pd = (probs.float() * mask / (1 - p)).to(probs.dtype)
        dv = torch.matmul(pd.transpose(-1, -2), dout)
        dpd = torch.matmul(dout, v.transpose(-1, -2))
        if dpd.is_cuda:
            dprobs = hip_ops().dropout_bwd(dpd.contiguous(), mask, p)
        else:
            dprobs = (dpd.float() * mask / (1 - p)).to(dpd.dtype)
        return dprobs, dv, None, None


def dropout_matmul(probs, v, p, training=True, generator=None):
    """dropout(probs, p) @ v, recomputing the dropped probabilities in backward."""
    if not training or p <= 0:
        return torch.matmul(probs, v)
    return _DropoutMatmulFn.apply(probs, v, float(p), _draw_seed(generator))


class _BiasDropoutResidualFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, res, p, seed, rng=None):
        if x.is_cuda:
            y, mask = hip_ops().bias_dropout_residual(x.contiguous(), bias, res.contiguous(), p, seed, 0, rng)
        else:
            g = torch.Generator().manual_seed(seed)
            mask = (torch.rand(x.shape, generator=g) >= p).to(torch.uint8)
            y = (res.float() + (x.float() + bias.float()) * mask / (1 - p)).to(x.dtype)
        ctx.save_for_backward(mask)
        ctx.p = p
        return y

    @staticmethod
    def backward(ctx, dy):
        (mask,) = ctx.saved_tensors
        if dy.is_cuda:
            dy = dy.contiguous()
            if dy.shape[-1] % (4 if dy.dtype == torch.float32 else 8) == 0 and dy.data_ptr() % 16 == 0:
                dx, db = hip_ops().dropout_bwd_db(dy, mask, ctx.p)  # bias gradient in the same pass
            else:
                dx = hip_ops().dropout_bwd(dy, mask, ctx.p)
                db = colsum(dx.reshape(-1, dx.shape[-1]))
        else:
            dx = (dy.float() * mask / (1 - ctx.p)).to(dy.dtype)
            db = dx.reshape(-1, dx.shape[-1]).float().sum(0).to(dy.dtype)
        return dx, db, dy, None, None, None


def bias_dropout_residual(x, bias, residual, p, training=True, generator=None, rng=None, site=0):
    """residual + dropout(x + bias), one fused pass (reference dropout_kernels.cu ForwardWithBias).
    rng: device int64 [seed, step] read by the kernel (graph-replayable masks); `site` then
    separates the call sites that share it."""
    if not training or p <= 0:
        return residual + (x + bias)
    if rng is not None and x.is_cuda:
        return _BiasDropoutResidualFn.apply(x, bias, residual, float(p), int(site) << 20, rng)
    return _BiasDropoutResidualFn.apply(x, bias, residual, float(p), _draw_seed(generator))


class _BiasDropoutResidualLNFn(torch.autograd.Function):
    """(LayerNorm(out), out) with out = res + dropout(x + bias): the residual sum and the LayerNorm
    of a pre-LN block in one HIP pass (ops/csrc/kernels/dropout.hip bdr_ln_*), and in backward the
    LayerNorm backward, the residual-gradient add, the dropout backward and the gamma / beta /
    bias column sums in one pass plus one fold.  `out` is returned for the residual path, like
    layer_norm_residual.  Reference: the fused bias-residual-LayerNorm of
    csrc/transformer/normalize_kernels.cu (fused_bias_residual_layer_norm) fed by
    dropout_kernels.cu ForwardWithBias, ds_transformer_cuda.cpp:224-240."""

    @staticmethod
    def forward(ctx, x, bias, res, gamma, beta, p, eps, seed, rng, slabs=None):
        y, out, mask, mean, rstd = hip_ops().bdr_ln_fwd(x, bias, res, gamma, beta, p, eps, seed, 0, rng,
                                                        _slab(slabs and slabs[0], x))
        ctx.dxb_slab = slabs and slabs[1]
        _macs(7 * x.numel())
        ctx.save_for_backward(out, gamma, mean, rstd, mask)
        ctx.p = p
        ctx.has_beta = beta is not None
        ctx.ln_params = (gamma, beta)
        ctx.bias = bias
        return y, out

    @staticmethod
    def backward(ctx, dy, dout):
        out, gamma, mean, rstd, mask = ctx.saved_tensors
        if dy is None:  # the LayerNorm output went unused: plain dropout backward of dout
            dx, db = hip_ops().dropout_bwd_db(dout.contiguous(), mask, ctx.p)
            return dx, db, dout, None, None, None, None, None, None, None
        from .linear import FUSE_WGRAD, _bound_grad
        g, b = ctx.ln_params
        acc = None
        if FUSE_WGRAD and ctx.needs_input_grad[3] and (b is None or ctx.needs_input_grad[4]):
            gg, gb = _bound_grad(g), (_bound_grad(b) if b is not None else None)
            if gg is not None and gg.is_contiguous() and (b is None or (gb is not None and gb.is_contiguous())):
                acc = (gg, gb)
        bacc = _bound_grad(ctx.bias) if (FUSE_WGRAD and ctx.needs_input_grad[1]) else None
        if bacc is not None and not bacc.is_contiguous():
            bacc = None
        dtot, dxb, dg, dbt, dbias = hip_ops().bdr_ln_bwd(
            dy.contiguous(), out, gamma, mean, rstd, ctx.has_beta, None if dout is None else dout.contiguous(), mask,
            ctx.p, None if acc is None else acc[0], None if acc is None else acc[1], bacc,
            _slab(ctx.dxb_slab, out, backward=True))
        return (dxb, None if bacc is not None else dbias, dtot, None if acc is not None else dg,
                None if (acc is not None or not ctx.has_beta) else dbt, None, None, None, None, None)


# bias + dropout + residual and the next LayerNorm in one kernel (False: two kernels, tests' A/B)
BDR_LN = True


def bdr_ln_supported(x: torch.Tensor, res: torch.Tensor, bias, gamma, beta) -> bool:
    if not BDR_LN:
        return False
    H = x.shape[-1]
    ts = [x, res, bias, gamma] + ([beta] if beta is not None else [])
    return (x.is_cuda and x.dtype in (torch.bfloat16, torch.float16) and H % 8 == 0 and H <= 1024
            and res.shape == x.shape and all(t.dtype == x.dtype and t.is_contiguous() and t.data_ptr() % 16 == 0
                                             for t in ts))


def bias_dropout_residual_ln(x, bias, residual, gamma, beta, eps, p, training=True, generator=None, rng=None,
                             site=0, slabs=None):
    """(LayerNorm(out), out) for out = residual + dropout(x + bias) -- the attention / MLP output
    of a pre-LN block feeding the next sub-layer's LayerNorm.  One fused HIP pass when supported
    (training with dropout, 16-bit rows of <= 1024), else bias_dropout_residual followed by
    layer_norm_residual (identical values and masks).  slabs: (LayerNorm output spec, x-gradient
    spec) layer slots of ops/wgrad_batch."""
    if training and p > 0 and bdr_ln_supported(x, residual, bias, gamma, beta):
        if rng is not None:
            return _BiasDropoutResidualLNFn.apply(x, bias, residual, gamma, beta, float(p), float(eps),
                                                  int(site) << 20, rng, slabs)
        return _BiasDropoutResidualLNFn.apply(x, bias, residual, gamma, beta, float(p), float(eps),
                                              _draw_seed(generator), None, slabs)
    out = bias_dropout_residual(x, bias, residual, p, training, generator, rng=rng, site=site)
    return layer_norm_residual(out, gamma, beta, eps, y_slab=slabs and slabs[0])


# --------------------------------------------------------------------------- embedding
class _EmbeddingFn(torch.autograd.Function):
    """Embedding lookup whose backward never reads anything back to the host: ids are sorted on
    the device and ops/csrc/kernels/embedding.hip sums the rows of equal ids in fp32 (fixed
    order: deterministic), launches sized by the token count.  PyTorch's dense embedding backward
    reads the number of distinct ids back to the host, which drains the GPU queue at the end of
    every backward.  With a bound weight gradient (the engine's p.grad view) the rows are added
    into it in place, like the fused weight gradients of ops/linear.py."""

    @staticmethod
    def forward(ctx, ids, weight, padding_idx):
        ctx.save_for_backward(ids)
        ctx.weight = weight
        ctx.wshape = tuple(weight.shape)  # a ZeRO-3 parameter may be released (empty) until re-gathered
        ctx.padding_idx = padding_idx
        return torch.nn.functional.embedding(ids, weight, padding_idx if padding_idx >= 0 else None)

    @staticmethod
    def backward(ctx, g):
        (ids,) = ctx.saved_tensors
        w = ctx.weight
        H = ctx.wshape[1]
        # the kernel takes int64 ids (nn.Embedding also accepts int32: widen before the sort)
        sorted_ids, perm = torch.sort(ids.reshape(-1).long(), stable=True)
        g2 = g.reshape(-1, H).contiguous()
        from .linear import FUSE_WGRAD, _bound_grad
        bound = _bound_grad(w) if FUSE_WGRAD else None
        if bound is not None and bound.is_contiguous():
            hip_ops().embedding_bwd(sorted_ids, perm, g2, bound, ctx.padding_idx, True)
            return None, None, None
        dw = torch.zeros(ctx.wshape, dtype=g2.dtype, device=g2.device)
        hip_ops().embedding_bwd(sorted_ids, perm, g2, dw, ctx.padding_idx, False)
        return None, dw, None


def embedding_supported(weight: torch.Tensor) -> bool:
    return (weight.is_cuda and weight.dtype in (torch.bfloat16, torch.float16) and weight.dim() == 2
            and weight.shape[1] % 8 == 0 and weight.is_contiguous())


class Embedding(torch.nn.Embedding):
    """nn.Embedding (same parameters / state dict) with the sync-free HIP backward on the GPU
    (16-bit weights, width % 8 == 0, dense gradients); otherwise torch's embedding."""

    def forward(self, ids):
        if (embedding_supported(self.weight) and self.max_norm is None and not self.sparse
                and not self.scale_grad_by_freq and torch.is_grad_enabled() and self.weight.requires_grad):
            pad = -1 if self.padding_idx is None else int(self.padding_idx)
            return _EmbeddingFn.apply(ids, self.weight, pad)
        return super().forward(ids)
