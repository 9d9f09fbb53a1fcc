"""Attention building blocks on the HIP kernels.

* `rotary_split(qkv, ...)`: GPT-NeoX fused QKV -> (q, k, v) head-major with partial rotary
  embedding and query pre-scaling in one memory pass (HIP), exact inverse in backward.
* `masked_softmax(scores, mask, scale, causal)`: scaled (+additive mask, +causal) row softmax
  (HIP), the analogue of the reference's attn_softmax kernels.
* `attention(q, k, v, ...)`: softmax(q k^T) v with hipBLASLt GEMMs around the fused softmax,
  or the fused flash-attention HIP kernel when built (no S x S materialisation).

CPU tensors use PyTorch reference math (unit tests on CPU CI).
"""

from __future__ import annotations

import math
from typing import Optional

import torch

from . import native

_CS_CACHE = {}


def rotary_table(seq_len: int, rot_dim: int, base: float, device, offset: int = 0) -> torch.Tensor:
    """[seq_len, rot_dim/2, 2] fp32 (cos, sin) table, cached per (len, dim, base, device)."""
    key = (seq_len + offset, rot_dim, base, str(device))
    t = _CS_CACHE.get(key)
    if t is None:
        inv_freq = 1.0 / (base ** (torch.arange(0, rot_dim, 2, dtype=torch.float64) / rot_dim))
        pos = torch.arange(seq_len + offset, dtype=torch.float64)
        ang = torch.outer(pos, inv_freq)
        t = torch.stack([ang.cos(), ang.sin()], dim=-1).float().to(device).contiguous()
        _CS_CACHE[key] = t
    return t[offset:offset + seq_len] if offset else t[:seq_len]


def _rotary_ref(x, cs, rot):
    """x [B,NH,S,HD]; rotate-half on the first `rot` dims."""
    half = rot // 2
    c = cs[..., 0][None, None]  # [1,1,S,half]
    s = cs[..., 1][None, None]
    x1, x2, rest = x[..., :half], x[..., half:rot], x[..., rot:]
    y1 = x1 * c - x2 * s
    y2 = x2 * c + x1 * s
    return torch.cat([y1, y2, rest], dim=-1)


class _RotarySplitFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cs, nh, hd, rot, qscale):
        ctx.meta = (nh, hd, rot, qscale)
        ctx.save_for_backward(cs)
        if qkv.is_cuda:
            q, k, v = native.hip_ops().rotary_split_fwd(qkv.contiguous(), cs, nh, hd, rot, qscale)
            return q, k, v
        B, S, _ = qkv.shape
        x = qkv.float().view(B, S, nh, 3, hd).permute(3, 0, 2, 1, 4)  # [3,B,NH,S,HD]
        q, k, v = x[0], x[1], x[2]
        if rot > 0:
            q = _rotary_ref(q, cs, rot)
            k = _rotary_ref(k, cs, rot)
        q = q * qscale
        dt = qkv.dtype
        return q.to(dt).contiguous(), k.to(dt).contiguous(), v.to(dt).contiguous()

    @staticmethod
    def backward(ctx, dq, dk, dv):
        (cs,) = ctx.saved_tensors
        nh, hd, rot, qscale = ctx.meta
        if dq.is_cuda:
            dqkv = native.hip_ops().rotary_split_bwd(dq.contiguous(), dk.contiguous(), dv.contiguous(), cs, rot,
                                                     qscale)
            return dqkv, None, None, None, None, None

        def inv(g):
            half = rot // 2
            c = cs[..., 0][None, None]
            s = cs[..., 1][None, None]
            g1, g2, rest = g[..., :half], g[..., half:rot], g[..., rot:]
            return torch.cat([g1 * c + g2 * s, g2 * c - g1 * s, rest], dim=-1)

        gq = dq.float() * qscale
        gk = dk.float()
        if rot > 0:
            gq, gk = inv(gq), inv(gk)
        B, NH, S, HD = dq.shape
        x = torch.stack([gq, gk, dv.float()], dim=0).permute(1, 3, 2, 0, 4).reshape(B, S, NH * 3 * HD)
        return x.to(dq.dtype), None, None, None, None, None


class _StashedRotarySplitFn(_RotarySplitFn):
    """Recompute-time stand-in: returns the (q, k, v) the first forward kept (selective
    recompute) instead of re-running the QKV GEMM's consumer; backward is the rotary split's."""

    @staticmethod
    def forward(ctx, qkv, cs, nh, hd, rot, qscale, stash):
        ctx.meta = (nh, hd, rot, qscale)
        ctx.save_for_backward(cs)
        return stash

    @staticmethod
    def backward(ctx, dq, dk, dv):
        return _RotarySplitFn.backward(ctx, dq, dk, dv) + (None,)


def rotary_split(qkv, num_heads: int, head_dim: int, rot_dim: int, base: float = 10000.0, qscale: float = 1.0,
                 stash=None):
    """stash: (q, k, v) kept from the first forward of a checkpointed block; the returned tensors
    are those, with the rotary split's backward attached (qkv is then only a gradient handle)."""
    cs = rotary_table(qkv.shape[1], max(rot_dim, 2), base, qkv.device)
    if stash is not None:
        return _StashedRotarySplitFn.apply(qkv, cs, num_heads, head_dim, rot_dim, qscale, tuple(stash))
    return _RotarySplitFn.apply(qkv, cs, num_heads, head_dim, rot_dim, qscale)


class _MaskedSoftmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mask, scale, causal, heads):
        if x.is_cuda and x.dtype != torch.float32:
            y = native.hip_ops().softmax_fwd(x.contiguous(), mask, scale, causal, heads)
        else:
            s = x.float() * scale
            if mask is not None:
                B = mask.shape[0]
                s = (s.view(B, -1, *s.shape[-2:]) + mask.float().view(B, 1, *mask.shape[-2:])).view_as(s)
            if causal:
                Sq, C = s.shape[-2], s.shape[-1]
                m = torch.ones(Sq, C, dtype=torch.bool, device=s.device).triu(C - Sq + 1)
                s = s.masked_fill(m, float("-inf"))
            y = torch.softmax(s, dim=-1).to(x.dtype)
        ctx.save_for_backward(y)
        ctx.scale = scale
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        if y.is_cuda and y.dtype != torch.float32:
            dx = native.hip_ops().softmax_bwd(dy.contiguous(), y, ctx.scale)
        else:
            yf, g = y.float(), dy.float()
            dx = (ctx.scale * yf * (g - (g * yf).sum(-1, keepdim=True))).to(y.dtype)
        return dx, None, None, None, None


def masked_softmax(scores, mask=None, scale: float = 1.0, causal: bool = False, heads: int = 1):
    """softmax(scale*scores + mask) with optional causal masking; scores [B*H.., Sq, C]."""
    return _MaskedSoftmaxFn.apply(scores, mask, scale, causal, heads)


def attention(q, k, v, causal: bool = True, mask=None, softmax_scale: float = 1.0, dropout_p: float = 0.0,
              training: bool = False, use_flash=None, out_layout: str = "bhsd"):
    """q,k,v [B,NH,S,HD] -> [B,NH,S,HD] (out_layout "bhsd") or [B,S,NH,HD] ("bshd", which the
    flash kernel writes directly so `.reshape(B, S, NH*HD)` is free).  q is expected
    pre-scaled when softmax_scale == 1.  The fused kernel is used for self-attention without
    mask/dropout unless `use_flash` is False."""
    if use_flash is None:
        use_flash = True
    if (use_flash and q.is_cuda and dropout_p == 0.0 and mask is None and q.shape == k.shape == v.shape
            and native.has_flash_attention(q)):
        return native.flash_attention(q, k, v, causal, softmax_scale, out_layout=out_layout)
    B, NH, S, HD = q.shape
    scores = torch.matmul(q, k.transpose(-1, -2))
    probs = masked_softmax(scores, mask, softmax_scale, causal, NH)
    if dropout_p > 0 and training:
        probs = torch.nn.functional.dropout(probs, p=dropout_p)
    out = torch.matmul(probs, v)
    return out.transpose(1, 2) if out_layout == "bshd" else out
