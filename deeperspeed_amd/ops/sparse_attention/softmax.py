"""Block-sparse softmax (reference parity: deepspeed/ops/sparse_attention/softmax.py `Softmax`):
scale, relative position embedding [Z|1, H|1, S, S], key-padding mask [Z, S] and attention
mask [S, S], each mask in 'add' or 'mul' (0 -> -inf) mode, over the non-zero blocks of every
row.  One wave64 per row on the GPU (sparse_attn.hip): the row is held in registers, so x is
read once and every bias evaluated once, written out of place."""

import torch

from .. import native
from .matmul import SparseLayout


def _as4(rpe):
    while rpe.dim() < 4:
        rpe = rpe.unsqueeze(0)
    return rpe


class _SparseSoftmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, L, scale, rpe, kpm, attn, kpm_mode, attn_mode, causal=False):
        if x.is_cuda and x.dtype in (torch.bfloat16, torch.float16):
            d = L.dev(x.device)
            x = x.contiguous()
            y = torch.empty_like(x)
            native.hip_ops().sparse_softmax_fwd(x, y, d["rowptr"], d["cols"], L.H, L.nbr, L.max_row, scale,
                                                None if rpe is None else _as4(rpe).contiguous(),
                                                None if kpm is None else kpm.contiguous(),
                                                None if attn is None else attn.contiguous(),
                                                kpm_mode == "mul", attn_mode == "mul", bool(causal))
        else:
            y = _softmax_ref(x, L, scale, rpe, kpm, attn, kpm_mode, attn_mode, causal)
        ctx.save_for_backward(y)
        ctx.L, ctx.scale = L, scale
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        L = ctx.L
        if y.is_cuda and y.dtype in (torch.bfloat16, torch.float16):
            dy = dy.contiguous()
            dx = torch.empty_like(dy)
            native.hip_ops().sparse_softmax_bwd(y, dy, dx, L.dev(y.device)["rowptr"], L.H, L.nbr, L.max_row,
                                                ctx.scale)
        else:
            dx = _softmax_bwd_ref(y, dy, L, ctx.scale)
        return dx, None, None, None, None, None, None, None, None


def _dense_index(L, device):
    nz = L.nz.long().to(device)
    blk = L.block
    r = torch.arange(blk, device=device)
    rows = (nz[:, 1:2] * blk + r).view(-1, blk, 1)  # [nnz, blk, 1]
    cols = (nz[:, 2:3] * blk + r).view(-1, 1, blk)  # [nnz, 1, blk]
    return nz[:, 0].view(-1, 1, 1), rows, cols


def _softmax_ref(x, L, scale, rpe, kpm, attn, kpm_mode, attn_mode, causal=False):
    Z, S = x.shape[0], L.nbr * L.block
    hh, rows, cols = _dense_index(L, x.device)
    v = x.float() * scale
    if rpe is not None:
        rp = _as4(rpe).float().expand(Z, L.H, S, S)
        v = v + rp[:, hh, rows, cols]
    if kpm is not None:
        m = kpm.float()
        m = torch.where(m == 0, float("-inf"), 0.0) if kpm_mode == "mul" else m
        v = v + m.expand(Z, S)[:, cols.expand(-1, L.block, -1)]
    if attn is not None:
        m = attn.float()
        m = torch.where(m == 0, float("-inf"), 0.0) if attn_mode == "mul" else m
        v = v + m[rows, cols].unsqueeze(0)
    if causal:
        v = v.masked_fill((cols > rows).unsqueeze(0), float("-inf"))
    dense = torch.full((Z, L.H, S, S), float("-inf"), device=x.device)
    dense[:, hh, rows, cols] = v
    p = torch.softmax(dense, -1).nan_to_num(0.0)
    return p[:, hh, rows, cols].to(x.dtype)


def _softmax_bwd_ref(y, dy, L, scale):
    Z, S = y.shape[0], L.nbr * L.block
    hh, rows, cols = _dense_index(L, y.device)
    yd = torch.zeros(Z, L.H, S, S, device=y.device)
    gd = torch.zeros_like(yd)
    yd[:, hh, rows, cols] = y.float()
    gd[:, hh, rows, cols] = dy.float()
    dx = scale * yd * (gd - (gd * yd).sum(-1, keepdim=True))
    return dx[:, hh, rows, cols].to(y.dtype)


class Softmax:
    def __init__(self, layout, block, bench=False):
        self.layout, self.block = layout, block
        self.num_blocks = int(layout.sum().item())
        self.spdims = tuple(layout.shape)
        self.L = SparseLayout(layout, block)
        self.bench = bench

    def __call__(self, x, scale=1.0, rpe=None, key_padding_mask=None, attn_mask=None, key_padding_mask_mode="add",
                 attn_mask_mode="add", causal=False):
        """`causal` (extension): mask col > row inside the non-zero blocks, so unidirectional
        layouts need no dense [S, S] attention mask."""
        for name, t in (("relative position embedding", rpe), ("Attention mask", attn_mask),
                        ("Key padding mask", key_padding_mask)):
            if t is not None and t.dtype != x.dtype:
                raise ValueError(f"{name} must be {x.dtype}")
        return _SparseSoftmaxFn.apply(x, self.L, float(scale), rpe, key_padding_mask, attn_mask,
                                      key_padding_mask_mode, attn_mask_mode, bool(causal))
