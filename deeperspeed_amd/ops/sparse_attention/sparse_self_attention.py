"""Block-sparse self-attention module (reference parity:
deepspeed/ops/sparse_attention/sparse_self_attention.py:14-174).

softmax(scale * Q K^T (+rpe, masks)) V.  On the GPU one fused kernel per direction walks the
layout's active tiles with the masks / RPE as score biases (ops/sparse_attention/flash.py);
elsewhere Q K^T is sampled on the layout (SDD), then the sparse softmax and a sparse x dense
product (DSD).  The layout is built once for
`max_seq_length` and broadcast from rank 0 on first use (random patterns stay identical on
every rank); shorter sequences use its top-left sub-layout."""

import torch
import torch.distributed as dist
import torch.nn as nn

from . import flash
from .matmul import MatMul
from .softmax import Softmax
from .sparsity_config import SparsityConfig


class SparseSelfAttention(nn.Module):
    def __init__(self, sparsity_config=SparsityConfig(num_heads=4), key_padding_mask_mode="add",
                 attn_mask_mode="mul", max_seq_length=2048):
        super().__init__()
        self.sparsity_config = sparsity_config
        self.master_layout = sparsity_config.make_layout(max_seq_length)
        self._need_layout_synchronization = True
        self.key_padding_mask_mode = key_padding_mask_mode
        self.attn_mask_mode = attn_mask_mode
        self.ops = {}
        # False: masked / RPE calls take the SDD / softmax / DSD kernels (A/B and parity tests)
        self.fused_masks = True

    def get_layout(self, L):
        if self._need_layout_synchronization and dist.is_available() and dist.is_initialized():
            t = self.master_layout
            if dist.get_backend() == "nccl":
                t = t.cuda()
            dist.broadcast(t, src=0)
            self.master_layout = t.cpu()
            self._need_layout_synchronization = False
        block = self.sparsity_config.block
        if L % block != 0:
            raise ValueError(f"Sequence Length, {L}, needs to be dividable by Block size {block}!")
        nb = L // block
        if nb > self.master_layout.shape[-1]:
            raise RuntimeError(f"sequence length {L} exceeds this SparseSelfAttention's max_seq_length "
                               f"({self.master_layout.shape[-1] * block}); build it with a larger max_seq_length")
        return self.master_layout[..., :nb, :nb].cpu()

    def get_ops(self, H, L):
        if L not in self.ops:
            layout = self.get_layout(L)
            block = self.sparsity_config.block
            self.ops[L] = (MatMul(layout, block, "sdd", trans_a=False, trans_b=True),
                           MatMul(layout, block, "dsd", trans_a=False, trans_b=False), Softmax(layout, block))
        return self.ops[L]

    def get_lut(self, L):
        """LUT of the fused kernel for sequence length L (None when the layout is outside its
        domain: block not in 16/32/64/128 or L not a multiple of 64)."""
        luts = self.__dict__.setdefault("_luts", {})
        if L not in luts:
            try:
                luts[L] = flash.SparseFlashLUT(self.get_layout(L), self.sparsity_config.block)
            except ValueError:
                luts[L] = None
        return luts[L]

    def transpose_key_for_scores(self, x, L):
        bsz, num_heads, seq_len, head_dim = x.size()
        if seq_len != L:
            return x.permute(0, 1, 3, 2)
        return x

    def transpose_mask_for_sparse(self, qtype, x, is_key_padding_mask=False):
        x = x.type(qtype)
        if is_key_padding_mask:
            xdim = x.dim()
            for d in range(xdim - 1, 0, -1):
                x = x.squeeze(dim=d)
            return x
        return x.squeeze()

    def forward(self, query, key, value, rpe=None, key_padding_mask=None, attn_mask=None):
        bsz, num_heads, tgt_len, head_dim = query.size()
        key = self.transpose_key_for_scores(key, tgt_len)
        if query.shape != key.shape or key.shape != value.shape:
            raise NotImplementedError("only self-attention is supported for now")
        if key_padding_mask is not None:
            key_padding_mask = self.transpose_mask_for_sparse(query.dtype, key_padding_mask, is_key_padding_mask=True)
            if key_padding_mask.dim() == 1:
                key_padding_mask = key_padding_mask.unsqueeze(0)
        if attn_mask is not None:
            attn_mask = self.transpose_mask_for_sparse(query.dtype, attn_mask)
        scaling = float(head_dim) ** -0.5
        plain = rpe is None and key_padding_mask is None and attn_mask is None
        if plain or self.fused_masks:
            lut = self.get_lut(tgt_len)
            if flash.supported(query, lut):  # one fused kernel per query tile (ops/sparse_attention/flash.py)
                kbias, ebias = flash.score_biases(query, rpe, key_padding_mask, attn_mask,
                                                  self.key_padding_mask_mode, self.attn_mask_mode)
                return flash.sparse_flash_attention(query, key, value, lut, scaling, kbias=kbias, ebias=ebias)
        sdd_nt, dsd_nn, softmax = self.get_ops(num_heads, tgt_len)
        w = sdd_nt(query, key)
        w = softmax(w, scale=scaling, rpe=rpe, key_padding_mask=key_padding_mask, attn_mask=attn_mask,
                    key_padding_mask_mode=self.key_padding_mask_mode, attn_mask_mode=self.attn_mask_mode)
        return dsd_nn(w, value)
