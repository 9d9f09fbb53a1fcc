"""Fused block-sparse (flash-style) attention on the CDNA4 kernels of ops/csrc/kernels/flash_attn.hip.

The reference computes block-sparse attention as three Triton launches -- SDD (Q K^T sampled on
the layout), a sparse row softmax and DSD (P V) -- with the sparse score matrix written to and
read back from HBM between them (deepspeed/ops/sparse_attention/matmul.py:117-238,
softmax.py:44-120, trsrc/softmax_fwd.tr:46-129).  Here one kernel walks, per 64-query tile, the
64-key tiles the layout activates and keeps scores / probabilities in registers (online
softmax); the backward is the same walk for dQ and the transposed walk for dK / dV.

`SparseFlashLUT` turns a layout [H or 1, nb, nb] of `block`-sized blocks into those walks:
per layout head, a CSR list of active key tiles per query tile and the transposed list, each
entry with a bitmask of the active layout sub-blocks when the layout block is smaller than the
64-element tile (block 16 -> 4x4 sub-blocks, 32 -> 2x2).  Tiles above the diagonal are dropped
for causal attention.  The reference softmax's score terms run inside the same kernels
(`score_biases`): the key-padding mask as a per-key fp32 bias, the relative position embedding
and the attention mask pre-summed into one [B|1, H|1, S, S] element bias read only on active
tiles ('mul' masks become 0 / -inf).  Shapes outside the kernel's domain (S % 64, head dim) fall
back to the SDD / softmax / DSD path.
"""

from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch

TILE = 64


class SparseFlashLUT:
    def __init__(self, layout: torch.Tensor, block: int, causal: bool = False):
        lay = layout.detach().cpu().to(torch.bool)
        if lay.dim() == 2:
            lay = lay.unsqueeze(0)
        if all(torch.equal(lay[0], lay[i]) for i in range(1, lay.shape[0])):
            lay = lay[:1]  # every head shares the layout: one LUT
        if block not in (16, 32, 64, 128):
            raise ValueError(f"block-sparse flash attention supports blocks of 16, 32, 64 or 128, not {block}")
        self.block = block
        self.causal = bool(causal)
        self.heads = lay.shape[0]
        nb = lay.shape[-1]
        self.seq = nb * block
        if self.seq % TILE:
            raise ValueError(f"sequence {self.seq} is not a multiple of the {TILE}-element tile")
        self.shift = min(6, int(block).bit_length() - 1)
        nt = self.seq // TILE
        L = lay.numpy()
        if block >= TILE:  # each tile lies inside one layout block
            rep = block // TILE
            act = np.repeat(np.repeat(L, rep, axis=1), rep, axis=2)
            masks = act.astype(np.int64)
        else:
            r = TILE // block
            sub = L.reshape(self.heads, nt, r, nt, r).transpose(0, 1, 3, 2, 4)  # [h, i, j, qsub, ksub]
            weights = (1 << np.arange(r * r, dtype=np.int64)).reshape(r, r)
            masks = (sub.astype(np.int64) * weights).sum(axis=(3, 4))
            act = masks != 0
        if self.causal:
            act = act & np.tril(np.ones((nt, nt), dtype=bool))[None]
        self.density = float(act.sum()) / act.size
        self.tiles = int(act.sum())
        self._host = self._csr(act, masks) + self._csr(act.transpose(0, 2, 1), masks.transpose(0, 2, 1))
        self._host += self._split_tasks(self._host[3], nt)
        self.nslot = self._nslot
        self._dev: Dict[torch.device, tuple] = {}

    # query tiles per dK / dV workgroup: longer key-tile lists (global columns) are split into
    # chunks whose fp32 partials are summed by a finish kernel
    CHUNK = 8

    def _split_tasks(self, colptr, nt):
        per_head, fins, slots = [], [], []
        for h in range(self.heads):
            heavy, light, fin, nslot = [], [], [], 0
            for kt in range(nt):
                e0, e1 = int(colptr[h * nt + kt]), int(colptr[h * nt + kt + 1])
                if e1 - e0 <= self.CHUNK:
                    if e1 > e0:
                        light.append((kt, e0, e1, -1))
                    continue
                n = -(-(e1 - e0) // self.CHUNK)
                fin.append((kt, nslot, n, 0))
                for c in range(n):
                    heavy.append((kt, e0 + c * self.CHUNK, min(e1, e0 + (c + 1) * self.CHUNK), nslot + c))
                nslot += n
            per_head.append(heavy + light)  # split (long) tiles launch first
            fins.append(fin)
            slots.append(nslot)
        ntask = max(1, max(len(t) for t in per_head))
        nfin = max(len(f) for f in fins)
        tasks = np.full((self.heads, ntask, 4), -1, dtype=np.int32)
        fin = np.full((self.heads, max(1, nfin), 4), -1, dtype=np.int32)
        for h in range(self.heads):
            if per_head[h]:
                tasks[h, :len(per_head[h])] = per_head[h]
            if fins[h]:
                fin[h, :len(fins[h])] = fins[h]
        self._nslot = max(slots) if slots else 0
        if nfin == 0:
            fin = fin[:, :0]
        return (tasks, fin)

    @staticmethod
    def _csr(act, masks):
        h, n, _ = act.shape
        counts = act.reshape(h * n, n).sum(axis=1)
        ptr = np.zeros(h * n + 1, dtype=np.int64)
        np.cumsum(counts, out=ptr[1:])
        hi, ri, ci = np.nonzero(act)  # row-major: (head, row) ascending, columns ascending
        bits = masks[hi, ri, ci].astype(np.int64)
        bits = np.where(bits >= 2**31, bits - 2**32, bits)  # uint32 bit patterns stored as int32
        return (ptr.astype(np.int32), ci.astype(np.int32), bits.astype(np.int32))

    def device_tensors(self, device):
        t = self._dev.get(device)
        if t is None:
            t = tuple(torch.from_numpy(np.ascontiguousarray(a)).to(device) for a in self._host)
            self._dev[device] = t
        return t


def supported(q: torch.Tensor, lut: Optional[SparseFlashLUT]) -> bool:
    if lut is None or not q.is_cuda or q.dtype not in (torch.bfloat16, torch.float16):
        return False
    B, H, S, D = q.shape
    if D not in (64, 96, 128) or S != lut.seq or (lut.heads not in (1, H)):
        return False
    from .. import native
    native.hip_ops()  # fails loudly when the extension is missing on a GPU box
    return True


def _as4(t):
    while t.dim() < 4:
        t = t.unsqueeze(0)
    return t


def _additive(mask: torch.Tensor, mode: str) -> torch.Tensor:
    m = mask.float()
    return torch.where(m == 0, float("-inf"), 0.0) if mode == "mul" else m


def score_biases(q, rpe=None, key_padding_mask=None, attn_mask=None, key_padding_mask_mode="add",
                 attn_mask_mode="add"):
    """(kbias, ebias) for the fused kernels from the reference Softmax's optional terms
    (softmax.py:230-315): kbias = key-padding mask [B, S] fp32, ebias = rpe [Z|1, H|1, S, S] +
    attention mask [S, S] in q's dtype (broadcast dims kept as stride-0 views)."""
    B, H, S, _ = q.shape
    kbias = ebias = None
    if key_padding_mask is not None:
        kp = key_padding_mask.reshape(-1, S) if key_padding_mask.dim() != 2 else key_padding_mask
        kbias = _additive(kp, key_padding_mask_mode).expand(B, S).contiguous()
    if rpe is not None or attn_mask is not None:
        e = None
        if rpe is not None:
            e = _as4(rpe).float()
        if attn_mask is not None:
            a = _additive(attn_mask.reshape(S, S), attn_mask_mode)[None, None]
            e = a if e is None else e + a
        if e.shape[0] not in (1, B) or e.shape[1] not in (1, H) or tuple(e.shape[2:]) != (S, S):
            raise ValueError(f"relative position embedding / attention mask of shape {tuple(e.shape)} does not "
                             f"broadcast to [{B}, {H}, {S}, {S}]")
        ebias = e.to(q.dtype).contiguous()
    return kbias, ebias


class _SparseFlash(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, lut, scale, out_bshd, kbias, ebias):
        from .. import native
        ops = native.hip_ops()
        rp, cols, masks = lut.device_tensors(q.device)[:3]
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        o, lse = ops.sparse_flash_fwd(q, k, v, rp, cols, masks, lut.heads, lut.causal, float(scale), lut.shift,
                                      bool(out_bshd), kbias, ebias)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.lut, ctx.scale, ctx.out_bshd = lut, float(scale), bool(out_bshd)
        ctx.kbias, ctx.ebias = kbias, ebias  # constants: no gradient (as in the reference softmax)
        return o

    @staticmethod
    def backward(ctx, do):
        from .. import native
        q, k, v, o, lse = ctx.saved_tensors
        lut = ctx.lut
        rp, cols, masks, _cp, rows, masks_t, tasks, fin = lut.device_tensors(q.device)
        dq, dk, dv = native.hip_ops().sparse_flash_bwd(do.contiguous(), q, k, v, o, lse, rp, cols, masks, rows,
                                                       masks_t, tasks, fin, lut.nslot, lut.heads, lut.causal,
                                                       ctx.scale, lut.shift, ctx.out_bshd, ctx.kbias, ctx.ebias)
        return dq, dk, dv, None, None, None, None, None


def sparse_flash_attention(q, k, v, lut: SparseFlashLUT, scale: float = 1.0, out_bshd: bool = False,
                           kbias: Optional[torch.Tensor] = None, ebias: Optional[torch.Tensor] = None):
    """softmax(scale * Q K^T [+ kbias[b, key] + ebias[b, h, q, key]] restricted to the layout
    [+ causal]) V for q, k, v [B, H, S, D]; returns [B, H, S, D], or [B, S, H, D] with out_bshd.
    kbias / ebias: see `score_biases` (rows with no unmasked key give 0)."""
    return _SparseFlash.apply(q, k, v, lut, scale, out_bshd, kbias, ebias)
