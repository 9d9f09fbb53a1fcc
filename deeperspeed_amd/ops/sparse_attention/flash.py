"""Fused block-sparse (flash-style) attention on the CDNA4 kernels of ops/csrc/kernels/flash_attn.hip.

The reference computes block-sparse attention as three Triton launches -- SDD (Q K^T sampled on
the layout), a sparse row softmax and DSD (P V) -- with the sparse score matrix written to and
read back from HBM between them (deepspeed/ops/sparse_attention/matmul.py:117-238,
softmax.py:44-120, trsrc/softmax_fwd.tr:46-129).  Here one kernel walks, per 64-query tile, the
key tiles the layout activates and keeps scores / probabilities in registers (online softmax);
the backward is the same walk for dQ and the transposed walk for dK / dV.

Gathered tiles.  The kernels' unit of work is a 64 x 64 MFMA tile, but a tile's 64 keys (or, in
the dK / dV walk, its 64 queries) need not be contiguous: every LUT entry names FOUR 16-row
blocks that are gathered into the tile, and a 16-bit mask says which (query 16-block, key
16-block) pairs of the 4 x 4 grid are active.  `SparseFlashLUT` builds the walks at that 16-row
granularity whatever the layout block (16 / 32 / 64 / 128):
  * forward / dQ: per contiguous 64-query tile, the union of the key 16-blocks its four query
    blocks activate, packed four at a time -- work scales with the active 16-blocks, not with the
    64-tiles they touch (the reference's default block 16 "fixed" layout puts one global key
    block in every 64-key window: 2,080 dense tiles at S = 4096 become 592 gathered ones);
  * dK / dV: the key 16-blocks are first grouped four at a time into output groups (contiguous,
    or sorted by how many query blocks attend them when that packs tighter -- the global columns
    of fixed / Longformer layouts land together), then per group the union of the query 16-blocks
    that attend it, packed four at a time.
Blocks above the diagonal are dropped for causal attention (the element-level diagonal is masked
in the kernels).  Layout blocks of 64 / 128 reproduce the contiguous tiles with full masks.

The reference softmax's score terms run inside the same kernels (`score_biases`): the key-padding
mask as a per-key fp32 bias, the relative position embedding and the attention mask pre-summed
into one [B|1, H|1, S, S] element bias read only on active tiles ('mul' masks become 0 / -inf).
Shapes outside the kernel's domain (S % 64, head dim) fall back to the SDD / softmax / DSD path.
"""

from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch

TILE = 64
SUB = 16  # rows per gathered block
NSUB = TILE // SUB


class SparseFlashLUT:
    """Gathered-tile walks of a block-sparse layout (see the module docstring).

    Host arrays (`_host`, in `device_tensors` order):
      rowptr  int32 [Hl * nqt + 1]   forward / dQ entries of each query tile
      cols    int32 [E, 4]           the four key 16-blocks of each entry (ascending; padding repeats
                                     the last one, its mask bits are 0)
      masks   int32 [E]              bit (qsub * 4 + kslot): query 16-block qsub of the tile x key slot
      colptr  int32 [Hl * nkg + 1]   dK / dV entries of each key group
      rows    int32 [E_t, 4]         the four query 16-blocks of each dK / dV entry
      masks_t int32 [E_t]            bit (qslot * 4 + kslot)
      tasks   int32 [Hl, ntask, 4]   (key group or -1, entry begin, entry end, partial slot or -1)
      fin     int32 [Hl, nfin, 4]    (key group or -1, first slot, chunks, 0) of split groups
      kgroups int32 [Hl, nkg, 4]     the four key 16-blocks of each group (ascending)
    """

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
        self.shift = 4  # kept for the kernels' signature: masks are always on the 16-row grid
        r = block // SUB
        L = np.repeat(np.repeat(lay.numpy(), r, axis=1), r, axis=2)  # [Hl, n16, n16]
        n16 = L.shape[-1]
        if self.causal:
            L = L & np.tril(np.ones((n16, n16), dtype=bool))[None]
        nqt = n16 // NSUB
        fwd = [self._fwd_walk(L[h], nqt) for h in range(self.heads)]
        bwd = [self._bwd_walk(L[h], nqt) for h in range(self.heads)]
        self.tiles = sum(len(f[1]) for f in fwd)
        self.density = float(self.tiles) / (self.heads * nqt * nqt)  # gathered 64x64 tiles processed
        self.block_density = float(L.sum()) / L.size
        rowptr, cols, masks = self._concat(fwd, nqt)
        colptr, rows, masks_t = self._concat([b[:3] for b in bwd], nqt)
        kgroups = np.stack([b[3] for b in bwd]).astype(np.int32)
        self._host = (rowptr, cols, masks, colptr, rows, masks_t)
        self._host += self._split_tasks(colptr, nqt)
        self._host += (kgroups,)
        self.nslot = self._nslot
        self._dev: Dict[torch.device, tuple] = {}

    # ------------------------------------------------------------------ walks
    @staticmethod
    def _pack(blocks, act):
        """Entries of 4 gathered blocks: blocks ascending; act(slot_block) -> [4] bools per
        gathered block (which of the 4 tile sub-rows / slots it pairs with).  Returns
        [(blk4, mask16)] with bit (tile_sub * 4 + slot)."""
        out = []
        for i in range(0, len(blocks), NSUB):
            chunk = list(blocks[i:i + NSUB])
            mask = 0
            for slot, b in enumerate(chunk):
                for sub, on in enumerate(act(b)):
                    if on:
                        mask |= 1 << (sub * NSUB + slot)
            chunk += [chunk[-1]] * (NSUB - len(chunk))
            out.append((chunk, mask))
        return out

    def _fwd_walk(self, L, nqt):
        ptr, ents = [0], []
        for qt in range(nqt):
            rows = L[qt * NSUB:(qt + 1) * NSUB]  # [4, n16]
            union = np.nonzero(rows.any(axis=0))[0]
            ents += self._pack(union, lambda b: rows[:, b])
            ptr.append(len(ents))
        return ptr, ents

    def _bwd_walk(self, L, nqt):
        n16 = L.shape[0]
        att = [np.nonzero(L[:, k])[0] for k in range(n16)]  # query blocks attending key block k
        contiguous = [list(range(g * NSUB, (g + 1) * NSUB)) for g in range(nqt)]
        order = sorted(range(n16), key=lambda k: (-len(att[k]), att[k][0] if len(att[k]) else n16, k))
        by_count = [sorted(order[g * NSUB:(g + 1) * NSUB]) for g in range(nqt)]

        def walk(groups):
            ptr, ents = [0], []
            for grp in groups:
                cols = L[:, grp]  # [n16, 4]
                union = np.nonzero(cols.any(axis=1))[0]
                ents += self._pack(union, lambda q: cols[q])
                ptr.append(len(ents))
            return ptr, ents

        a, b = walk(contiguous), walk(by_count)
        ptr, ents, groups = (a + (contiguous,)) if len(a[1]) <= len(b[1]) else (b + (by_count,))
        # bits of a dK / dV entry: (query slot * 4 + key slot) -- _pack built (key slot * 4 +
        # query slot) from the group's point of view, so transpose the 4 x 4 grid
        fixed = []
        for blk4, m in ents:
            t = 0
            for ks in range(NSUB):
                for qs in range(NSUB):
                    if (m >> (ks * NSUB + qs)) & 1:
                        t |= 1 << (qs * NSUB + ks)
            fixed.append((blk4, t))
        return ptr, fixed, None, np.array(groups, dtype=np.int32)

    @staticmethod
    def _concat(walks, n):
        ptr = [0]
        blocks, masks = [], []
        for w in walks:
            p, ents = w[0], w[1]
            base = ptr[-1]
            ptr += [base + x for x in p[1:]]
            blocks += [e[0] for e in ents]
            masks += [e[1] for e in ents]
        blk = np.array(blocks, dtype=np.int32).reshape(-1, NSUB)
        m = np.array(masks, dtype=np.int64)
        return np.array(ptr, dtype=np.int32), blk, m.astype(np.int32)

    # entries per dK / dV workgroup: longer lists (the global columns of BigBird / Longformer /
    # fixed layouts) are split into chunks whose fp32 partials are summed by a finish kernel
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
            per_head.append(heavy + light)  # split (long) groups launch first
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
        rp, cols, masks, _cp, rows, masks_t, tasks, fin, kgroups = lut.device_tensors(q.device)
        dq, dk, dv = native.hip_ops().sparse_flash_bwd(do.contiguous(), q, k, v, o, lse, rp, cols, masks, rows,
                                                       masks_t, tasks, fin, kgroups, lut.nslot, lut.heads,
                                                       lut.causal, ctx.scale, lut.shift, ctx.out_bshd, ctx.kbias,
                                                       ctx.ebias)
        return dq, dk, dv, None, None, None, None, None


class _StashedSparseFlash(_SparseFlash):
    """Recompute-time stand-in (selective recompute): (o, lse) kept from the checkpointed first
    forward (`sparse_flash_fwd_lse`); the backward is _SparseFlash's."""

    @staticmethod
    def forward(ctx, q, k, v, lut, scale, out_bshd, kbias, ebias, stash):
        o, lse = stash
        ctx.save_for_backward(q.contiguous(), k.contiguous(), v.contiguous(), o, lse)
        ctx.lut, ctx.scale, ctx.out_bshd = lut, float(scale), bool(out_bshd)
        ctx.kbias, ctx.ebias = kbias, ebias
        return o

    @staticmethod
    def backward(ctx, do):
        return _SparseFlash.backward(ctx, do) + (None,)


def sparse_flash_fwd_lse(q, k, v, lut: SparseFlashLUT, scale: float = 1.0, out_bshd: bool = False,
                         kbias: Optional[torch.Tensor] = None, ebias: Optional[torch.Tensor] = None):
    """Forward only (no autograd): (o, lse) for a later stashed backward (selective recompute)."""
    from .. import native
    rp, cols, masks = lut.device_tensors(q.device)[:3]
    return native.hip_ops().sparse_flash_fwd(q.contiguous(), k.contiguous(), v.contiguous(), rp, cols, masks,
                                             lut.heads, lut.causal, float(scale), lut.shift, bool(out_bshd), kbias,
                                             ebias)


def sparse_flash_attention(q, k, v, lut: SparseFlashLUT, scale: float = 1.0, out_bshd: bool = False,
                           kbias: Optional[torch.Tensor] = None, ebias: Optional[torch.Tensor] = None, stash=None):
    """softmax(scale * Q K^T [+ kbias[b, key] + ebias[b, h, q, key]] restricted to the layout
    [+ causal]) V for q, k, v [B, H, S, D]; returns [B, H, S, D], or [B, S, H, D] with out_bshd.
    kbias / ebias: see `score_biases` (rows with no unmasked key give 0).
    stash: (o, lse) from sparse_flash_fwd_lse of the same inputs (selective recompute)."""
    if stash is not None:
        return _StashedSparseFlash.apply(q, k, v, lut, scale, out_bshd, kbias, ebias, tuple(stash))
    return _SparseFlash.apply(q, k, v, lut, scale, out_bshd, kbias, ebias)
