"""Block-sparse matrix products (reference parity: deepspeed/ops/sparse_attention/matmul.py:
`MatMul(layout, block, mode in {sdd, dsd, dds}, trans_a, trans_b)`).

Sparse operands/results use the reference storage: [Z, nnz, block, block], blocks in
torch.nonzero(layout) order.  Everything reduces to two HIP kernels
(ops/csrc/kernels/sparse_attn.hip): a "dense x dense^T -> sampled sparse" product and a
CSR-driven "sparse x dense -> dense" product.  Both take their dense operands as strided
views of either orientation (unit stride along the last or the second-last dim) and stage
tiles into LDS as they lie in memory, so trans_a/trans_b, dds and every backward product run
without transpose or gather copies; a transposed sparse operand is a walk of layout^T whose
blocks the kernel reads transposed, and dds writes its output through a transposed view.
CPU tensors run an equivalent PyTorch gather/scatter implementation (the numerics reference
of the GPU tests).
"""

import torch
import torch.nn.functional as F

from .. import native


class SparseLayout:
    """Host-computed LUTs for one (layout, block): CSR by block-row, its transpose, caches
    of the device copies."""

    def __init__(self, layout: torch.Tensor, block: int):
        layout = layout.detach().to(torch.int64).cpu()
        if layout.dim() == 2:
            layout = layout.unsqueeze(0)
        self.layout, self.block = layout, int(block)
        self.H, self.nbr, self.nbc = layout.shape
        nz = layout.nonzero().contiguous()
        self.nnz = nz.shape[0]
        self.nz = nz.to(torch.int32)
        self.rowptr = torch.cat([torch.zeros(1, dtype=torch.int64), layout.sum(-1).reshape(-1).cumsum(0)]).to(torch.int32)
        self.cols = nz[:, 2].to(torch.int32)
        idx = torch.full(layout.shape, -1, dtype=torch.int64)
        idx[nz[:, 0], nz[:, 1], nz[:, 2]] = torch.arange(self.nnz)
        lt = layout.transpose(1, 2)
        nzt = lt.nonzero().contiguous()
        self.perm_t = idx[nzt[:, 0], nzt[:, 2], nzt[:, 1]]  # transposed order -> original index
        self.rowptr_t = torch.cat([torch.zeros(1, dtype=torch.int64), lt.sum(-1).reshape(-1).cumsum(0)]).to(torch.int32)
        self.cols_t = nzt[:, 2].to(torch.int32)
        self.nz_t = nzt.to(torch.int32)
        self.max_row = int(layout.sum(-1).max().item()) * self.block if self.nnz else 0
        self._dev = {}

    def segments(self, trans: bool):
        """Row-segment LUT of the dsd kernel for one orientation: every (head, block-row) row as
        (row, first, end, slot) with slot -1, except rows much longer than the mean (e.g. BigBird's
        global columns walked transposed), which are cut into segments with their own fp32
        partial slots plus a finish entry (row, slot0, nslots, 0).  Longest segments first."""
        rowptr = (self.rowptr_t if trans else self.rowptr).long()
        lens = rowptr[1:] - rowptr[:-1]
        cap = max(2 * int(torch.ceil(lens.float().mean()).item()) if lens.numel() else 1, max(1, 512 // self.block))
        seg, fin, slot = [], [], 0
        long_rows = set((lens > cap).nonzero().flatten().tolist())
        for row in range(lens.numel()):
            a, b = int(rowptr[row]), int(rowptr[row + 1])
            if row not in long_rows:
                seg.append((row, a, b, -1))
                continue
            k = -(-(b - a) // cap)
            step = -(-(b - a) // k)
            fin.append((row, slot, k, 0))
            for j in range(k):
                seg.append((row, a + j * step, min(b, a + (j + 1) * step), slot))
                slot += 1
        seg.sort(key=lambda t: t[1] - t[2])  # longest first
        as_t = lambda x: torch.tensor(x, dtype=torch.int32).reshape(-1, 4)  # noqa: E731
        return as_t(seg), as_t(fin), slot

    def dev(self, device):
        key = str(device)
        if key not in self._dev:
            t = lambda x: x.contiguous().to(device)  # noqa: E731 (nonzero() results are column-major)
            self._dev[key] = dict(nz=t(self.nz), rowptr=t(self.rowptr), cols=t(self.cols), perm_t=t(self.perm_t),
                                  rowptr_t=t(self.rowptr_t), cols_t=t(self.cols_t), nz_t=t(self.nz_t),
                                  perm_t32=t(self.perm_t.to(torch.int32)))
            for name, tr in (("seg", False), ("seg_t", True)):
                sg, fn, ns = self.segments(tr)
                self._dev[key][name] = (t(sg), t(fn), ns)
        return self._dev[key]


def _pad_last(x, mult):
    pad = (-x.shape[-1]) % mult
    return F.pad(x, (0, pad)) if pad else x


def _use_hip(*ts):
    return all(t.is_cuda for t in ts) and ts[0].dtype in (torch.bfloat16, torch.float16)


def _stageable(x):
    """Can the HIP products read this [Z,H,R,K] view in place?  (unit stride along the last or
    second-last dim; that extent, the other strides and the base 16-byte aligned)."""
    if x.stride(-1) == 1 and x.shape[-1] > 1:
        u = 3
    elif x.stride(-2) == 1:
        u = 2
    else:
        return False
    if x.shape[u] % 8 or x.data_ptr() % 16:
        return False
    return all(x.shape[d] == 1 or x.stride(d) % 8 == 0 for d in range(4) if d != u)


def _hip_operand(x):
    return x if _stageable(x) else x.contiguous()


def sdd(a: torch.Tensor, bn: torch.Tensor, L: SparseLayout, alpha: float = 1.0) -> torch.Tensor:
    """Sampled (a @ bn^T) on L: a [Z,H,nbr*blk,K], bn [Z,H,nbc*blk,K] -> [Z,nnz,blk,blk].
    a / bn may be transposed views (e.g. trans_a, or the backward's dc^T)."""
    blk = L.block
    if _use_hip(a, bn):
        d = L.dev(a.device)
        if a.shape[-1] % 8:
            a, bn = _pad_last(a, 8), _pad_last(bn, 8)
        return native.hip_ops().sparse_sdd(_hip_operand(a), _hip_operand(bn), d["nz"], blk, alpha)
    Z, K = a.shape[0], a.shape[-1]
    nz = L.nz.long().to(a.device)
    av = a.reshape(Z, L.H, L.nbr, blk, K)[:, nz[:, 0], nz[:, 1]]
    bv = bn.reshape(Z, L.H, L.nbc, blk, K)[:, nz[:, 0], nz[:, 2]]
    return (torch.matmul(av.float(), bv.float().transpose(-1, -2)) * alpha).to(a.dtype)


def dsd(s: torch.Tensor, L: SparseLayout, trans: bool, d: torch.Tensor, out_t: bool = False) -> torch.Tensor:
    """(S or S^T as dense) @ d; s [Z,nnz,blk,blk] on L, d [Z,H,K,N] (any orientation) ->
    [Z,H,M,N].  out_t: the result is a transposed view of a contiguous [Z,H,N,M] tensor."""
    blk = L.block
    Z, N = d.shape[0], d.shape[-1]
    nbr, nbc = (L.nbc, L.nbr) if trans else (L.nbr, L.nbc)
    if _use_hip(s, d):
        dv = L.dev(s.device)
        seg, fin, nslots = dv["seg_t"] if trans else dv["seg"]
        cols = dv["cols_t"] if trans else dv["cols"]
        npad = (-N) % 8
        if npad:
            d = F.pad(d, (0, npad))
        d = _hip_operand(d)
        Np, M = N + npad, nbr * blk
        if out_t:
            out = torch.empty(Z, L.H, Np, M, dtype=d.dtype, device=d.device).transpose(-1, -2)
        else:
            out = torch.empty(Z, L.H, M, Np, dtype=d.dtype, device=d.device)
        native.hip_ops().sparse_dsd(s.contiguous(), seg, fin, nslots, cols, dv["perm_t32"] if trans else None, d,
                                    out, L.H, nbr, blk)
        return out[..., :N] if npad else out
    if trans:
        s = s[:, L.perm_t.to(s.device)].transpose(-1, -2)
    nzt = (L.nz_t if trans else L.nz).long().to(s.device)
    dv = d.reshape(Z, L.H, nbc, blk, N)[:, nzt[:, 0], nzt[:, 2]]  # [Z,nnz,blk,N]
    contrib = torch.matmul(s.float(), dv.float())
    out = torch.zeros(Z, L.H * nbr, blk, N, dtype=torch.float32, device=s.device)
    out.index_add_(1, nzt[:, 0] * nbr + nzt[:, 1], contrib)
    return out.view(Z, L.H, nbr * blk, N).to(d.dtype)


def dds(d: torch.Tensor, s: torch.Tensor, L: SparseLayout, trans: bool) -> torch.Tensor:
    """d @ (S or S^T as dense); d [Z,H,M,K] -> [Z,H,M,N] (= (S_eff^T @ d^T)^T, written in place
    through a transposed output view on the GPU)."""
    return dsd(s, L, not trans, d.transpose(-1, -2), out_t=True).transpose(-1, -2)


def _t(x):
    return x.transpose(-1, -2)


class _SparseMatMul(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, L, mode, trans_a, trans_b):
        ctx.save_for_backward(a, b)
        ctx.L, ctx.mode, ctx.ta, ctx.tb = L, mode, trans_a, trans_b
        if mode == "sdd":
            ae = _t(a) if trans_a else a
            bn = b if trans_b else _t(b)
            return sdd(ae, bn, L)
        if mode == "dsd":
            be = _t(b) if trans_b else b
            return dsd(a, L, trans_a, be)
        ae = _t(a) if trans_a else a
        return dds(ae, b, L, trans_b)

    @staticmethod
    def backward(ctx, dc):
        a, b = ctx.saved_tensors
        L, mode, ta, tb = ctx.L, ctx.mode, ctx.ta, ctx.tb
        da = db = None
        if mode == "sdd":
            ae = _t(a) if ta else a  # [M,K]
            bn = b if tb else _t(b)  # [N,K] == B_eff^T
            if ctx.needs_input_grad[0]:
                dae = dsd(dc, L, False, bn)
                da = _t(dae) if ta else dae
            if ctx.needs_input_grad[1]:
                dbe = dds(_t(ae), dc, L, False)  # [K,N]
                db = _t(dbe) if tb else dbe
        elif mode == "dsd":
            be = _t(b) if tb else b  # [K,N]
            if ctx.needs_input_grad[0]:
                da = sdd(be, dc, L) if ta else sdd(dc, be, L)
            if ctx.needs_input_grad[1]:
                dbe = dsd(a, L, not ta, dc)
                db = _t(dbe) if tb else dbe
        else:  # dds
            ae = _t(a) if ta else a  # [M,K]
            if ctx.needs_input_grad[0]:
                dae = dds(dc, b, L, not tb)
                da = _t(dae) if ta else dae
            if ctx.needs_input_grad[1]:
                db = sdd(_t(dc), _t(ae), L) if tb else sdd(_t(ae), _t(dc), L)
        return da, db, None, None, None, None


class MatMul:
    """Block-sparse matmul.  mode: 'sdd' (dense x dense -> sparse), 'dsd' (sparse x dense ->
    dense), 'dds' (dense x sparse -> dense); trans_a / trans_b transpose the operands."""

    def __init__(self, layout, block, mode, trans_a=False, trans_b=False, bench=False):
        if mode not in ("sdd", "dsd", "dds"):
            raise NotImplementedError("Supported modes are: sdd, dsd, dds")
        self.layout, self.block, self.mode = layout, block, mode
        self.trans_a, self.trans_b = trans_a, trans_b
        self.spdims = tuple(layout.shape)
        self.L = SparseLayout(layout, block)
        self.bench = bench

    def __call__(self, a, b):
        return _SparseMatMul.apply(a, b, self.L, self.mode, self.trans_a, self.trans_b)
