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

Set DSA_FUSE_WGRAD=0 to disable (identical math up to one rounding of the accumulate).

Reduction-contiguous wgrad operands (DSA_WGRAD_NT, default on for GPU tensors): hipBLASLt on
gfx950 runs dW = dy^T x at ~1.1 PF/s with the token-major operands autograd holds, and at
~1.45 PF/s when both operands are contiguous along the token (reduction) dimension
(profiles/aux/wgrad_dgrad_variants_neox20b.jsonl).  The HIP transpose kernel
(ops/csrc/kernels/transpose.hip) makes dy^T and x^T first; the transpose of dy also produces
the bias gradient (its column sum) from the same read.
"""

from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import lt_tune
from . import wgrad_batch as _wb

FUSE_WGRAD = os.environ.get("DSA_FUSE_WGRAD", "1") != "0"
WGRAD_NT = os.environ.get("DSA_WGRAD_NT", "1") != "0"
# smallest out*in weight that takes the transposed path (the transposes move ~4*M*(out+in)
# bytes; below this the GEMM saving does not pay for them)
WGRAD_NT_MIN_NUMEL = int(float(os.environ.get("DSA_WGRAD_NT_MIN_NUMEL", "1e7")))
# cap on the transient transposed copies (bytes of dy^T + x^T): the LM head's dlogits at 16k
# tokens (1.65 GB) keeps the token-major formulation instead of adding its copy to the peak
WGRAD_NT_MAX_BYTES = int(float(os.environ.get("DSA_WGRAD_NT_MAX_BYTES", "1.2e9")))
# input gradient dx = dy W from W^T [in, out] (reduction-contiguous, one HIP transpose of the
# weight per use): hipBLASLt ~1.45 vs ~1.28 PF/s at the GPT-NeoX-20B shapes, 1.05-1.2 vs
# 0.98-1.03 PF/s at BERT-Large's (profiles/r2m_gemm_shapes_bert_neox.md)
DGRAD_NT = os.environ.get("DSA_DGRAD_NT", "1") != "0"
DGRAD_NT_MIN_NUMEL = int(float(os.environ.get("DSA_DGRAD_NT_MIN_NUMEL", "1e6")))
# split-K weight gradient for small weights over many tokens: [out, in] gives too few 256x256
# output tiles to fill 256 CUs (BERT-Large: 16-64 tiles at 8k tokens, 300-800 TF/s), so the
# tokens are cut into WGRAD_SPLIT batches of one strided-batched GEMM whose partial products
# are summed in fp32 (1.25-1.6x at the BERT-Large shapes, same profile).  DSA_WGRAD_SPLIT=1 off.
WGRAD_SPLIT = int(os.environ.get("DSA_WGRAD_SPLIT", "4"))
WGRAD_SPLIT_MAX_TILES = 128
WGRAD_SPLIT_MIN_TOKENS = 4096


# DSA_LINEAR_LT=1: forward GEMMs through the autotuned hipBLASLt wrapper (bias in the
# epilogue).  Bias-free microbenchmarks favour it by up to 6 % at the GPT-NeoX-20B shapes, but
# the whole 20B step measured 1.3 % slower with it (same box, profiles/r2n_linear_lt_ab.md), so
# torch's F.linear stays the default.
LINEAR_LT = os.environ.get("DSA_LINEAR_LT", "0") == "1"

_count = [0]  # in-place accumulations performed (tests / diagnostics)
_nt_count = [0]  # wgrads formed from transposed operands
_lt_nt_count = [0]  # wgrads formed by the measured NT solution on token-major operands


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


# DSA_SHARE_GRAD_T=0: every weight gradient transposes its own output gradient
SHARE_GRAD_T = os.environ.get("DSA_SHARE_GRAD_T", "1") != "0"


def nt_wgrad_planned(M: int, out_features: int, in_features: int, elem_size: int = 2, g_ready: bool = False,
                     x_ready: bool = False) -> bool:
    """Whether the weight gradient of a [out, in] linear over M tokens takes the
    reduction-contiguous (transposed-operand) path -- the predicate producers of pre-transposed
    operands check before offering one.  g_ready / x_ready: that operand is already available
    transposed, so it adds no transient copy."""
    if not WGRAD_NT or out_features * in_features < WGRAD_NT_MIN_NUMEL:
        return False
    if lt_tune.wgrad_nt(M, out_features, in_features, elem_size):
        return False  # the measured NT GEMM reads the token-major operands directly
    if (WGRAD_SPLIT > 1 and M >= WGRAD_SPLIT_MIN_TOKENS and M % WGRAD_SPLIT == 0
            and -(-out_features // 256) * -(-in_features // 256) <= WGRAD_SPLIT_MAX_TILES
            and not lt_tune.use_wgrad_t(M, out_features, in_features)):
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
    if tiles <= WGRAD_SPLIT_MAX_TILES and lt_tune.use_wgrad_t(M, out, inp):
        return 1  # a measured TN solution fills the chip without splitting (ops/lt_tune.py)
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


# DSA_WT_PREFETCH=1: the dgrad weight transposes run one linear ahead on a side stream (opt-in: on
# the 20B N = 1 step it measured 8,833 vs 8,860 tok/s just-in-time on one box, profiles/r4d_*: the
# concurrent transposes take CU time from the GEMMs, which fill every CU, about as much as they
# take off the critical path)
WT_PREFETCH = os.environ.get("DSA_WT_PREFETCH", "0") == "1"


class WeightTPrefetch:
    """W^T for the input gradients, made one linear AHEAD on a side stream.

    The reduction-contiguous dgrad (dx = dy W via W^T) transposes each weight once per micro-batch
    backward: memory-bound kernels (GPT-NeoX-20B: ~0.33 ms per layer) in the compute stream's
    dependency chain, 1.6 % of a 20B step.  The weights do not change during a backward, and the
    backward visits the linears in the same order every micro-batch, so the first backward of a
    run records that order and later ones transpose the NEXT weight into one of two persistent
    buffers on a side stream while the current linear's GEMMs run -- the transpose leaves the
    critical path (HBM traffic beside compute-bound GEMMs).  The side stream orders itself after
    everything already queued on the compute stream (the forward that waited for any overlapped
    optimizer step; the GEMM that last read the slot it overwrites); the consumer waits on the
    slot's event.  A pass whose order differs from the recorded one falls back to just-in-time
    transposes for the rest of that pass and re-records.  Bit-identical results."""

    def __init__(self):
        self.order = []  # weights in dgrad order, recorded from the previous backward
        self.seen = []  # this pass
        self.bufs = [None, None]
        self.ready = {}  # id(weight) -> (slot, event)
        self.stream = None
        self.next_slot = 0
        self.valid = True  # this pass still follows the recorded order
        self.hits = 0  # prefetched transposes consumed (tests / diagnostics)

    def _prefetch(self, w):
        if w.data.numel() != w.numel() or w.data.data_ptr() == 0:
            return  # a ZeRO-3 parameter released until re-gathered: transposed just in time
        from . import native
        slot = self.next_slot
        self.next_slot ^= 1
        n = w.numel()
        buf = self.bufs[slot]
        if buf is None or buf.numel() < n or buf.dtype != w.dtype or buf.device != w.device:
            self.bufs[slot] = buf = torch.empty(max(n, buf.numel() if buf is not None else 0), dtype=w.dtype,
                                                device=w.device)
        if self.stream is None:
            from ..runtime.overlap_step import new_stream
            self.stream = new_stream(w.device)
        cur = torch.cuda.current_stream(w.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            native.transpose2d(w.data, out=buf[:n].view(w.shape[1], w.shape[0]))
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self.ready[id(w)] = (slot, ev)

    def get(self, weight):
        """W^T [in, out] for this weight: the prefetched copy or a fresh transpose."""
        from . import native
        i = len(self.seen)
        if i >= 65536:  # no engine calls end_pass() (plain torch training): stop recording
            self.seen, self.order, self.valid, i = [], [], False, 0
        self.seen.append(weight)
        if self.valid and (i >= len(self.order) or self.order[i] is not weight):
            self.valid = False
        ent = self.ready.pop(id(weight), None)
        if ent is not None:
            self.hits += 1
            slot, ev = ent
            torch.cuda.current_stream(weight.device).wait_event(ev)
            wt = self.bufs[slot][:weight.numel()].view(weight.shape[1], weight.shape[0])
        else:
            wt = native.transpose2d(weight)
        if self.valid and i + 1 < len(self.order):
            self._prefetch(self.order[i + 1])
        return wt

    def end_pass(self):
        """End of a backward: the order just seen becomes the prefetch plan of the next one."""
        if self.seen:
            self.order = self.seen
        self.seen = []
        self.ready.clear()
        self.valid = True


_wt_prefetch = WeightTPrefetch()


# Weight transposes made once per optimizer step, off the critical path.  The reduction-contiguous
# input gradient needs W^T for every linear in every backward; the weights only change at the
# optimizer step.  With an engine that keeps whole weights resident (ZeRO stage < 3) the first
# FORWARD use of a weight after a step launches its transpose into a persistent buffer on a
# low-priority HIP stream of its own hardware queue -- beside the forward GEMMs, which leave CUs
# idle at BERT-Large's shapes -- and the backward (of every micro-batch until the next step) waits
# on that event instead of transposing just in time.  A cached transpose is used only while the
# weight's storage, its autograd version counter and the engine's step epoch (bumped after every
# optimizer step and checkpoint load: the fused optimizers write weights through raw pointers)
# all match the ones it was made from.  Opt-in (DSA_WT_CACHE=1): on BERT-Large it measured 3-4 %
# SLOWER than just-in-time transposes (2,318-2,353 vs 2,415 samples/s at seq 128, 536 vs 554 at
# seq 512, same box, profiles/r5e_bert_wt_cache_ab.jsonl) -- the concurrent transposes delay the
# forward's dependency chain by more than they take off the backward's.  It pays only where a
# step runs several micro-batches (one transpose per weight per step instead of per micro-batch).
# DSA_WT_CACHE_MAX_GB caps the buffers (default 8 GiB).
WT_CACHE = os.environ.get("DSA_WT_CACHE", "0") == "1"
WT_CACHE_MAX_BYTES = float(os.environ.get("DSA_WT_CACHE_MAX_GB", "8")) * 2**30


class WeightTCache:
    def __init__(self):
        self.enabled = False
        self.epoch = 0
        self.ent = {}  # id(weight) -> [weakref(weight), W^T buffer, key, event]
        self.bytes = 0
        self.stream = None
        self.hits = 0  # transposes served from the cache (tests / diagnostics)
        self.made = 0  # transposes launched by prepare()

    def enable(self, on: bool = True):
        self.enabled = bool(on) and WT_CACHE
        if not self.enabled:
            self.clear()

    def clear(self):
        if self.stream is not None and self.ent:
            torch.cuda.current_stream(self.stream.device).wait_stream(self.stream)
        self.ent.clear()
        self.bytes = 0

    def bump(self):
        """The weights may have changed (optimizer step, checkpoint load): every entry is stale."""
        self.epoch += 1
        dead = [k for k, e in self.ent.items() if e[0]() is None]
        for k in dead:
            e = self.ent.pop(k)
            self.bytes -= e[1].numel() * e[1].element_size()

    def _key(self, w):
        return (w.data_ptr(), w._version, self.epoch)

    def prepare(self, w, tokens: int):
        """Forward-time hook of a linear over `tokens` rows: make W^T for its backward."""
        if not (self.enabled and w.is_cuda and w.dim() == 2 and w.dtype in (torch.bfloat16, torch.float16)
                and DGRAD_NT and w.numel() >= DGRAD_NT_MIN_NUMEL and tokens >= 1024):
            return
        if torch.cuda.is_current_stream_capturing():
            return
        if lt_tune.DGRAD and lt_tune.use_dgrad(tokens, w.size(0), w.size(1)):
            return  # that input gradient reads W untransposed
        e = self.ent.get(id(w))
        key = self._key(w)
        if e is not None and e[0]() is w and e[2] == key:
            return
        from . import native
        if not native.transpose_supported(w):
            return
        if e is None or e[0]() is not w:
            n = w.numel() * w.element_size()
            if e is not None:
                self.bytes -= e[1].numel() * e[1].element_size()
                del self.ent[id(w)]
            if self.bytes + n > WT_CACHE_MAX_BYTES:
                return
            import weakref
            e = self.ent[id(w)] = [weakref.ref(w), torch.empty(w.shape[1], w.shape[0], dtype=w.dtype,
                                                               device=w.device), None, None]
            self.bytes += n
        if self.stream is None:
            from ..runtime.overlap_step import priority_stream
            self.stream = priority_stream(w.device, 1 << 20)  # lowest priority, own hardware queue
        cur = torch.cuda.current_stream(w.device)
        # after the optimizer step that wrote w and the backward GEMMs that last read the buffer
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            native.transpose2d(w.detach(), out=e[1])
            ev = torch.cuda.Event()
            ev.record(self.stream)
        e[2], e[3] = key, ev
        self.made += 1

    def get(self, w):
        """W^T made by prepare() for this weight's current value, or None."""
        e = self.ent.get(id(w)) if self.enabled else None
        if e is None or e[0]() is not w or e[2] != self._key(w):
            return None
        torch.cuda.current_stream(w.device).wait_event(e[3])
        self.hits += 1
        return e[1]


weight_t_cache = WeightTCache()


def end_backward_pass():
    clear_transposed()
    _wt_prefetch.end_pass()


def input_grad(g2: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """dx = g2 @ W for g2 = dy [M, out], W [out, in]."""
    if lt_tune.DGRAD and _lt_ok(g2, weight) and lt_tune.use_dgrad(g2.size(0), weight.size(0), weight.size(1)):
        # a measured NN solution runs at the TN rate: no weight transpose (ops/lt_tune.py)
        return _lt_ops().gemm_lt(g2, weight)
    if (DGRAD_NT and g2.is_cuda and g2.dtype == weight.dtype and weight.numel() >= DGRAD_NT_MIN_NUMEL
            and g2.size(0) >= 1024):
        from . import native
        wt = weight_t_cache.get(weight)
        if wt is None and _wb.state.wstacks:
            # a slot of a stacked weight: its W^T is a column block of one per-step stack transpose
            wt = _wb.stacked_wt(weight, weight_t_cache.epoch)
        if wt is not None:
            return g2 @ wt.t()
        if native.transpose_supported(weight):
            if WT_PREFETCH and not torch.cuda.is_current_stream_capturing():
                return g2 @ _wt_prefetch.get(weight).t()
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
    if (gw is not None and lt_tune.WGRAD and _lt_ok(g2, x2, gw) and (not has_b or _lt_ok(bias.grad))
            and lt_tune.wgrad_nt(g2.size(0), g2.size(1), x2.size(1), g2.element_size())):
        # one NT GEMM on the token-major operands, accumulated into the bound gradient: cheaper
        # than transposing both operands for this shape by the measured rates (ops/lt_tune.py)
        _lt_ops().gemm_lt(g2, x2, trans_a=True, out=gw, accumulate=True)
        if has_b:
            from . import native
            native.colsum(g2, bias.grad, accumulate=True)
        _count[0] += 1
        _lt_nt_count[0] += 1
        return None, None
    if gw is not None and gw.is_contiguous():
        nt = _nt_operands(g2, x2, bias.grad if has_b else None, offer_gt)
        if nt is not None:
            if lt_tune.WGRAD and gw.dtype == torch.bfloat16 and lt_tune.use_wgrad_t(g2.size(0), g2.size(1), x2.size(1)):
                _lt_ops().gemm_lt(nt[0], nt[1], trans_b=True, out=gw, accumulate=True)  # measured solution
            else:
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
    elif (lt_tune.WGRAD and _lt_ok(g2, x2, gw)
          and lt_tune.wgrad_nt(g2.size(0), g2.size(1), x2.size(1), g2.element_size())):
        _lt_ops().gemm_lt(g2, x2, trans_a=True, out=gw, accumulate=True)
    else:
        nt = _nt_operands(g2, x2, None) if gw.is_contiguous() else None
        if nt is None:
            gw.addmm_(g2.t(), x2)
        elif lt_tune.WGRAD and gw.dtype == torch.bfloat16 and lt_tune.use_wgrad_t(g2.size(0), g2.size(1), x2.size(1)):
            _lt_ops().gemm_lt(nt[0], nt[1], trans_b=True, out=gw, accumulate=True)
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
    if (LINEAR_LT and x.is_cuda and x.dtype in (torch.bfloat16, torch.float16) and weight.dtype == x.dtype
            and weight.is_contiguous() and x.is_contiguous() and x.numel() > 0
            and (bias is None or (bias.dtype == x.dtype and bias.is_contiguous()))):
        from . import native
        y = native.hip_ops().linear_lt(x.view(-1, x.shape[-1]), weight, bias, None, False, None)
        return y.view(*x.shape[:-1], weight.shape[0])
    return F.linear(x, weight, bias)


# Input and weight gradients of one linear on two streams when both GEMMs are too small to fill
# the chip (BERT-Large at 8k tokens: 48-512 output tiles of 256 x 256 each against 256 CUs): the
# dgrad runs on the compute stream, the wgrad (+ bias gradient) beside it on a side stream, and
# the compute stream waits for both before anything else -- autograd's gradient hooks and every
# later kernel see finished gradients, exactly as with the serial order.  Large linears (GPT-NeoX
# 20B: 768 + 576 tiles) stay serial: a GEMM that fills every CU gains nothing from company.
# Opt-in (DSA_PAR_WGRAD=1): on BERT-Large it measured 8 % SLOWER than the serial order (2,073 vs
# 2,258 samples/s at seq 128, 479 vs 519 at seq 512, profiles/r4e_notes.md) -- two hipBLASLt
# kernels sharing the CUs run each other's tiles into stragglers, and every linear adds two stream
# waits to a partly launch-bound step.  DSA_PAR_WGRAD_MAX_TILES bounds the summed tile count.
PAR_WGRAD = os.environ.get("DSA_PAR_WGRAD", "0") == "1"
PAR_WGRAD_MAX_TILES = int(os.environ.get("DSA_PAR_WGRAD_MAX_TILES", "768"))
_par_streams = {}
_par_count = [0]


def _tiles(a: int, b: int) -> int:
    return -(-a // 256) * -(-b // 256)


def _linear_backward(ctx, g):
    x, weight = ctx.saved_tensors
    bias = ctx.bias
    g2 = g.reshape(-1, g.shape[-1])
    x2 = x.reshape(-1, x.shape[-1])
    need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
    need_b = bias is not None and ctx.needs_input_grad[2]
    if (PAR_WGRAD and need_x and (need_w or need_b) and g2.is_cuda and not torch.cuda.is_current_stream_capturing()
            and _tiles(g2.size(0), weight.size(1)) + _tiles(weight.size(0), weight.size(1)) <= PAR_WGRAD_MAX_TILES):
        dev = g2.device
        side = _par_streams.get(dev)
        if side is None:
            from ..runtime.overlap_step import new_stream
            side = _par_streams[dev] = new_stream(dev)
        cur = torch.cuda.current_stream(dev)
        side.wait_stream(cur)
        dx = input_grad(g2, weight).view(x.shape)
        with torch.cuda.stream(side):
            dw, db = accumulate_param_grads(g2, x2, weight, bias, need_w, need_b, ctx.share_gt)
        cur.wait_stream(side)
        for t in (dw, db):  # made on the side stream, consumed by autograd on the compute stream
            if t is not None:
                t.record_stream(cur)
        _par_count[0] += 1
        return dx, dw, db, None
    dx = input_grad(g2, weight).view(x.shape) if need_x else None
    dw, db = accumulate_param_grads(g2, x2, weight, bias, need_w, need_b, ctx.share_gt)
    return dx, dw, db, None


class _AccumLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, share_gt=False):
        ctx.save_for_backward(x, weight)
        ctx.bias = bias
        ctx.share_gt = share_gt
        y = forward_gemm(x, weight, bias)
        if weight_t_cache.enabled and ctx.needs_input_grad[0]:
            weight_t_cache.prepare(weight, x.numel() // max(1, x.shape[-1]))
        return y

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
