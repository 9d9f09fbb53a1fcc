"""Layer-batched weight gradients for deep stacks of equal layers.

A BERT-Large encoder layer has four linears whose weight gradients dW = dY^T X (a reduction over
the 8k tokens of a step) are each too small for 256 CUs: 16-64 output tiles of 256 x 256, so the
per-layer path splits the token reduction four ways and folds fp32 partials (0.4-0.7 PF/s; ~6.5 ms
of a 26.5 ms seq-128 step).  The same gradient of all 24 layers together is 384-1536 tiles -- one
strided-batched hipBLASLt GEMM at 0.7-1.1 PF/s (profiles/r5f_wgrad_batched.jsonl).  hipBLASLt's
grouped GEMM (per-problem pointers) rejects every solution on this build and rocBLAS's pointer-array
batched GEMM runs at ~3 TF/s, so the operands must sit at a constant stride:

* slabs -- the producers of every X and dY of these linears (LayerNorm, bias-GeLU, encoder flash
  attention forward and backward, the fused dropout + LayerNorm backward) write into per-layer
  slots of persistent [layers, ...] buffers (`view`), at most one buffer per kind (a new shape
  replaces an idle buffer; a kind whose shape keeps changing -- progressive layer drop, varying
  batch shapes -- stops using slabs).  A slot belongs to the pass that took it: an engine forward
  (`begin_forward` / `end_forward` tag its slots and hook its output's autograd node) or the
  backward that runs (its own slots and recomputes).  The end of a backward frees only its own
  slots and those of the forwards whose graph it ran through, so with two forwards in flight the
  other one's saved activations are never lent again; a taken slot simply gets ordinary memory;
* gradient stacks -- the parameters of equal shape get their .grad bound to slots of one
  [layers, out, in] buffer (`bind_grad_stacks`, persistent gradients zeroed in place by the
  optimizer);
* deferral -- inside an engine backward whose gradients nobody reads before it returns (no ZeRO
  bucket hooks), ops/linear.py records (dY, X, dW) instead of running the GEMM (`record`), and the
  end of the backward runs each shape's records as ONE batched GEMM when all three operands are
  consecutive slots of their buffers (`flush`), else one GEMM per record.

Bias gradients are still formed in place.  Same math as the per-layer path up to fp32 summation
order.  No reference counterpart: the reference computes each
layer's weight gradients inside its layer backward (csrc/transformer/ds_transformer_cuda.cpp:370-540).
"""

from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch

ENABLED = True
MIN_TOKENS = 1024
# a kind whose slab shape changed this many times (progressive layer drop, varying batch shapes)
# stops using slabs: each change would allocate a fresh [count, ...] buffer
MAX_RESHAPES = 3
# the batched GEMMs through the extension's strided-batched hipBLASLt call, whose solution is timed
# per shape on first use (gemm_lt_batched), instead of torch.baddbmm_'s first heuristic answer
LT_BATCHED = True


def _batched_gemm(dy: torch.Tensor, x: torch.Tensor, dw: torch.Tensor) -> None:
    """dw[l] += dy[l]^T x[l] over contiguous [L, M, N] / [L, M, K] / [L, N, K] slab views."""
    if LT_BATCHED and dy.is_cuda and dy.dtype in (torch.bfloat16, torch.float16) and x.dtype == dy.dtype \
            and dw.dtype in (dy.dtype, torch.float32) and dy.is_contiguous() and x.is_contiguous() \
            and dw.is_contiguous():
        from . import native
        native.hip_ops().gemm_lt_batched(dy, x, True, False, dw, True)
    else:
        dw.baddbmm_(dy.transpose(1, 2), x)


class _Slab:
    def __init__(self, buf: torch.Tensor, key=None):
        self.buf = buf
        self.key = key
        self.busy = [None] * buf.shape[0]  # owner tag of each lent slot (None = free)
        self.slot_bytes = buf[0].numel() * buf.element_size()
        self.base = buf.data_ptr()

    def slot_of(self, t: torch.Tensor) -> Optional[int]:
        off = t.data_ptr() - self.base
        if off < 0 or off % self.slot_bytes or off // self.slot_bytes >= len(self.busy):
            return None
        if t.numel() != self.buf[0].numel():
            return None
        return off // self.slot_bytes


class _State:
    def __init__(self):
        self.slabs_on = False  # set by an engine whose backward may defer (no gradient hooks)
        self.slabs: Dict[str, _Slab] = {}  # one per kind
        self.reshapes: Dict[str, int] = {}
        self.off_kinds = set()  # kinds whose shape kept changing
        self.fwd = None  # tag of the engine forward running (begin_forward)
        self.next_tag = 1
        self.bwd = None  # tag of the deferred backward running
        self.seen = set()  # forward tags whose graph the running backward reached
        self.stacks: List[_Slab] = []  # persistent gradient stacks
        self.defer = False
        self.pending: List[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]] = []
        self.batched = 0  # batched GEMMs launched (tests / diagnostics)
        self.single = 0  # records run one by one
        self.recorded = 0
        self.last_miss = None  # why the last group could not be batched (diagnostics)
        # a whole training step is being captured as one HIP graph (runtime/step_graph): slots
        # lent and the deferred weight gradients flushed inside that one graph stay valid, so
        # slabs and deferral keep working (per-layer graphs share no slot state: off there)
        self.whole_step_capture = False


state = _State()


def _capture_blocks() -> bool:
    return torch.cuda.is_current_stream_capturing() and not state.whole_step_capture


def enable(on: bool = True):
    """An engine whose gradients are only read after its backward returns turns slabs on."""
    state.slabs_on = bool(on) and ENABLED


def view(kind: str, index: int, count: int, like: torch.Tensor, backward: bool = False) -> Optional[torch.Tensor]:
    """Slot `index` of the [count, *like.shape] slab `kind`, or None (slabs off, the kind's shape
    unstable, the slot taken by a pass still in flight).  Callers ask only for tensors of a forward
    that records a graph (inside an autograd Function grad mode is off, so the caller decides that
    before entering it).  The slot is tagged with its owner: the running deferred backward (its
    recomputes and input gradients), else the running engine forward, else an anonymous pass that
    the next backward end frees."""
    if not (state.slabs_on and like.is_cuda and 0 <= index < count) or count < 2 or kind in state.off_kinds:
        return None
    if _capture_blocks():
        return None
    key = (count, tuple(like.shape), like.dtype, like.device)
    slab = state.slabs.get(kind)
    if slab is not None and slab.key != key:
        if any(t is not None for t in slab.busy):
            return None  # the old buffer is still read by a pass in flight
        n = state.reshapes[kind] = state.reshapes.get(kind, 0) + 1
        del state.slabs[kind]
        slab = None
        if n >= MAX_RESHAPES:
            state.off_kinds.add(kind)
            return None
    if slab is None:
        slab = state.slabs[kind] = _Slab(torch.empty((count,) + tuple(like.shape), dtype=like.dtype,
                                                     device=like.device), key)
    if slab.busy[index] is not None:
        return None
    slab.busy[index] = ("b", state.bwd) if state.bwd is not None else (("f", state.fwd) if state.fwd is not None
                                                                       else ("a", 0))
    return slab.buf[index]


def begin_forward():
    """An engine forward starts: the slots it takes are its own until a backward reaches its graph."""
    if not state.slabs_on:
        return None
    state.fwd = state.next_tag
    state.next_tag += 1
    return state.fwd


def end_forward(tag, outputs):
    """Hook the autograd nodes of the forward's outputs, so the backward that runs through this
    forward's graph (even from a loss derived from them) frees its slots; a forward without a graph
    frees them now."""
    state.fwd = None
    if tag is None:
        return
    ts = [outputs] if isinstance(outputs, torch.Tensor) else (
        list(outputs.values()) if isinstance(outputs, dict) else list(outputs) if isinstance(outputs, (tuple, list))
        else [])
    nodes = [t.grad_fn for t in ts if isinstance(t, torch.Tensor) and t.grad_fn is not None]
    if not nodes:
        _free(lambda o: o == ("f", tag))
        return
    for node in nodes:
        node.register_prehook(lambda grad_out, _t=tag: state.seen.add(_t))


def _free(pred):
    for slab in state.slabs.values():
        slab.busy = [None if (o is not None and pred(o)) else o for o in slab.busy]


def release(tag=None):
    """End of a backward: its own slots, the slots of the forwards whose graph it ran through and
    anonymous slots may be written again."""
    seen, state.seen = state.seen, set()
    _free(lambda o: o == ("b", tag) or o[0] == "a" or (o[0] == "f" and o[1] in seen))


def bind_grad_stacks(params, min_count: int = 4, min_numel: int = 1 << 20) -> int:
    """Bind the .grad of every group of >= min_count equal-shape parameters -- weights of >= min_numel
    elements, and the 1-D biases / LayerNorm parameters whose in-place gradient sums let their
    linear's weight gradient be deferred -- to consecutive slots of one zeroed [n, *shape] buffer
    (persistent gradients: the fp16 optimizer zeroes them in place instead of dropping them).
    Returns the number of parameters bound."""
    groups: Dict[tuple, list] = {}
    for p in params:
        if (p.requires_grad and p.is_cuda and (p.dim() == 1 or (p.dim() == 2 and p.numel() >= min_numel))
                and not _captured(p)):
            groups.setdefault((tuple(p.shape), p.dtype, p.device), []).append(p)
    n = 0
    for (shape, dtype, dev), ps in groups.items():
        if len(ps) < min_count:
            continue
        buf = torch.zeros((len(ps),) + shape, dtype=dtype, device=dev)
        for i, p in enumerate(ps):
            if p.grad is not None:  # keep what was accumulated before binding
                buf[i].copy_(p.grad)
            p.grad = buf[i]
            p._dsa_persistent_grad = True
        state.stacks.append(_Slab(buf))
        n += len(ps)
    return n


def _captured(p) -> bool:
    """A parameter whose storage or .grad address a HIP graph holds (make_graphed_encoder), or whose
    .grad is already a persistent buffer someone else bound: rebinding it would leave the graph
    writing into freed memory."""
    return getattr(p, "_dsa_graph_captured", False) or getattr(p, "_dsa_persistent_grad", False)


def zero_stacks(grads):
    """Zero persistent gradients in place: the gradient stacks among them as whole buffers (one
    fill each instead of one per tensor); returns the gradients that are not stack slots."""
    rest, hit = [], set()
    for g in grads:
        o = _owner(g, state.stacks) if state.stacks else None
        if o is None:
            rest.append(g)
        else:
            hit.add(id(o[0]))
    for slab in state.stacks:
        if id(slab) in hit:
            slab.buf.zero_()
    return rest


class deferred:
    """Context of one backward whose bound weight gradients are recorded and run at its end."""

    def __init__(self, enabled: bool = True):
        self.enabled = bool(enabled) and ENABLED

    def __enter__(self):
        self.owner = self.enabled and not state.defer
        if self.owner:
            state.defer = True
            state.bwd = self.tag = state.next_tag
            state.next_tag += 1
            state.seen = set()
        return self

    def __exit__(self, exc_type, exc, tb):
        if not self.owner:
            return False
        state.defer = False
        state.bwd = None
        if exc_type is not None:
            state.pending.clear()
            release(self.tag)
            return False
        flush()
        release(self.tag)
        return False


def deferrable(g2: torch.Tensor, x2: torch.Tensor, gw: torch.Tensor) -> bool:
    return (state.defer and g2.is_cuda and g2.dtype in (torch.bfloat16, torch.float16) and x2.dtype == g2.dtype
            and gw.dtype == g2.dtype and g2.dim() == 2 and x2.dim() == 2 and g2.is_contiguous()
            and x2.is_contiguous() and gw.is_contiguous() and g2.size(0) >= MIN_TOKENS
            and not _capture_blocks())


def in_slab(t: torch.Tensor) -> bool:
    """t is a slot of a slab: worth deferring (a record whose input is ordinary memory can never
    join a batched GEMM, so it runs where autograd reaches it)."""
    return any(slab.slot_of(t) is not None for slab in state.slabs.values())


def record(g2: torch.Tensor, x2: torch.Tensor, gw: torch.Tensor):
    if gw.requires_grad:
        raise RuntimeError(f"wgrad_batch.record: gradient buffer requires grad: shape {tuple(gw.shape)} "
                           f"leaf {gw.is_leaf} param {isinstance(gw, torch.nn.Parameter)} base "
                           f"{None if gw._base is None else tuple(gw._base.shape)}")
    state.pending.append((g2, x2, gw))
    state.recorded += 1


def _key(g2, x2):
    return (tuple(g2.shape), tuple(x2.shape), g2.dtype, g2.device)


def _owner(t: torch.Tensor, pools) -> Optional[Tuple[_Slab, int]]:
    for slab in pools:
        i = slab.slot_of(t)
        if i is not None:
            return slab, i
    return None


def _batch(items):
    """(dY [L, M, N], X [L, M, K], dW [L, N, K]) strided views over consecutive slots when every
    record's operands sit in one slab each, in the same slot order; else None."""
    slabs = list(state.slabs.values())
    locs = []
    for g2, x2, gw in items:
        a, b, c = _owner(g2, slabs), _owner(x2, slabs), _owner(gw, state.stacks)
        if a is None or b is None or c is None:
            state.last_miss = ("operand outside the slabs", tuple(g2.shape), tuple(x2.shape), a is None, b is None,
                               c is None)
            return None
        locs.append((a, b, c))
    order = sorted(range(len(items)), key=lambda i: locs[i][1][1])
    views = []
    for k in range(3):
        slab0 = locs[order[0]][k][0]
        first = locs[order[0]][k][1]
        for j, i in enumerate(order):
            s, idx = locs[i][k]
            if s is not slab0 or idx != first + j:
                state.last_miss = ("slots not consecutive", k, [locs[i][k][1] for i in order])
                return None
        rows, cols = items[0][k].shape
        views.append(slab0.buf[first:first + len(items)].view(len(items), rows, cols))
    return views


@torch.no_grad()
def flush():
    """Run every recorded weight gradient (see the module docstring).  Gradient accumulation is
    not part of any graph: the GEMMs run outside autograd, as they would inside the backward."""
    pend, state.pending = state.pending, []
    groups: Dict[tuple, list] = {}
    for g2, x2, gw in pend:
        groups.setdefault(_key(g2, x2), []).append((g2, x2, gw))
    for items in groups.values():
        if len(items) > 1 and len({gw.data_ptr() for _, _, gw in items}) == len(items):
            v = _batch(items)
            if v is not None:
                dy, x, dw = v
                _batched_gemm(dy, x, dw)
                state.batched += 1
                continue
        from .linear import wgrad_into
        for g2, x2, gw in items:  # a weight used twice accumulates in order, by the per-layer path
            wgrad_into(g2, x2, gw)
            state.single += 1
