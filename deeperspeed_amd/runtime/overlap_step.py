"""Optimizer step overlapped with the next forward pass (MI355X extension).

`zero_optimization.overlap_step`: the optimizer math of one step (fused LAMB / Adam, HBM-bound)
runs on a side HIP stream, bucket by bucket in forward order, while the next forward's GEMMs
(compute-bound) start on the compute stream.  Each module's forward pre-hook waits only for the
events of the bucket(s) holding its own parameters, so layer 0 resumes as soon as the first
bucket is updated instead of after the whole step.

The reference runs the step serially between backward and the next forward
(deepspeed/runtime/engine.py:896-930 `_take_model_step`); the numerics here are identical --
only the stream placement changes.  Parameters read outside their owning module's forward (tied
weights used through F.linear by another module) are covered by a calibration pass: the first
overlapped forward waits for the whole step at the root module and records which modules' hooks
fire; afterwards the root waits for the buckets of every module that did not.

Used by the per-tensor mixed-precision wrapper (runtime/fp16/unfused_optimizer.py, LAMB).
"""

from __future__ import annotations

import contextlib
from typing import Dict, List, Sequence

import torch

# Side / copy streams are torch pool streams.  Measured alternatives, removed: hardware queues of
# their own for every side stream (20B N=1: 8,720 vs 8,868 tok/s, profiles/r4s_notes.md), HIP
# low-priority streams (same step time, profiles/r5d_notes.md), a CU-masked step stream.  Only the
# offloaded optimizer step -- which IS the critical path -- puts its copy streams on dedicated
# hardware queues (ZeRO sharded_base._new_stream, profiles/r4ag_notes.md).


def side_stream(device, num_cus: int = 0) -> torch.cuda.Stream:
    """A side stream; with num_cus > 0 one restricted to that many CUs (ops/csrc/bindings.cpp
    cu_masked_stream), else a stream on a hardware queue of its own (new_stream)."""
    if num_cus <= 0:
        return new_stream(device)
    from ..ops import native
    hip = native.hip_ops()
    total = int(hip.device_cu_count())
    num_cus = min(num_cus, total)
    step = total / num_cus
    bits = {int(i * step) for i in range(num_cus)}
    words = [0] * ((total + 31) // 32)
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    return torch.cuda.ExternalStream(hip.cu_masked_stream(words), device=device)


def dedicated_stream(device) -> torch.cuda.Stream:
    """A stream on a hardware queue of its own.  HIP spreads ordinary streams over
    GPU_MAX_HW_QUEUES (4) pooled queues, so a copy or optimizer stream can share the compute
    stream's queue, and its cross-stream waits (barrier packets) then stall the compute stream's
    kernels (profiles/r4q_notes.md).  A CU-masked stream gets a queue of its own; the mask here
    enables every CU, so only the queue differs."""
    return side_stream(device, 1 << 30)


_keep = []  # external streams live for the process (torch does not own them)


def priority_stream(device, priority: int) -> torch.cuda.Stream:
    from ..ops import native
    hip = native.hip_ops()
    least, greatest = hip.stream_priority_range()
    priority = max(min(int(priority), least), greatest)
    with torch.cuda.device(device):
        s = torch.cuda.ExternalStream(hip.priority_stream(priority), device=device)
    _keep.append(s)
    return s


def new_stream(device) -> torch.cuda.Stream:
    """The framework's side / copy streams: streams from torch's pool."""
    return torch.cuda.Stream(device=device)


def _in_backward() -> bool:
    return torch._C._current_graph_task_id() != -1


def forward_order_buckets(module: torch.nn.Module, params: Sequence[torch.nn.Parameter],
                          bucket_numel: int) -> List[List[int]]:
    """Indices into `params`, grouped into buckets of >= bucket_numel elements in the order the
    module tree registers them (forward order for sequential models).  Parameters not owned by
    any module of the tree form the last bucket."""
    pos = {id(p): i for i, p in enumerate(params)}
    order, seen = [], set()
    for m in module.modules():
        for p in m.parameters(recurse=False):
            i = pos.get(id(p))
            if i is not None and i not in seen:
                seen.add(i)
                order.append(i)
    rest = [i for i in range(len(params)) if i not in seen]
    buckets, cur, n = [], [], 0
    for i in order:
        cur.append(i)
        n += params[i].numel()
        if n >= bucket_numel:
            buckets.append(cur)
            cur, n = [], 0
    if cur:
        buckets.append(cur)
    if rest:
        buckets.append(rest)
    return buckets


class OverlapStep:
    """Side stream + per-bucket events + the forward pre-hooks that wait on them."""

    def __init__(self, module: torch.nn.Module, params: Sequence[torch.nn.Parameter], buckets: List[List[int]],
                 device):
        self.stream = new_stream(device)
        owner = {id(params[i]): b for b, idxs in enumerate(buckets) for i in idxs}
        self._module_buckets: Dict[torch.nn.Module, list] = {}
        self._handles = []
        for m in module.modules():
            # a parameter registered in several modules (tied weights) is waited for by each
            keys = sorted({owner[id(p)] for p in m.parameters(recurse=False) if id(p) in owner})
            if keys:
                self._module_buckets[m] = keys
                self._handles.append(m.register_forward_pre_hook(self._wait_module))
        self._handles.append(module.register_forward_pre_hook(self._root_wait))
        self._events: Dict[int, torch.cuda.Event] = {}
        self._done = None
        self._calibrating = False
        self._fired = set()
        self._uncovered = None  # bucket keys the root waits for; None = not calibrated yet

    # ------------------------------------------------------------------ hooks
    def _root_wait(self, module, inputs):
        if not self._events or _in_backward():
            return
        cur = torch.cuda.current_stream()
        if self._uncovered is None:
            cur.wait_event(self._done)  # calibration pass: the whole step
            self._calibrating = True
            self._fired = set()
            return
        for key in self._uncovered:
            ev = self._events.get(key)
            if ev is not None:
                cur.wait_event(ev)

    def _wait_module(self, module, inputs):
        if self._calibrating:
            self._fired.add(module)
        if not self._events or _in_backward():
            return
        cur = torch.cuda.current_stream()
        for key in self._module_buckets.get(module, ()):
            ev = self._events.get(key)
            if ev is not None:
                cur.wait_event(ev)

    # ------------------------------------------------------------------ step
    @contextlib.contextmanager
    def launch(self):
        """Context in which the step's kernels are issued on the side stream (after everything
        already queued on the compute stream)."""
        self.synchronize()
        side, cur = self.stream, torch.cuda.current_stream()
        side.wait_stream(cur)
        self._events = {}
        with torch.cuda.stream(side):
            yield side
        self._done = torch.cuda.Event()
        self._done.record(side)

    def bucket_done(self, key: int):
        ev = torch.cuda.Event()
        ev.record(self.stream)
        self._events[key] = ev

    def synchronize(self):
        """Order the compute stream after the whole overlapped step (no host wait)."""
        if self._calibrating:
            self._calibrating = False
            self._uncovered = sorted({k for m, keys in self._module_buckets.items() if m not in self._fired
                                      for k in keys})
        if self._done is not None:
            torch.cuda.current_stream().wait_event(self._done)
            self._done = None
            self._events = {}

    def remove(self):
        for h in self._handles:
            h.remove()
        self._handles = []
