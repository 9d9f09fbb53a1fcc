"""Pinned-host parking for tensors kept between a checkpointed forward and its recompute.

Selective recompute (models/gpt_neox.py `NeoXAttention.stash_outputs`) keeps a layer's attention
tensors from the first forward so that the recompute in backward skips the QKV GEMM, the rotary
split and the flash forward.  HBM holds such stashes for as many layers as fit; `HostStash`
parks the others in pinned host memory instead (the reference's `cpu_checkpointing` idea,
checkpointing.py:356-478, applied to the stash): the device -> host copy runs on a copy stream
right after the layer's forward (the SDMA engines, not the CUs, move the bytes), and the
backward prefetches a layer's tensors host -> device while the layers above it are still in
backward, so the recompute finds them resident.

Ordering rules (all on-device, no host waits on the hot path):
  * the D2H copy waits for the producing kernels (event on the compute stream) and the source
    tensors are `record_stream`-ed on the copy stream, so the allocator cannot hand their memory
    to the compute stream before the copy has read it;
  * a layer's pinned buffers are reused every micro-batch: the next D2H into them waits for the
    previous H2D out of them;
  * the compute stream waits for a prefetch's H2D event before using the tensors;
  * at most `max_backlog` parked layers may have their D2H outstanding: beyond that the compute
    stream waits for the oldest copy, bounding the HBM those sources pin.

Measured (profiles/aux/host_stash_ab.log, 20B ZeRO-3 bench on one MI355X): parking the 21
non-HBM layers moves 7.9 GiB per forward each way, more than the PCIe link carries while the
forward runs, so the backlog waits stretched the step's forward from 1.02 s to 2.52 s (6951 vs
8328 tok/s).  The bench therefore leaves it off (opt-in: DSA_STASH_OFFLOAD=1); it pays only
where the forward is long relative to the stash (bigger micro-batch per layer, slower compute).
"""

from __future__ import annotations

import collections
from typing import Dict, List, Optional, Sequence

import torch


class StashEntry:
    __slots__ = ("owner", "host", "d2h_done", "dev", "h2d_done", "device")

    def __init__(self, owner, host, d2h_done, device):
        self.owner = owner
        self.host = host
        self.d2h_done = d2h_done
        self.dev: Optional[List[torch.Tensor]] = None
        self.h2d_done = None
        self.device = device


class HostStash:
    def __init__(self, max_backlog: int = 8):
        self.max_backlog = max(1, int(max_backlog))
        self._d2h = None
        self._h2d = None
        # per owner: pinned buffer sets not holding a parked stash, each with the event after
        # which it may be overwritten (the H2D that last read it); several sets per owner when
        # several forwards are in flight before their backwards (pipeline 1F1B)
        self._free: Dict[int, List[tuple]] = collections.defaultdict(list)
        self._backlog = collections.deque()  # d2h events of parked entries, oldest first
        self.parked_bytes = 0

    def _streams(self, device):
        if self._d2h is None:
            from ..overlap_step import new_stream
            self._d2h = new_stream(device)
            self._h2d = new_stream(device)
        return self._d2h, self._h2d

    def _take_buffers(self, owner: int, tensors: Sequence[torch.Tensor]):
        shapes = [(t.shape, t.dtype) for t in tensors]
        free = self._free[owner]
        for i, (bufs, ev) in enumerate(free):
            if [(b.shape, b.dtype) for b in bufs] == shapes:
                free.pop(i)
                return bufs, ev
        bufs = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in tensors]
        self.parked_bytes += sum(b.numel() * b.element_size() for b in bufs)
        return bufs, None

    def park(self, owner: int, tensors: Sequence[torch.Tensor]) -> StashEntry:
        """Start copying `tensors` to pinned buffers of this owner; returns the handle."""
        cur = torch.cuda.current_stream()
        d2h, _ = self._streams(tensors[0].device)
        while len(self._backlog) >= self.max_backlog:
            cur.wait_event(self._backlog.popleft())
        bufs, free_after = self._take_buffers(owner, tensors)
        ready = torch.cuda.Event()
        ready.record(cur)
        with torch.cuda.stream(d2h):
            d2h.wait_event(ready)
            if free_after is not None:
                d2h.wait_event(free_after)  # the last H2D out of these buffers has read them
            for t, b in zip(tensors, bufs):
                b.copy_(t, non_blocking=True)
                t.record_stream(d2h)
            done = torch.cuda.Event()
            done.record(d2h)
        self._backlog.append(done)
        return StashEntry(owner, bufs, done, tensors[0].device)

    def prefetch(self, entry: StashEntry):
        """Start the host -> device copy of a parked entry (idempotent); its pinned buffers
        return to the owner's free list, reusable once this copy has read them."""
        if entry.dev is not None or entry.host is None:
            return
        _, h2d = self._streams(entry.device)
        with torch.cuda.stream(h2d):
            h2d.wait_event(entry.d2h_done)
            entry.dev = [torch.empty(b.shape, dtype=b.dtype, device=entry.device) for b in entry.host]
            for d, b in zip(entry.dev, entry.host):
                d.copy_(b, non_blocking=True)
            entry.h2d_done = torch.cuda.Event()
            entry.h2d_done.record(h2d)
        self._free[entry.owner].append((entry.host, entry.h2d_done))
        entry.host = None

    def fetch(self, entry: StashEntry):
        """Device tensors of an entry, ordered on the current stream."""
        self.prefetch(entry)
        cur = torch.cuda.current_stream()
        cur.wait_event(entry.h2d_done)
        for d in entry.dev:
            d.record_stream(cur)
        out = tuple(entry.dev)
        entry.dev = None
        return out


_HOST_STASH: Optional[HostStash] = None


def host_stash() -> HostStash:
    global _HOST_STASH
    if _HOST_STASH is None:
        _HOST_STASH = HostStash()
    return _HOST_STASH
