"""Optimizer-state swapping to NVMe (reference parity:
deepspeed/runtime/swap_tensor/optimizer_utils.py:118-526 `OptimizerSwapper`,
partitioned_optimizer_swapper.py, pipelined_optimizer_swapper.py).

State is kept per (flat group, bucket) as one file per tensor name (fp32 master, exp_avg,
exp_avg_sq) under `<nvme_path>/zero_stage_<s>/rank<r>/`.  The pipelined swapper walks the
buckets with three pinned buffer sets: while bucket k is updated on the CPU (AVX-512 Adam,
result streamed to the GPU), bucket k+1 is being read and bucket k-1 written by the async I/O
engine (ops/csrc/cpu/aio.cpp: O_DIRECT, thread pool), so the step time approaches
max(disk bandwidth, CPU Adam) instead of their sum.
"""

import os
import shutil
from typing import Callable, Dict, Hashable, List, Sequence

import torch

from ...utils.logging import logger
from .utils import aligned_numel, _pinned


def _aio_module():
    from ...ops.builder import load
    return load("_cpu_ops")


def make_aio_handle(aio_config=None):
    c = dict(block_size=1 << 20, queue_depth=8, single_submit=False, overlap_events=True, thread_count=1)
    c.update(aio_config or {})
    return _aio_module().aio_handle(block_size=int(c["block_size"]), queue_depth=int(c["queue_depth"]),
                                    single_submit=bool(c["single_submit"]), overlap_events=bool(c["overlap_events"]),
                                    thread_count=max(1, int(c["thread_count"])))


class OptimizerSwapper:
    """Synchronous per-key swap in/out of named fp32 tensors (PartitionedOptimizerSwapper)."""

    def __init__(self, folder: str, names: Sequence[str] = ("master", "exp_avg", "exp_avg_sq"), aio_config=None):
        self.folder = folder
        if os.path.isdir(folder):
            shutil.rmtree(folder, ignore_errors=True)
        os.makedirs(folder, exist_ok=True)
        self.names = tuple(names)
        self.numel: Dict[Hashable, int] = {}
        self.read_h = make_aio_handle(aio_config)
        self.write_h = make_aio_handle(aio_config)
        self.max_numel = 0
        self._bufs: List[Dict[str, torch.Tensor]] = []
        self.bytes_read = self.bytes_written = 0

    def path(self, key, name):
        k = "_".join(str(x) for x in (key if isinstance(key, tuple) else (key,)))
        return os.path.join(self.folder, f"{k}_{name}.swp")

    def _ensure_buffers(self, sets):
        an = aligned_numel(self.max_numel, 4)
        while len(self._bufs) < sets:
            self._bufs.append({n: _pinned(an, torch.float32) for n in self.names})
        for b in self._bufs:
            if b[self.names[0]].numel() < an:
                for n in self.names:
                    b[n] = _pinned(an, torch.float32)

    def register(self, key, tensors: Dict[str, torch.Tensor], numel: int = None):
        """Create the swap files of `key` from initial values (missing names start at 0; with
        `numel` and no tensors, every name starts at 0)."""
        n = int(numel) if numel is not None else next(iter(tensors.values())).numel()
        self.numel[key] = n
        self.max_numel = max(self.max_numel, n)
        self._ensure_buffers(1)
        buf = self._bufs[0]
        an = aligned_numel(n, 4)
        for name in self.names:
            t = buf[name][:an]
            t.zero_()
            if name in tensors:
                t[:n].copy_(tensors[name].reshape(-1))
            assert self.write_h.sync_pwrite(t, self.path(key, name)) >= 0
        self.bytes_written += an * 4 * len(self.names)

    def _views(self, bufset, key):
        n = self.numel[key]
        an = aligned_numel(n, 4)
        return {name: bufset[name][:an] for name in self.names}, n

    def swap_in(self, key, bufset, async_op=False):
        views, _ = self._views(bufset, key)
        for name, t in views.items():
            assert self.read_h.async_pread(t, self.path(key, name)) == 0
            self.bytes_read += t.numel() * 4
        if not async_op:
            self.read_h.wait()

    def swap_out(self, key, bufset, async_op=False):
        views, _ = self._views(bufset, key)
        for name, t in views.items():
            assert self.write_h.async_pwrite(t, self.path(key, name)) == 0
            self.bytes_written += t.numel() * 4
        if not async_op:
            self.write_h.wait()

    def read(self, key, name) -> torch.Tensor:
        n = self.numel[key]
        t = torch.empty(aligned_numel(n, 4), dtype=torch.float32)
        assert self.read_h.sync_pread(t, self.path(key, name)) >= 0
        return t[:n].clone()

    def write(self, key, name, value: torch.Tensor):
        n = self.numel[key]
        t = torch.zeros(aligned_numel(n, 4), dtype=torch.float32)
        t[:n].copy_(value.reshape(-1))
        assert self.write_h.sync_pwrite(t, self.path(key, name)) >= 0

    def update(self, keys: Sequence, fn: Callable):
        """Sequential swap-in / fn(key, tensors) / swap-out (no overlap)."""
        self._ensure_buffers(1)
        for key in keys:
            self.swap_in(key, self._bufs[0])
            views, n = self._views(self._bufs[0], key)
            fn(key, {k: v[:n] for k, v in views.items()})
            self.swap_out(key, self._bufs[0])

    def purge(self):
        shutil.rmtree(self.folder, ignore_errors=True)


PartitionedOptimizerSwapper = OptimizerSwapper


class PipelinedOptimizerSwapper(OptimizerSwapper):
    """Read of bucket k+1 and write of bucket k-1 overlap the update of bucket k."""

    def update(self, keys: Sequence, fn: Callable):
        keys = list(keys)
        if not keys:
            return
        self._ensure_buffers(3)
        self.swap_in(keys[0], self._bufs[0], async_op=True)
        for i, key in enumerate(keys):
            cur = self._bufs[i % 3]
            self.read_h.wait()  # bucket i is resident
            if i + 1 < len(keys):
                # the set receiving bucket i+1 was written out two iterations ago
                self.write_h.wait()
                self.swap_in(keys[i + 1], self._bufs[(i + 1) % 3], async_op=True)
            views, n = self._views(cur, key)
            fn(key, {k: v[:n] for k, v in views.items()})
            self.swap_out(key, cur, async_op=True)
        self.write_h.wait()


def log_swap_config(folder, aio_config):
    logger.info(f"ZeRO-Infinity optimizer swapping to {folder} (aio={aio_config})")
