"""ZeRO-Infinity parameter partitions on NVMe (reference parity:
deepspeed/runtime/swap_tensor/partitioned_param_swapper.py:36-308 `AsyncPartitionedParameterSwapper`,
`PartitionedParamStatus`).

Each (flat group, unit bucket) chunk of this rank's low-precision parameter shard is one file
under `<nvme_path>/zero_stage_3/params_rank<r>_mp<m>/`.  Nothing of the shard stays in host
RAM: a fetch reads the chunk through the C++ O_DIRECT engine (ops/csrc/cpu/aio.cpp) into one of
`buffer_count` page-aligned pinned buffers, and the caller stages it to HBM with an async
`hipMemcpyAsync` (torch non_blocking copy) whose completion event guards the buffer's reuse.
After the (offloaded) optimizer step the updated chunk is written from a pinned staging buffer
with an async write; `synchronize_writes()` retires them before the next fetch.

MI355X design notes: the pool holds whole unit chunks (a ZeRO-3 unit is at most
`stage3_unit_max_numel` elements, so one read per unit and rank, no per-parameter files), reads
and writes use separate aio handles so the step's write-back overlaps the next reads.
"""

import os
import shutil
from enum import Enum
from typing import Dict, Hashable, List, Optional

import torch

from .optimizer_utils import make_aio_handle
from .utils import aligned_numel, _pinned


class PartitionedParamStatus(Enum):
    AVAILABLE = 1      # in a pinned buffer
    NOT_AVAILABLE = 2  # on NVMe only
    INFLIGHT = 3       # read submitted


class AsyncPartitionedParameterSwapper:
    def __init__(self, folder: str, dtype: torch.dtype, buffer_count: int = 5, aio_config=None):
        self.folder = folder
        if os.path.isdir(folder):
            shutil.rmtree(folder, ignore_errors=True)
        os.makedirs(folder, exist_ok=True)
        self.dtype = dtype
        self.esize = torch.empty(0, dtype=dtype).element_size()
        self.buffer_count = max(2, int(buffer_count))
        self.read_h = make_aio_handle(aio_config)
        self.write_h = make_aio_handle(aio_config)
        self.numel: Dict[Hashable, int] = {}
        self.status: Dict[Hashable, PartitionedParamStatus] = {}
        self._buf_numel = 0
        self._pool: List[torch.Tensor] = []
        self._free: List[int] = []
        self._events: Dict[int, object] = {}   # buffer -> event of the H2D copy still reading it
        self._pending_writes: List[int] = []
        self.bytes_read = self.bytes_written = 0

    # -------------------------------------------------------------- files / buffers
    def path(self, key) -> str:
        k = "_".join(str(x) for x in (key if isinstance(key, tuple) else (key,)))
        return os.path.join(self.folder, f"p{k}.swp")

    def swappable_tensor(self, numel: int) -> bool:
        return numel > 0

    def _ensure_pool(self, numel: int):
        an = aligned_numel(numel, self.esize)
        if an <= self._buf_numel and self._pool:
            return
        self.synchronize_writes()
        self._wait_events()
        self._buf_numel = max(an, self._buf_numel)
        self._pool = [_pinned(self._buf_numel, self.dtype) for _ in range(self.buffer_count)]
        self._free = list(range(self.buffer_count))

    def _wait_events(self):
        for ev in self._events.values():
            if ev is not None:
                ev.synchronize()
        self._events.clear()

    def _acquire(self) -> int:
        if not self._free:
            self.synchronize_writes()
        if not self._free:
            raise RuntimeError("param swapper: no free pinned buffer (raise offload_param.buffer_count)")
        i = self._free.pop(0)
        ev = self._events.pop(i, None)
        if ev is not None:
            ev.synchronize()  # the previous H2D copy out of this buffer has finished
        return i

    def _release(self, i: int, event=None):
        if event is not None:
            self._events[i] = event
        self._free.append(i)

    # -------------------------------------------------------------- API
    def register(self, key, tensor: torch.Tensor):
        """Create `key`'s file from its initial (host) value."""
        n = tensor.numel()
        self.numel[key] = n
        self._ensure_pool(n)
        i = self._acquire()
        an = aligned_numel(n, self.esize)
        buf = self._pool[i][:an]
        buf.zero_()
        buf[:n].copy_(tensor.reshape(-1))
        assert self.write_h.sync_pwrite(buf, self.path(key)) >= 0
        self.bytes_written += an * self.esize
        self.status[key] = PartitionedParamStatus.NOT_AVAILABLE
        self._release(i)

    def read_to_device(self, key, device, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Read `key` from NVMe and stage it to `device` (async H2D on the current stream)."""
        n = self.numel[key]
        i = self._acquire()
        an = aligned_numel(n, self.esize)
        buf = self._pool[i][:an]
        self.status[key] = PartitionedParamStatus.INFLIGHT
        assert self.read_h.sync_pread(buf, self.path(key)) >= 0
        self.bytes_read += an * self.esize
        self.status[key] = PartitionedParamStatus.AVAILABLE
        if out is None:
            out = torch.empty(n, dtype=self.dtype, device=device)
        ev = None
        if out.is_cuda:
            out.copy_(buf[:n], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:
            out.copy_(buf[:n])
        self._release(i, ev)
        self.status[key] = PartitionedParamStatus.NOT_AVAILABLE
        return out

    def read(self, key) -> torch.Tensor:
        return self.read_to_device(key, "cpu")

    def staging(self, key) -> torch.Tensor:
        """A pinned buffer view receiving `key`'s new value; `swap_out(key)` writes it."""
        n = self.numel[key]
        i = self._acquire()
        self._staged = getattr(self, "_staged", {})
        self._staged[key] = i
        return self._pool[i][:n]

    def swap_out(self, key, async_op: bool = True):
        i = self._staged.pop(key)
        n = self.numel[key]
        an = aligned_numel(n, self.esize)
        buf = self._pool[i][:an]
        if an > n:
            buf[n:].zero_()
        if torch.cuda.is_available():
            torch.cuda.current_stream().synchronize()  # device->staging copies issued by the optimizer
        assert self.write_h.async_pwrite(buf, self.path(key)) == 0
        self.bytes_written += an * self.esize
        self._pending_writes.append(i)
        if not async_op:
            self.synchronize_writes()

    def write(self, key, value: torch.Tensor):
        buf = self.staging(key)
        buf.copy_(value.reshape(-1))
        self.swap_out(key, async_op=False)

    def synchronize_writes(self):
        if self._pending_writes:
            self.write_h.wait()
            for i in self._pending_writes:
                self._release(i)
            self._pending_writes = []

    def synchronize_reads(self):
        self.read_h.wait()

    def purge(self):
        self.synchronize_writes()
        shutil.rmtree(self.folder, ignore_errors=True)
