"""Defragmenting arena allocator for parameter storage.

Reference parity: deepspeed/runtime/zero/contiguous_memory_allocator.py:9-283.  One large
device buffer; tensors are views into it; when a request does not fit in any single free
block but the total free space suffices, live tensors are compacted to the front (their
owners' `.data` is re-pointed) so the request can be served contiguously.
"""

import torch


class ContiguousMemoryAllocator:
    def __init__(self, size, dtype, device):
        self.buffer = torch.zeros(size, dtype=dtype, device=device)
        self.size = size
        self.total_free = size
        self.largest_contiguous = size
        self._max_allocated = 0
        self.contiguous_sizes = {0: size}  # free blocks: address -> size
        self.tensor_addresses = {}  # tensor id -> address
        self.tensor_sizes = {}  # address -> size
        self.tensor_ids = {}  # address -> tensor id
        self.tensor_map = {}  # tensor id -> tensor view
        self.id_to_params = {}  # tensor id -> [params using it]
        self.count = 0

    # --------------------------------------------------------------- public API
    def allocate_tensor(self, size):
        assert size <= self.total_free, f"not enough memory: asked {size}, free {self.total_free}"
        if self.largest_contiguous < size:
            self._defragment_memory()
        addr = self._best_fit(size)
        t = self._carve(addr, size)
        self._max_allocated = max(self._max_allocated, self.size - self.total_free)
        return t

    def assign_to_param(self, tensor, param, numel, shape):
        tid = id(tensor)
        assert tid in self.tensor_map, "tensor was not allocated by this allocator"
        assert tensor.numel() >= numel
        self.id_to_params.setdefault(tid, []).append(param)
        param.data = tensor.narrow(0, 0, numel).view(shape)

    def release_tensor(self, tensor):
        tid = id(tensor)
        addr = self.tensor_addresses.pop(tid)
        size = self.tensor_sizes.pop(addr)
        self.tensor_ids.pop(addr)
        self.tensor_map.pop(tid)
        self.id_to_params.pop(tid, None)
        self.total_free += size
        self.contiguous_sizes[addr] = size
        self._coalesce()

    def release_tensor_with_id(self, tid):
        self.release_tensor(self.tensor_map[tid])

    def print_allocation(self, resolution=200):
        out = ["."] * resolution
        for addr, size in self.tensor_sizes.items():
            lo = addr * resolution // self.size
            hi = max(lo + 1, (addr + size) * resolution // self.size)
            for i in range(lo, min(hi, resolution)):
                out[i] = "|"
        print("".join(out))

    def max_allocated(self):
        return self._max_allocated

    # --------------------------------------------------------------- internals
    def _best_fit(self, size):
        best, best_size = None, None
        for addr, sz in self.contiguous_sizes.items():
            if sz >= size and (best_size is None or sz < best_size):
                best, best_size = addr, sz
        assert best is not None, "no contiguous block after defragmentation"
        return best

    def _carve(self, addr, size):
        free = self.contiguous_sizes.pop(addr)
        if free > size:
            self.contiguous_sizes[addr + size] = free - size
        t = self.buffer.narrow(0, addr, size)
        tid = id(t)
        self.tensor_addresses[tid] = addr
        self.tensor_sizes[addr] = size
        self.tensor_ids[addr] = tid
        self.tensor_map[tid] = t
        self.total_free -= size
        self._update_largest()
        return t

    def _coalesce(self):
        merged = {}
        for addr in sorted(self.contiguous_sizes):
            size = self.contiguous_sizes[addr]
            if merged:
                last = max(merged)
                if last + merged[last] == addr:
                    merged[last] += size
                    continue
            merged[addr] = size
        self.contiguous_sizes = merged
        self._update_largest()

    def _update_largest(self):
        self.largest_contiguous = max(self.contiguous_sizes.values()) if self.contiguous_sizes else 0

    def _defragment_memory(self):
        """Slide every live tensor to the lowest free address (in address order)."""
        cur = 0
        for addr in sorted(self.tensor_sizes):
            size = self.tensor_sizes[addr]
            tid = self.tensor_ids[addr]
            if addr != cur:
                self.buffer.narrow(0, cur, size).copy_(self.buffer.narrow(0, addr, size).clone())
                new_t = self.buffer.narrow(0, cur, size)
                old_t = self.tensor_map.pop(tid)
                old_t.data = new_t.data  # existing references see the new storage
                self.tensor_map[tid] = old_t
                self.tensor_addresses[tid] = cur
                del self.tensor_sizes[addr], self.tensor_ids[addr]
                self.tensor_sizes[cur] = size
                self.tensor_ids[cur] = tid
                for p in self.id_to_params.get(tid, []):
                    p.data = old_t.narrow(0, 0, p.numel()).view(p.shape)
            cur += size
        self.contiguous_sizes = {cur: self.size - cur} if cur < self.size else {}
        self._update_largest()
