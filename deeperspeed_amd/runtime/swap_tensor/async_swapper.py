"""Asynchronous tensor swap-out through pinned staging buffers (reference parity:
deepspeed/runtime/swap_tensor/async_swapper.py:16-173)."""

import torch

from .utils import aligned_numel, swap_out_tensors


class AsyncTensorSwapper:
    def __init__(self, aio_handle, numel_alignment=None, timers=None):
        self.aio_handle = aio_handle
        self.numel_alignment = numel_alignment
        self.timers = timers
        self.free_buffers, self.ready = [], []
        self.outstanding = 0
        self.num_elements_swapped = 0

    def has_buffers(self):
        return len(self.free_buffers) > 0 or len(self.ready) > 0

    def add_buffers(self, buffer_list):
        self.free_buffers += [(b, 0) for b in buffer_list]

    def get_timer_names(self):
        return ["swap_submit_write", "swap_wait_write"]

    def release_buffers(self):
        self._wait()
        out = [b for b, _ in self.free_buffers]
        self.free_buffers = []
        return out

    def swap_out_tensors(self, tensor_list, path_list):
        for t, p in zip(tensor_list, path_list):
            self._swap_out_tensor(t, p)

    def _swap_out_tensor(self, tensor, path):
        if not self.free_buffers:
            self._wait()
        buf, _ = self.free_buffers.pop(0)
        n = tensor.numel()
        an = aligned_numel(n, tensor.element_size()) if self.numel_alignment is None else \
            (n + self.numel_alignment - 1) // self.numel_alignment * self.numel_alignment
        assert an <= buf.numel(), "swap buffer too small"
        staging = buf.narrow(0, 0, an)
        staging[:n].copy_(tensor.reshape(-1).to(staging.dtype))
        if an > n:
            staging[n:].zero_()
        swap_out_tensors(self.aio_handle, [staging], [path])
        self.ready.append(buf)
        self.outstanding += 1
        self.num_elements_swapped += n

    def _wait(self):
        if self.outstanding:
            self.aio_handle.wait()
        self.outstanding = 0
        self.free_buffers += [(b, 0) for b in self.ready]
        self.ready = []
