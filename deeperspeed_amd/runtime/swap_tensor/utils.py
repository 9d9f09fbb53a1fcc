"""Pinned, aligned host buffers for NVMe swapping (reference parity:
deepspeed/runtime/swap_tensor/utils.py:37-241 `SwapBuffer`, `SwapBufferPool`,
`SwapBufferManager`).  O_DIRECT I/O needs 4 KiB-aligned sizes, so every buffer is rounded up
to `numel_alignment` elements."""

from typing import List

import torch

AIO_ALIGNED_BYTES = 4096


def swap_in_tensors(swap_handle, tensor_buffers, swap_paths):
    for buf, path in zip(tensor_buffers, swap_paths):
        assert swap_handle.async_pread(buf, path) == 0


def swap_out_tensors(swap_handle, tensor_buffers, swap_paths):
    for buf, path in zip(tensor_buffers, swap_paths):
        assert swap_handle.async_pwrite(buf, path) == 0


def get_sized_buffer(buffer, num_elems):
    assert num_elems <= buffer.numel()
    return buffer.narrow(0, 0, num_elems) if num_elems < buffer.numel() else buffer


def aligned_numel(numel, element_size):
    align = AIO_ALIGNED_BYTES // element_size
    return (numel + align - 1) // align * align


def _pinned(numel, dtype):
    from ...ops import native
    return native.pinned_zeros(numel, dtype)


class SwapBuffer:
    def __init__(self, buffer):
        self.buffer = buffer
        self.reset()

    def reset(self):
        self.offset = 0
        self.swap_tensors = {}
        self.compute_tensors = {}
        self.swap_paths = {}
        self.num_elem = 0

    def insert_tensor(self, tensor, swap_path, aligned_numel_):
        swap_tensor, compute_tensor = self.allocate_tensor(swap_path, tensor.numel(), aligned_numel_)
        compute_tensor.data.copy_(tensor.data)
        return swap_tensor, compute_tensor

    def allocate_tensor(self, swap_path, numel, aligned_numel_):
        assert self.has_space(aligned_numel_)
        assert self.offset not in self.swap_tensors
        swap_tensor = self.buffer.narrow(0, self.offset, aligned_numel_)
        compute_tensor = swap_tensor.narrow(0, 0, numel)
        self.swap_tensors[self.offset] = swap_tensor
        self.compute_tensors[self.offset] = compute_tensor
        self.swap_paths[self.offset] = swap_path
        self.offset += aligned_numel_
        self.num_elem += numel
        return swap_tensor, compute_tensor

    def has_space(self, numel):
        return self.offset + numel <= self.buffer.numel()

    def get_swap_tensors(self):
        return list(self.swap_tensors.values())

    def get_swap_paths(self):
        return list(self.swap_paths.values())

    def get_compute_tensors(self):
        return list(self.compute_tensors.values())

    def get_num_elem(self):
        return self.num_elem


class SwapBufferPool:
    def __init__(self, buffers: List[torch.Tensor]):
        self.buffers = [SwapBuffer(b) for b in buffers]
        self.current = 0

    def reset(self):
        self.current = 0
        for b in self.buffers:
            b.reset()

    def allocate_tensor(self, numel, swap_path, aligned_numel_):
        if self.has_space(aligned_numel_):
            return self._get_current_buffer().allocate_tensor(swap_path, numel, aligned_numel_)
        return None, None

    def insert_tensor(self, tensor, swap_path, aligned_numel_):
        if self.has_space(aligned_numel_):
            return self._get_current_buffer().insert_tensor(tensor, swap_path, aligned_numel_)
        return None, None

    def has_space(self, numel):
        if self._get_current_buffer().has_space(numel):
            return True
        if self.current == len(self.buffers) - 1:
            return False
        self.current += 1
        return self._get_current_buffer().has_space(numel)

    def swap_out(self, aio_handle, async_op=False):
        for b in self._get_used_buffers():
            swap_out_tensors(aio_handle, b.get_swap_tensors(), b.get_swap_paths())
        if not async_op:
            assert len(self._get_used_buffers()) == 0 or aio_handle.wait() >= 0

    def swap_in(self, aio_handle, async_op=False):
        for b in self._get_used_buffers():
            swap_in_tensors(aio_handle, b.get_swap_tensors(), b.get_swap_paths())
        if not async_op:
            aio_handle.wait()

    def _get_current_buffer(self):
        return self.buffers[self.current]

    def _get_used_buffers(self):
        return self.buffers[:self.current + 1]


class SwapBufferManager:
    def __init__(self, num_elems, count, dtype):
        self.num_elems, self.count, self.dtype = num_elems, count, dtype
        self.all_buffers = [_pinned(num_elems, dtype) for _ in range(count)]
        self.free_buffer_index = list(range(count))
        self.used_buffer_index = {}
        self.gigabytes = (self.all_buffers[0].element_size() * num_elems * count) / (1024 ** 3)

    def allocate(self, num_elems, count, dtype):
        assert dtype == self.dtype and num_elems <= self.num_elems
        if count > len(self.free_buffer_index):
            return None
        used = self.free_buffer_index[-count:]
        self.free_buffer_index = self.free_buffer_index[:-count]
        out = []
        for i in used:
            t = self.all_buffers[i].narrow(0, 0, num_elems)
            out.append(t)
            self.used_buffer_index[t.data_ptr()] = i
        return out

    def allocate_all(self, num_elems, dtype):
        return self.allocate(num_elems, len(self.free_buffer_index), dtype)

    def free(self, buffers):
        for b in buffers:
            self.free_buffer_index.append(self.used_buffer_index.pop(b.data_ptr()))
