"""Compressed (1-bit, error-compensated) all-reduce over RCCL.

Reference parity: deepspeed/runtime/comm/nccl.py:13-186 (`NcclBackend.compressed_allreduce`).
Two phases, as in the reference, but with tensor-native collectives and HIP kernels instead
of CuPy lists:
  1. every rank compresses its (momentum + worker error) to signs + one scale, and an
     `all_to_all_single` delivers chunk p of every rank's signs to rank p ("server" p);
     the worker scales are `all_gather_into_tensor`-ed;
  2. each server averages its P chunks, adds its server error, re-compresses, and the
     compressed server chunks + scales are all-gathered and unpacked into the result.
Per step each rank moves n/8 bytes in phase 1 and n/8 in phase 2 (vs 2*2n bytes for a bf16
ring all-reduce): the traffic reduction 1-bit Adam targets.  Sizes must be padded to a
multiple of 8*world (the optimizers do that).
"""

import torch
import torch.distributed as dist

from ...ops import native


class NcclBackend:
    def __init__(self, mpu=None):
        if mpu is None:
            self.world_group = None
        else:
            self.world_group = mpu.get_data_parallel_group()
        self.rank = dist.get_rank(group=self.world_group)
        self.size = dist.get_world_size(group=self.world_group)

    def compressed_allreduce(self, buffer_m: torch.Tensor, worker_error: torch.Tensor, server_error: torch.Tensor,
                             local_rank=None) -> torch.Tensor:
        original_shape = buffer_m.size()
        original_size = buffer_m.numel()
        n = worker_error.numel()
        flat = buffer_m.reshape(-1).float()
        if original_size != n:
            flat = torch.cat([flat, torch.zeros(n - original_size, device=flat.device)])
        assert n % (8 * self.size) == 0 and server_error.numel() * self.size == n, "bad 1-bit buffer sizes"
        # phase 1: worker compression, signs all-to-all, scales all-gather
        packed, wscale = native.onebit_worker_compress(flat.contiguous(), worker_error)
        recv_signs = torch.empty_like(packed)
        dist.all_to_all_single(recv_signs, packed, group=self.world_group)
        scales = torch.empty(self.size, dtype=torch.float32, device=flat.device)
        dist.all_gather_into_tensor(scales, wscale, group=self.world_group)
        # server: average my chunk, compress again
        spacked, sscale = native.onebit_server_compress(recv_signs, scales, server_error)
        # phase 2: gather every server chunk
        all_signs = torch.empty(spacked.numel() * self.size, dtype=torch.uint8, device=flat.device)
        dist.all_gather_into_tensor(all_signs, spacked, group=self.world_group)
        all_scales = torch.empty(self.size, dtype=torch.float32, device=flat.device)
        dist.all_gather_into_tensor(all_scales, sscale, group=self.world_group)
        out = torch.empty(n, dtype=torch.float32, device=flat.device)
        native.onebit_unpack(all_signs, all_scales, out)
        res = out[:original_size].view(original_shape)
        buffer_m.data.copy_(res.to(buffer_m.dtype))
        return buffer_m
