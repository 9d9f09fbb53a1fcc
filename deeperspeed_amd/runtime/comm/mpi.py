"""MPI transport for the 1-bit compressed all-reduce (reference runtime/comm/mpi.py).

Requires mpi4py (not part of this image); the RCCL backend (`comm/nccl.py`) is the MI355X
path.  The compression math is shared with the RCCL backend."""

import torch

from ...ops import native


class MpiBackend:
    def __init__(self, cuda_aware=False):
        try:
            from mpi4py import MPI
        except ImportError as e:  # pragma: no cover - depends on the environment
            raise ImportError("MpiBackend needs mpi4py; use comm_backend_name='nccl' (RCCL)") from e
        self.comm = MPI.COMM_WORLD
        self.rank = self.comm.Get_rank()
        self.size = self.comm.Get_size()
        self.cuda_aware = cuda_aware

    def compressed_allreduce(self, buffer_m, worker_error, server_error, local_rank=None):  # pragma: no cover
        import numpy as np
        n = worker_error.numel()
        flat = buffer_m.reshape(-1).float()
        if flat.numel() != n:
            flat = torch.cat([flat, torch.zeros(n - flat.numel(), device=flat.device)])
        packed, wscale = native.onebit_worker_compress(flat.contiguous(), worker_error)
        send = packed.cpu().numpy().reshape(self.size, -1)
        recv = np.empty_like(send)
        self.comm.Alltoall(send, recv)
        scales = np.empty(self.size, dtype=np.float32)
        self.comm.Allgather(wscale.cpu().numpy(), scales)
        spacked, sscale = native.onebit_server_compress(torch.from_numpy(recv.reshape(-1)).to(flat.device),
                                                        torch.from_numpy(scales).to(flat.device), server_error)
        all_signs = np.empty(spacked.numel() * self.size, dtype=np.uint8)
        self.comm.Allgather(spacked.cpu().numpy(), all_signs)
        all_scales = np.empty(self.size, dtype=np.float32)
        self.comm.Allgather(sscale.cpu().numpy(), all_scales)
        out = torch.empty(n, dtype=torch.float32, device=flat.device)
        native.onebit_unpack(torch.from_numpy(all_signs).to(flat.device), torch.from_numpy(all_scales).to(flat.device),
                             out)
        buffer_m.data.copy_(out[:buffer_m.numel()].view_as(buffer_m).to(buffer_m.dtype))
        return buffer_m
