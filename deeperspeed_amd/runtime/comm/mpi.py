"""MPI transport for the 1-bit compressed all-reduce (reference runtime/comm/mpi.py:170-290).

The RCCL backend (`comm/nccl.py`) is the MI355X path; this one serves clusters that launch
with MPI.  The compression math is shared with the RCCL backend (HIP kernels in onebit.hip).

Two transports, as in the reference:

* ``cuda_aware=True`` hands device tensors straight to MPI (a GPU-aware MPI build reads HIP
  memory through ``__cuda_array_interface__``): the sign exchange and the scale gather of each
  phase are posted together as non-blocking collectives and waited as one set, after the
  producing stream has finished.
* ``cuda_aware=False`` stages through reusable pinned host buffers: one asynchronous D2H per
  buffer on the current stream, a single stream sync, the MPI collectives on host memory, and
  asynchronous H2D copies back.  (The reference re-allocates host copies with ``cupy.asnumpy``
  every call.)

``comm`` may be injected (any object with Get_rank / Get_size / Ialltoall / Iallgather whose
requests have ``Wait``): the CPU tests drive the backend with an in-process communicator,
since mpi4py is not installed in this image."""

import torch

from ...ops import native


class MpiBackend:
    def __init__(self, cuda_aware=False, comm=None):
        if comm is None:
            try:
                from mpi4py import MPI
            except ImportError as e:  # pragma: no cover - depends on the environment
                raise ImportError("MpiBackend needs mpi4py; use comm_backend_name='nccl' (RCCL)") from e
            comm = MPI.COMM_WORLD
        self.comm = comm
        self.rank = comm.Get_rank()
        self.size = comm.Get_size()
        self.cuda_aware = bool(cuda_aware)
        self._host = {}

    # ------------------------------------------------------------------ transport
    def _staging(self, name, t):
        """Reusable host buffer for device tensor `t` (pinned when `t` is on the GPU)."""
        key = (name, t.dtype, t.numel())
        buf = self._host.get(key)
        if buf is None:
            buf = torch.empty(t.numel(), dtype=t.dtype, pin_memory=t.is_cuda)
            self._host[key] = buf
        return buf

    def _collectives(self, ops):
        """Run [(kind, send, recv)] (kind in {'alltoall', 'allgather'}) as one set of
        non-blocking MPI collectives; `recv` tensors hold the results afterwards."""
        on_gpu = any(s.is_cuda for _, s, _ in ops)
        if self.cuda_aware or not on_gpu:
            if on_gpu:
                torch.cuda.current_stream().synchronize()  # MPI reads what the kernels wrote
            bufs = [(k, s if on_gpu else s.numpy(), r if on_gpu else r.numpy()) for k, s, r in ops]
            reqs = [self._post(k, s, r) for k, s, r in bufs]
            for q in reqs:
                q.Wait()
            return
        staged = []
        for i, (k, s, r) in enumerate(ops):
            hs, hr = self._staging(f"s{i}", s), self._staging(f"r{i}", r)
            hs.copy_(s.reshape(-1), non_blocking=True)
            staged.append((k, hs, hr, r))
        torch.cuda.current_stream().synchronize()
        reqs = [self._post(k, hs.numpy(), hr.numpy()) for k, hs, hr, _ in staged]
        for q in reqs:
            q.Wait()
        for _, _, hr, r in staged:
            r.view(-1).copy_(hr, non_blocking=True)

    def _post(self, kind, send, recv):
        if kind == "alltoall":
            return self.comm.Ialltoall(send, recv)
        return self.comm.Iallgather(send, recv)

    # ------------------------------------------------------------------ 1-bit all-reduce
    def compressed_allreduce(self, buffer_m, worker_error, server_error, local_rank=None):
        original_shape, original_size = buffer_m.size(), buffer_m.numel()
        n = worker_error.numel()
        flat = buffer_m.reshape(-1).float()
        if original_size != n:
            flat = torch.cat([flat, torch.zeros(n - original_size, device=flat.device)])
        assert n % (8 * self.size) == 0 and server_error.numel() * self.size == n, "bad 1-bit buffer sizes"
        dev = flat.device
        # phase 1: every rank compresses its whole buffer; chunk j of the signs goes to server j
        packed, wscale = native.onebit_worker_compress(flat.contiguous(), worker_error)
        recv_signs = torch.empty_like(packed)
        scales = torch.empty(self.size, dtype=torch.float32, device=dev)
        self._collectives([("alltoall", packed, recv_signs), ("allgather", wscale.reshape(1), scales)])
        # server: average my chunk over the ranks, add the server error, re-compress
        spacked, sscale = native.onebit_server_compress(recv_signs, scales, server_error)
        # phase 2: every server chunk to every rank
        all_signs = torch.empty(spacked.numel() * self.size, dtype=torch.uint8, device=dev)
        all_scales = torch.empty(self.size, dtype=torch.float32, device=dev)
        self._collectives([("allgather", spacked, all_signs), ("allgather", sscale.reshape(1), all_scales)])
        out = torch.empty(n, dtype=torch.float32, device=dev)
        native.onebit_unpack(all_signs, all_scales, out)
        buffer_m.data.copy_(out[:original_size].view(original_shape).to(buffer_m.dtype))
        return buffer_m
