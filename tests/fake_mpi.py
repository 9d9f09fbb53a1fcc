"""In-process stand-in for an mpi4py communicator (mpi4py is not installed in this image):
`world(n)` returns n communicators meant to be driven from n threads.  Supports what
runtime/comm/mpi.py uses -- Get_rank, Get_size, Ialltoall, Iallgather -- on numpy arrays or
torch tensors (host or device); requests complete at Wait() in call order on every rank."""

import threading

import numpy as np
import torch


def _np(buf):
    if isinstance(buf, torch.Tensor):
        return buf.detach().cpu().numpy().reshape(-1)
    return np.asarray(buf).reshape(-1)


def _write(buf, arr):
    if isinstance(buf, torch.Tensor):
        buf.view(-1).copy_(torch.from_numpy(arr.copy()).to(buf.device))
    else:
        buf.reshape(-1)[:] = arr


class _Shared:
    def __init__(self, n):
        self.n = n
        self.barrier = threading.Barrier(n)
        self.slots = {}
        self.lock = threading.Lock()


class _Request:
    def __init__(self, comm, seq, kind, send, recv):
        self.comm, self.seq, self.kind, self.send, self.recv = comm, seq, kind, send, recv

    def Wait(self):
        sh, r = self.comm.shared, self.comm.rank
        with sh.lock:
            sh.slots.setdefault(self.seq, [None] * sh.n)[r] = _np(self.send).copy()
        sh.barrier.wait()
        parts = sh.slots[self.seq]
        if self.kind == "alltoall":
            chunk = parts[0].size // sh.n
            out = np.concatenate([p[r * chunk:(r + 1) * chunk] for p in parts])
        else:
            out = np.concatenate(parts)
        _write(self.recv, out)
        sh.barrier.wait()
        if r == 0:
            with sh.lock:
                del sh.slots[self.seq]


class FakeComm:
    def __init__(self, shared, rank):
        self.shared, self.rank, self.seq = shared, rank, 0
        self.calls = []

    def Get_rank(self):
        return self.rank

    def Get_size(self):
        return self.shared.n

    def _req(self, kind, send, recv):
        self.seq += 1
        self.calls.append((kind, type(send).__name__))
        return _Request(self, self.seq, kind, send, recv)

    def Ialltoall(self, send, recv):
        return self._req("alltoall", send, recv)

    def Iallgather(self, send, recv):
        return self._req("allgather", send, recv)


def world(n):
    sh = _Shared(n)
    return [FakeComm(sh, r) for r in range(n)]


def run_threads(n, fn):
    """fn(rank, comm) on n threads; re-raises the first exception."""
    comms, out, errs = world(n), [None] * n, []

    def body(r):
        try:
            out[r] = fn(r, comms[r])
        except BaseException as e:  # noqa: BLE001 - surfaced to the caller
            errs.append(e)
            comms[r].shared.barrier.abort()

    ts = [threading.Thread(target=body, args=(r,)) for r in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise errs[0]
    return out, comms
