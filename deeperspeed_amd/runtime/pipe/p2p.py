"""Point-to-point activation/gradient transfer between adjacent pipeline stages.

Reference parity: deepspeed/runtime/pipe/p2p.py:13-96 (send/recv between stage ids through
the grid, optional fp32 upcast for bf16 -- DeeperSpeed p2p.py:31-61, barrier).  The
reference emulates p2p with `dist.broadcast` on two-rank groups, fully synchronous; here
transfers are true RCCL send/recv (`batch_isend_irecv`), which over xGMI is a single
direct link between the two GPUs.  `async_op=True` returns the work handles so the engine
can overlap a transfer with compute.
"""

from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

_grid = None

# Optional log of every p2p transfer this rank issues, in issue order:
# (kind "send" | "recv", peer global rank, shape, dtype).  RCCL serialises the send/recv of a
# rank pair on one communicator stream, so the two ranks of every pair must issue complementary
# sequences (rank a's k-th op towards b is the mirror of b's k-th op towards a) or the pair can
# deadlock; gloo queues both directions independently and cannot show such a bug.  The log lets
# a test (tests/test_pipe_p2p_order.py) or a debugging run check the invariant on any backend.
_op_log = None


def record_ops(enable: bool = True):
    """Start (clearing) or stop the transfer log."""
    global _op_log
    _op_log = [] if enable else None


def op_log():
    return list(_op_log or [])


def _log(kind, peer, t):
    if _op_log is not None:
        _op_log.append((kind, int(peer), tuple(t.shape), str(t.dtype)))


def check_pair_order(logs):
    """logs: {global rank: op_log()}.  Returns a list of human-readable violations (empty if every
    pair issues complementary send/recv sequences)."""
    errs = []
    flip = {"send": "recv", "recv": "send"}
    for a, la in logs.items():
        for b, lb in logs.items():
            if b <= a:
                continue
            ab = [(k, sh, dt) for k, peer, sh, dt in la if peer == b]
            ba = [(flip[k], sh, dt) for k, peer, sh, dt in lb if peer == a]
            if ab == ba:
                continue
            n = next((i for i, (x, y) in enumerate(zip(ab, ba)) if x != y), min(len(ab), len(ba)))
            errs.append(f"ranks {a}<->{b}: op {n} differs: rank {a} issues "
                        f"{ab[n] if n < len(ab) else None}, rank {b} mirrors {ba[n] if n < len(ba) else None} "
                        f"({len(ab)} vs {len(ba)} ops)")
    return errs


def init_process_groups(grid):
    global _grid
    _grid = grid
    assert _grid.pipe_parallel_size > 1, "There is no pipeline parallelism"


def _is_valid_send_recv(src_stage, dest_stage):
    first_stage, last_stage = 0, _grid.pipe_parallel_size - 1
    assert abs(src_stage - dest_stage) == 1 or (src_stage == first_stage and dest_stage == last_stage) or \
        (src_stage == last_stage and dest_stage == first_stage), \
        "Functionality currently limited to send and receive between adjacent ranks only"


def _peer(stage):
    return _grid.stage_to_global(stage_id=stage)


def _host_staged(t):
    """gloo has no device-memory send/recv: stage through host memory (CPU tests and
    several-ranks-on-one-GPU rehearsals only; RCCL moves device memory directly)."""
    return t.is_cuda and dist.get_backend() == "gloo"


def send(tensor, dest_stage, async_op=False, fp32_comm=False):
    src_stage = _grid.get_stage_id()
    _is_valid_send_recv(src_stage, dest_stage)
    t = tensor.float() if (fp32_comm and tensor.dtype == torch.bfloat16) else tensor
    _log("send", _peer(dest_stage), t)
    if _host_staged(t):
        dist.send(t.detach().cpu().contiguous(), _peer(dest_stage))
        return None
    work = dist.isend(t.contiguous(), _peer(dest_stage))
    if async_op:
        return work
    work.wait()
    return None


def recv(tensor, src_stage, async_op=False, fp32_comm=False):
    dest_stage = _grid.get_stage_id()
    _is_valid_send_recv(src_stage, dest_stage)
    _log("recv", _peer(src_stage), tensor.float() if (fp32_comm and tensor.dtype == torch.bfloat16) else tensor)
    if _host_staged(tensor):
        buf = torch.empty(tensor.shape, dtype=torch.float32 if (fp32_comm and tensor.dtype == torch.bfloat16)
                          else tensor.dtype)
        dist.recv(buf, _peer(src_stage))
        tensor.copy_(buf)
        return None
    if fp32_comm and tensor.dtype == torch.bfloat16:
        buf = torch.empty(tensor.shape, dtype=torch.float32, device=tensor.device)
        work = dist.irecv(buf, _peer(src_stage))
        work.wait()
        tensor.copy_(buf)
        return None
    work = dist.irecv(tensor, _peer(src_stage))
    if async_op:
        return work
    work.wait()
    return None


class P2PHandle:
    """Outstanding batched transfer.  `wait()` makes the caller's stream wait for it (RCCL: a
    stream dependency, no host block) and finishes an fp32-staged receive by casting into the
    target buffers.  The handle keeps every tensor of the transfer alive until then."""

    __slots__ = ("works", "keep", "staged", "done")

    def __init__(self, works, keep=(), staged=()):
        self.works = list(works or [])
        self.keep = list(keep)
        self.staged = list(staged)
        self.done = False

    def wait(self):
        if self.done:
            return
        for w in self.works:
            w.wait()
        with torch.no_grad():  # targets may already be leaves that require grad
            for t, b in self.staged:
                t.copy_(b)
        self.works, self.keep, self.staged = [], [], []
        self.done = True


_DONE = P2PHandle(())
_DONE.done = True


def send_many(tensors: List[torch.Tensor], dest_stage, fp32_comm=False, async_op=False):
    """Send a list of tensors in one batched call (one RCCL group launch).  async_op=True
    returns a P2PHandle to wait on later (the engine overlaps the transfer with compute)."""
    if tensors and _host_staged(tensors[0]):
        for t in tensors:
            send(t, dest_stage, fp32_comm=fp32_comm)
        return _DONE if async_op else None
    ops = []
    peer = _peer(dest_stage)
    keep = []
    for t in tensors:
        x = t.float() if (fp32_comm and t.dtype == torch.bfloat16) else t.contiguous()
        _log("send", peer, x)
        keep.append(x)
        ops.append(dist.P2POp(dist.isend, x, peer))
    h = P2PHandle(dist.batch_isend_irecv(ops) if ops else [], keep=keep)
    if async_op:
        return h
    h.wait()
    return None


def recv_many(tensors: List[torch.Tensor], src_stage, fp32_comm=False, async_op=False):
    """Receive into `tensors` (one batched call).  With fp32_comm the bf16 targets receive
    through fp32 staging buffers, cast when the handle is waited: non-blocking too."""
    if tensors and _host_staged(tensors[0]):
        for t in tensors:
            recv(t, src_stage, fp32_comm=fp32_comm)
        return _DONE if async_op else None
    ops, staged = [], []
    peer = _peer(src_stage)
    for t in tensors:
        if fp32_comm and t.dtype == torch.bfloat16:
            b = torch.empty(t.shape, dtype=torch.float32, device=t.device)
            staged.append((t, b))
            _log("recv", peer, b)
            ops.append(dist.P2POp(dist.irecv, b, peer))
        else:
            _log("recv", peer, t)
            ops.append(dist.P2POp(dist.irecv, t, peer))
    h = P2PHandle(dist.batch_isend_irecv(ops) if ops else [], keep=tensors, staged=staged)
    if async_op:
        return h
    h.wait()
    return None


def barrier(stage_id):
    global _grid
    group_id = _grid.stage_to_global(stage_id=stage_id)
    if dist.get_rank() >= 0:
        print("Barrier Group ID", group_id)
    dist.barrier()
