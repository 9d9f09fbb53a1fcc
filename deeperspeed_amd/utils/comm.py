"""Framework collectives: one place that issues RCCL calls for ZeRO/engine traffic, with
optional tracing and race/consistency checking.

* `DSA_ROCTX=1`    - every collective and engine phase is wrapped in a roctx range
                     (torch.cuda.nvtx maps to roctx on ROCm), so rocprofv3 `--marker-trace`
                     timelines show kernel / RCCL overlap per bucket.
* `DSA_DEBUG_COLLECTIVES=1` - every collective is appended to a per-rank log
                     (sequence id, op, numel, dtype); `verify_collective_order()` (called by the
                     engine at every optimizer step in this mode) checks that all ranks issued the
                     identical sequence - the class of bug that otherwise deadlocks or silently
                     mixes buckets - and gathered ZeRO buckets are checksummed across ranks
                     (`check_replicated`).
Reference counterpart: none (the reference relies on torch.cuda.synchronize() and ad-hoc
asserts, stage2.py:627-630, stage3.py:1896-1899).
"""

from __future__ import annotations

import contextlib
import hashlib
import os
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

TRACE = os.environ.get("DSA_ROCTX", "0") == "1"
DEBUG = os.environ.get("DSA_DEBUG_COLLECTIVES", "0") == "1"

_log: List[Tuple[int, str, int, str]] = []
_seq = 0
# always on (an int and a tuple per call): how many collectives this rank has issued and the last
# one, which a watchdog prints when a rank stalls -- equal counts on every rank point at a slow or
# hung collective, different counts at a rank that took another path (order divergence)
_issued = 0
_last: Tuple[str, int, str] = ("none", 0, "")
# bytes per collective kind (all_gather: the gathered output, reduce_scatter / all_reduce: the
# input), always counted: the emulated-world bench turns them into the xGMI rate a real job needs
_bytes: Dict[str, int] = {}
# opt-in full (tag, numel, dtype) trace, independent of DEBUG's per-step log (tests compare the
# sequence an emulated rank issues with a real world-N rank's)
_trace: Optional[List[Tuple[str, int, str]]] = None

# Emulated world (bench.py --emulate-world N): one process runs rank 0 of an N-rank data-parallel
# job -- the ZeRO optimizers size shards, buckets and units for N ranks (`world_size` / `rank`
# below) -- and every framework collective is replaced by a local stand-in that writes the bytes
# the real collective would: all-gather = N copies of the local chunk, reduce-scatter = the sum of
# the N slices of the input (the local HBM traffic of RCCL's reduce kernel), all-reduce = nothing.
# Values are meaningless (the loss too); memory, kernels and the issued collective sequence are the
# real rank's.  Reference counterpart: none.
_emulated = 0


class _Done:
    """Work handle of a stand-in collective: already complete on the issuing stream."""

    def wait(self, timeout=None):
        return True

    def is_completed(self):
        return True


def set_emulated_world(n: int):
    global _emulated
    _emulated = int(n) if n and int(n) > 1 else 0


def emulated_world() -> int:
    return _emulated


def world_size(group=None) -> int:
    """Data-parallel world size the ZeRO layout is built for (the emulated N when set)."""
    if _emulated:
        return _emulated
    return dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1


def rank(group=None) -> int:
    if _emulated:
        return 0
    return dist.get_rank(group) if (dist.is_available() and dist.is_initialized()) else 0


def bytes_by_kind() -> Dict[str, int]:
    return dict(_bytes)


def reset_bytes():
    _bytes.clear()


def start_trace():
    global _trace
    _trace = []


def stop_trace() -> List[Tuple[str, int, str]]:
    global _trace
    out, _trace = _trace or [], None
    return out


def set_debug(enabled: bool):
    global DEBUG
    DEBUG = bool(enabled)


@contextlib.contextmanager
def trace_range(name: str):
    if TRACE and torch.cuda.is_available():
        torch.cuda.nvtx.range_push(name)
        try:
            yield
        finally:
            torch.cuda.nvtx.range_pop()
    else:
        yield


def _record(op: str, t: torch.Tensor, kind: str = "other"):
    global _seq, _issued, _last
    _issued += 1
    _last = (op, int(t.numel()), str(t.dtype))
    _bytes[kind] = _bytes.get(kind, 0) + t.numel() * t.element_size()
    if _trace is not None:
        _trace.append(_last)
    if DEBUG:
        _log.append((_seq, op, int(t.numel()), str(t.dtype)))
        _seq += 1


def all_gather_into_tensor(out, inp, group=None, async_op=False, tag="all_gather"):
    _record(tag, out, "all_gather")
    with trace_range(f"rccl.{tag}[{out.numel()}]"):
        if _emulated:
            out.view(_emulated, -1).copy_(inp.reshape(1, -1).expand(_emulated, -1))
            return _Done() if async_op else None
        return dist.all_gather_into_tensor(out, inp, group=group, async_op=async_op)


def reduce_scatter_tensor(out, inp, group=None, async_op=False, tag="reduce_scatter"):
    _record(tag, inp, "reduce_scatter")
    with trace_range(f"rccl.{tag}[{inp.numel()}]"):
        if _emulated:
            torch.sum(inp.view(_emulated, -1), 0, out=out.view(-1))
            return _Done() if async_op else None
        return dist.reduce_scatter_tensor(out, inp, group=group, async_op=async_op)


def all_reduce(t, op=dist.ReduceOp.SUM, group=None, async_op=False, tag="all_reduce"):
    _record(tag, t, "all_reduce")
    with trace_range(f"rccl.{tag}[{t.numel()}]"):
        if _emulated:
            return _Done() if async_op else None
        return dist.all_reduce(t, op=op, group=group, async_op=async_op)


def progress() -> str:
    """One line: collectives issued by this rank so far and the last one."""
    return f"collectives issued={_issued} last={_last[0]}[{_last[1]} {_last[2]}]"


def collective_log():
    return list(_log)


def reset_log():
    global _seq
    _log.clear()
    _seq = 0


def _digest(entries) -> int:
    h = hashlib.sha1(repr(entries).encode()).digest()
    return int.from_bytes(h[:7], "little")  # fits an int64 exactly


def verify_collective_order(group=None, device=None):
    """All ranks must have issued the same collectives (op, size, dtype) in the same order.
    Raises RuntimeError naming the first divergent entry; clears the log when consistent."""
    if not DEBUG or not (dist.is_available() and dist.is_initialized()):
        return True
    dev = device or (torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available()
                     else torch.device("cpu"))
    mine = _digest(_log)
    t = torch.tensor([mine, -mine, len(_log)], dtype=torch.int64, device=dev)
    lo = t.clone()
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    consistent = int(t[0]) == mine == -int(t[1]) and int(t[2]) == int(lo[2])
    if not consistent:
        logs = [None] * dist.get_world_size(group)
        dist.all_gather_object(logs, _log, group=group)
        first = None
        for i in range(max(len(x) for x in logs)):
            row = [x[i] if i < len(x) else None for x in logs]
            if any(r != row[0] for r in row):
                first = (i, row)
                break
        raise RuntimeError(f"collective order diverged across ranks at entry {first}")
    reset_log()
    return True


def check_replicated(t: torch.Tensor, group=None, name="tensor"):
    """Debug check that a gathered (supposedly identical) tensor matches on all ranks."""
    if not DEBUG or not (dist.is_available() and dist.is_initialized()):
        return True
    s = t.detach().float().sum().reshape(1)
    hi, lo = s.clone(), s.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    if not torch.equal(hi, lo):
        raise RuntimeError(f"{name}: replicated tensor differs across ranks (checksum {lo.item()} .. {hi.item()})")
    return True
