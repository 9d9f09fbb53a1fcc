"""Multi-process test harness (reference parity: tests/unit/common.py:16-104).

`@distributed_test(world_size=N)` runs the decorated test body in N spawned processes with
RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set (127.0.0.1) and torch.distributed initialised on
`gloo` (CPU) -- the same engine code paths that run on RCCL on the MI355X.  A worker that
fails or hangs fails the test; stragglers are killed after a timeout.
"""

import datetime
import functools
import os
import socket
import sys
import time
import traceback

import pytest
import torch
import torch.multiprocessing as mp

DEFAULT_TIMEOUT = int(os.environ.get("DSA_TEST_TIMEOUT", "240"))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world_size, port, fn, args, kwargs, errq, backend="gloo"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"] = str(rank)
    os.environ["LOCAL_RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(world_size)
    os.environ.setdefault("OMP_NUM_THREADS", "2")
    torch.set_num_threads(2)
    try:
        import torch.distributed as dist
        if backend == "nccl":  # RCCL: one rank per visible GPU
            torch.cuda.set_device(rank % torch.cuda.device_count())
        # the parent owns the rendezvous store (bound to a kernel-chosen port before any worker
        # starts), so no two runs can race for a port picked by probing
        store = dist.TCPStore("127.0.0.1", port, is_master=False, timeout=datetime.timedelta(seconds=120))
        dist.init_process_group(backend, store=store, rank=rank, world_size=world_size)
        fn(*args, **kwargs)
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:
        errq.put((rank, traceback.format_exc()))
        sys.exit(1)


def run_distributed(fn, world_size, *args, timeout=DEFAULT_TIMEOUT, backend="gloo", **kwargs):
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    import torch.distributed as dist
    server = dist.TCPStore("127.0.0.1", 0, is_master=True, wait_for_workers=False)
    port = server.port
    procs = [ctx.Process(target=_worker, args=(r, world_size, port, fn, args, kwargs, errq, backend))
             for r in range(world_size)]
    for p in procs:
        p.start()
    deadline = time.time() + timeout
    failed = None
    while any(p.is_alive() for p in procs):
        if not errq.empty():
            failed = errq.get()
            break
        if time.time() > deadline:
            failed = (-1, f"timeout after {timeout}s")
            break
        time.sleep(0.05)
    if failed is not None:
        for p in procs:
            if p.is_alive():
                p.terminate()
    for p in procs:
        p.join(10)
    if failed is None and not errq.empty():
        failed = errq.get()
    if failed is None:
        bad = [p.exitcode for p in procs if p.exitcode != 0]
        if bad:
            failed = (-1, f"worker exit codes {bad}")
    del server
    if failed is not None:
        pytest.fail(f"rank {failed[0]} failed:\n{failed[1]}")


def distributed_test(world_size=2, timeout=DEFAULT_TIMEOUT):
    """Decorator: the test body runs on every rank. Body must be a module-level function."""
    sizes = world_size if isinstance(world_size, (list, tuple)) else [world_size]

    def deco(fn):
        @functools.wraps(fn)
        def wrapper(*args, **kwargs):
            for ws in sizes:
                run_distributed(_Call(fn.__module__, fn.__name__ + "__body"), ws, *args, timeout=timeout, **kwargs)
        # the undecorated body is reachable by name from the spawned workers
        setattr(sys.modules[fn.__module__], fn.__name__ + "__body", fn)
        return wrapper

    return deco


class _Call:
    """Picklable reference to a module-level function (resolved in the worker)."""

    def __init__(self, module, name):
        self.module = module
        self.name = name

    def __call__(self, *args, **kwargs):
        import importlib
        tests_dir = os.path.dirname(os.path.abspath(__file__))
        root = os.path.dirname(tests_dir)
        for p in (root, tests_dir):
            if p not in sys.path:
                sys.path.insert(0, p)
        mod = importlib.import_module(self.module)
        return getattr(mod, self.name)(*args, **kwargs)


def ds_env_single():
    """Env for single-process engine tests (no spawn)."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(_free_port()))
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("LOCAL_RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
