"""Native async I/O engine (ops/csrc/cpu/aio.cpp): io_uring rings per worker with queue
depth, single vs block submit and overlapped vs lock-step completion, plus the positional
I/O fallback.  Reference behaviour: csrc/aio/common/deepspeed_aio_common.cpp:69-160,265
(tests/perf/aio_bench_perf_sweep.py sweeps the same knobs)."""

import itertools
import os
import subprocess
import sys

import pytest
import torch


def _aio():
    from deeperspeed_amd.ops.aio import AsyncIOBuilder
    return AsyncIOBuilder().load()


@pytest.mark.parametrize("single_submit,overlap,threads,qd", list(itertools.product(
    [False, True], [False, True], [1, 3], [1, 8])))
def test_aio_modes_roundtrip(tmp_path, single_submit, overlap, threads, qd):
    aio = _aio()
    h = aio.aio_handle(block_size=1 << 16, queue_depth=qd, single_submit=single_submit,
                       overlap_events=overlap, thread_count=threads)
    assert h.get_queue_depth() == qd and h.get_single_submit() == single_submit
    # page-aligned pinned-like host buffer (O_DIRECT path) and an odd-sized one (buffered)
    for n in (1 << 20, 300001, -(1 << 20)):
        if n < 0:  # explicitly 4 KiB-aligned buffer: the O_DIRECT path
            n = -n
            base = torch.empty(n + 1024)
            off = ((-base.data_ptr()) % 4096) // 4
            x = base[off: off + n]
            x.copy_(torch.randn(n))
            assert x.data_ptr() % 4096 == 0
        else:
            x = torch.randn(n)
        f = str(tmp_path / f"x{n}.swp")
        assert h.sync_pwrite(x, f) == 1
        assert os.path.getsize(f) == x.nbytes
        y = torch.empty_like(x)
        assert h.sync_pread(y, f) == 1
        assert torch.equal(x, y)


def test_aio_many_async_requests(tmp_path):
    aio = _aio()
    h = aio.aio_handle(block_size=1 << 15, queue_depth=16, single_submit=False, overlap_events=True,
                       thread_count=2)
    xs = [torch.randn(100000 + 4096 * i) for i in range(6)]
    for i, x in enumerate(xs):
        h.async_pwrite(x, str(tmp_path / f"{i}.swp"))
    assert h.wait() == len(xs)
    ys = [torch.empty_like(x) for x in xs]
    for i, y in enumerate(ys):
        h.async_pread(y, str(tmp_path / f"{i}.swp"))
    assert h.wait() == len(xs)
    for x, y in zip(xs, ys):
        assert torch.equal(x, y)


def test_aio_validate_and_errors(tmp_path):
    aio = _aio()
    h = aio.aio_handle(block_size=1 << 16, queue_depth=4, single_submit=False, overlap_events=True, thread_count=1)
    x = torch.randn(50000)
    f = str(tmp_path / "v.swp")
    assert h.write(x, f, True) == 1  # validated write
    y = torch.empty_like(x)
    assert h.read(y, f, True) == 1 and torch.equal(x, y)
    big = torch.empty(100000)
    with pytest.raises(RuntimeError):  # reading past the end of the file is refused up front
        h.sync_pread(big, f)
    with pytest.raises(RuntimeError):
        h.sync_pread(big, str(tmp_path / "missing.swp"))


def test_aio_engine_reported_and_psync_fallback(tmp_path):
    aio = _aio()
    assert aio.aio_engine() in ("io_uring", "psync")
    h = aio.aio_handle(block_size=1 << 16, queue_depth=4, single_submit=False, overlap_events=True, thread_count=1)
    assert h.get_engine() == aio.aio_engine()
    # forced fallback in a fresh process (the engine choice is made once per process)
    code = ("import torch, sys; sys.path.insert(0, %r)\n"
            "from deeperspeed_amd.ops.aio import AsyncIOBuilder\n"
            "a = AsyncIOBuilder().load(); assert a.aio_engine() == 'psync'\n"
            "h = a.aio_handle(65536, 4, False, True, 2); x = torch.randn(123457); f = %r\n"
            "assert h.sync_pwrite(x, f) == 1; y = torch.empty_like(x); assert h.sync_pread(y, f) == 1\n"
            "assert torch.equal(x, y); print('ok')\n") % (os.path.dirname(os.path.dirname(__file__)),
                                                           str(tmp_path / "p.swp"))
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, DSA_AIO_ENGINE="psync"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr


def test_aio_uring_failure_drains_and_falls_back(tmp_path, monkeypatch):
    """An io_uring_enter failure mid-transfer (injected: the 3rd enter of the worker returns
    EIO) fails that request, waits for every SQE already in flight against the buffer, then
    moves the worker to pread/pwrite: later requests still round-trip exactly."""
    aio = _aio()
    if aio.aio_engine() != "io_uring":
        pytest.skip("io_uring not available in this container")
    monkeypatch.setenv("DSA_AIO_INJECT_ENTER_FAIL", "3")
    h = aio.aio_handle(block_size=1 << 12, queue_depth=8, single_submit=True, overlap_events=True, thread_count=1)
    x = torch.randn(1 << 18)
    assert h.sync_pwrite(x, str(tmp_path / "a.swp")) != 1  # the injected failure is reported
    for i in range(3):
        y = torch.randn(300001)
        f = str(tmp_path / f"b{i}.swp")
        assert h.sync_pwrite(y, f) == 1
        z = torch.empty_like(y)
        assert h.sync_pread(z, f) == 1
        assert torch.equal(y, z)
