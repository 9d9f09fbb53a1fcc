"""Async NVMe I/O (reference: deepspeed/ops/aio, csrc/aio) -- native engine in `_cpu_ops`."""

from ..builder import AsyncIOBuilder  # noqa: F401
