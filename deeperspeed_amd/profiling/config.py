"""`flops_profiler` section at the reference's import path (deepspeed/profiling/config.py)."""

from ..runtime.config import DeepSpeedFlopsProfilerConfig  # noqa: F401
