"""`flops_profiler` key constants at the reference's import path (deepspeed/profiling/constants.py)."""

from ..runtime import key_schema as _ks

globals().update(_ks.export(_ks.FLOPS_PROFILER))
