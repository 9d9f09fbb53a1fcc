"""Pipelined optimizer-state NVMe swapper at the reference's import path
(deepspeed/runtime/swap_tensor/pipelined_optimizer_swapper.py); implementation in optimizer_utils.py."""

from .optimizer_utils import PipelinedOptimizerSwapper  # noqa: F401
